// scalar_ladder.cpp -- times the drop-in scalar CRC32C exactly as an
// unchanged caller links it: bmqp::Crc32c::calculate(const void*, unsigned)
// and calculate(const bdlbb::Blob&) from include/bmqp_crc32c.h, in
// libbmqcrc.so (built by blazingmq_amd/build.py into tools/bin/).
//
// The loop is the reference's (bmqp_crc32c.t.cpp:1116-1120): one buffer CRC'd
// k_NUM_ITERS = 100,000 times on one thread after one untimed call, over its
// size ladder (bmqp_crc32c.t.cpp:95-118), buffer filled from rand() like
// :1108.  Long sizes take fewer iterations (at least 20, about 0.2 s each)
// so the whole ladder runs in seconds; the count is printed.  The Blob form
// splits the same bytes into 4 KiB buffers (the SDK/broker blob buffer size,
// bmqt_sessionoptions.cpp:37) and chains them like bmqp_crc32c.cpp:47-67.
//
//   tools/bin/scalar_ladder [SIZE ...]  one JSON line per size (default: the ladder)
#include "bmqp_crc32c.h"

#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include <algorithm>
#include <vector>

using BloombergLP::bdlbb::Blob;
using BloombergLP::bdlbb::BlobBuffer;
using BloombergLP::bmqp::Crc32c;

static double now()
{
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

template <class F>
static double ns_per_call(F&& f, int* iters_out)
{
    unsigned c = f();
    int iters = 100000;
    const double t0 = now();
    for (int l = 0; l < 100; ++l) {
        c ^= f();
    }
    const double est = (now() - t0) / 100;
    if (est * iters > 0.2) {
        iters = std::max(20, (int)(0.2 / std::max(est, 1e-9)));
    }
    const double t1 = now();
    for (int l = 0; l < iters; ++l) {
        c ^= f();
    }
    const double dt = now() - t1;
    *iters_out = iters;
    volatile unsigned sink = c;
    (void)sink;
    return dt * 1e9 / iters;
}

int main(int argc, char** argv)
{
    const int ladder[] = {11,    16,    21,     59,     64,      69,      251,      256,
                          261,   1019,  1024,   1029,   4091,    4096,    4101,     16379,
                          16384, 16389, 65536,  262144, 1048576, 4194304, 16777216, 67108864};
    const int k_MAX = 67108864;
    std::vector<char> buffer(k_MAX);
    std::generate_n(buffer.begin(), k_MAX, rand);
    std::vector<int> sizes(ladder, ladder + sizeof ladder / sizeof ladder[0]);
    if (argc > 1) {
        sizes.clear();
        for (int i = 1; i < argc; ++i) {
            sizes.push_back(std::max(0, std::min(k_MAX, atoi(argv[i]))));
        }
    }
    for (int length : sizes) {
        int iters = 0, biters = 0;
        const double ns = ns_per_call([&] { return Crc32c::calculate(buffer.data(), length); },
                                      &iters);
        Blob blob;
        for (int off = 0; off < length; off += 4096) {
            blob.appendDataBuffer(BlobBuffer(buffer.data() + off, std::min(4096, length - off)));
        }
        const double bns = ns_per_call([&] { return Crc32c::calculate(blob); }, &biters);
        const unsigned a = Crc32c::calculate(buffer.data(), length), b = Crc32c::calculate(blob);
        printf("{\"size\": %d, \"calculate_ns\": %.1f, \"iters\": %d, \"blob_4KiB_ns\": %.1f, "
               "\"blob_iters\": %d, \"blob_buffers\": %d, \"blob_equal\": %s}\n",
               length, ns, iters, bns, biters, blob.numDataBuffers(), a == b ? "true" : "false");
        fflush(stdout);
        if (a != b) {
            return 1;
        }
    }
    return 0;
}
