// scalar_ab.cpp -- same-box A/B of the scalar CPU CRC32C methods in
// blazingmq_amd/csrc/crc32c_cpu.cpp (which it includes with BMQCRC_CPU_AB).
//
//   g++ -O2 -std=c++17 tools/scalar_ab.cpp -o /tmp/scalar_ab && /tmp/scalar_ab [check|time]
//
// check: every method equals the bitwise definition on random lengths,
//        seeds and misalignments (0..5000 bytes, plus the ladder sizes).
// time:  the reference's benchmark loop (bmqp_crc32c.t.cpp:1116-1120: one
//        buffer CRC'd 100,000 times on one thread) per method on the
//        reference's size ladder (bmqp_crc32c.t.cpp:95-118), one JSON line per
//        size with ns per call, beside bmqp_crc32c.h:109-132's published time.
//        `time MASK [SIZES...]`: methods by bit (0 product, 1 serial, 2 three-way,
//        3 fold, 4 slicing-by-8), other sizes instead of the ladder.
#define BMQCRC_CPU_AB 1
#include "../blazingmq_amd/csrc/crc32c_cpu.cpp"

#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include <vector>

using namespace bmqcrc;

static uint32_t bitwise(const uint8_t* p, size_t n, uint32_t crc)
{
    uint32_t c = ~crc;
    for (size_t i = 0; i < n; ++i) {
        c ^= p[i];
        for (int k = 0; k < 8; ++k) {
            c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
        }
    }
    return ~c;
}

static double now()
{
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

static const char* kName[] = {"product", "serial_crc32q", "three_way_clmul", "fold_vpclmul512",
                              "slicing_by_8"};

int main(int argc, char** argv)
{
    const bool check = argc < 2 || !strcmp(argv[1], "check");
    const int ladder[] = {11,   16,   21,    59,    64,    69,    251,    256,    261,
                          1019, 1024, 1029,  4091,  4096,  4101,  16379,  16384,  16389,
                          65536, 262144, 1048576, 4194304, 16777216, 67108864};
    const double published[] = {9,    9,    10,    13,    12,     13,     30,     30,
                                37,   155,  45,    50,    299,    176,    190,    864,
                                724,  754,  2858,  11925, 50937,  198662, 796534, 9976933};
    std::vector<uint8_t> buf((64u << 20) + 64);
    uint64_t s = 0xB1A2E5;
    for (auto& b : buf) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        b = (uint8_t)(s >> 33);
    }
    if (check) {
        int bad = 0, runs = 0;
        for (int it = 0; it < 20000; ++it) {
            s = s * 6364136223846793005ull + 1442695040888963407ull;
            const uint32_t len = it < 24 ? ladder[it] : (uint32_t)((s >> 20) % 5001);
            const uint32_t mis = (uint32_t)(s >> 50) % 64;
            const uint32_t seed = (uint32_t)(s >> 7);
            if (it < 24 && len > 70000) {
                continue;  // the bitwise definition is slow; ladder tops checked below
            }
            const uint32_t want = bitwise(buf.data() + mis, len, seed);
            for (int m = 0; m <= 4; ++m) {
                if (!cpu_has(m) || (m == 3 && len < 64)) {
                    continue;
                }
                ++runs;
                const uint32_t got = cpu_crc32c_method(m, buf.data() + mis, len, seed);
                if (got != want) {
                    if (++bad < 10) {
                        printf("MISMATCH method %s len %u mis %u: %08x != %08x\n", kName[m], len,
                               mis, got, want);
                    }
                }
            }
        }
        // the long ladder sizes: every method against slicing-by-8
        for (int len : {262144, 1048576, 4194304, 67108864}) {
            const uint32_t want = cpu_crc32c_method(4, buf.data() + 3, len, 77);
            for (int m = 0; m <= 3; ++m) {
                if (cpu_has(m) && cpu_crc32c_method(m, buf.data() + 3, len, 77) != want) {
                    printf("MISMATCH method %s len %d\n", kName[m], len);
                    ++bad;
                }
            }
        }
        // combine: crc(A||B) == combine(crc A, crc B, |B|)
        for (int it = 0; it < 2000; ++it) {
            s = s * 6364136223846793005ull + 1442695040888963407ull;
            const uint32_t la = (uint32_t)(s >> 20) % 3000, lb = (uint32_t)(s >> 40) % 3000;
            const uint32_t a = cpu_crc32c(buf.data(), la, 5), b = cpu_crc32c(buf.data() + la, lb, 0);
            if (cpu_combine(a, b, lb) != cpu_crc32c(buf.data(), la + lb, 5)) {
                printf("MISMATCH combine %u %u\n", la, lb);
                ++bad;
            }
        }
        printf("{\"check\": \"%s\", \"runs\": %d, \"bad\": %d, \"sse42\": %d, \"clmul\": %d, "
               "\"avx512_vpclmul\": %d}\n",
               bad ? "FAIL" : "PASS", runs, bad, (int)cpu_has(1), (int)cpu_has(2), (int)cpu_has(3));
        return bad ? 1 : 0;
    }
    const int methods = argc > 2 ? atoi(argv[2]) : 0x1f;
    const int nsizes = argc > 3 ? argc - 3 : 24;  // sizes after the mask replace the ladder
    for (int i = 0; i < nsizes; ++i) {
        const int len = argc > 3 ? atoi(argv[3 + i]) : ladder[i];
        const int iters = len >= (1 << 22) ? 200 : len >= 65536 ? 5000 : 100000;
        printf("{\"size\": %d, \"iters\": %d, \"published_ns\": %.0f", len, iters,
               argc > 3 ? 0.0 : published[i]);
        for (int m = 0; m <= 4; ++m) {
            if (!(methods >> m & 1) || !cpu_has(m) || (m == 3 && len < 64) ||
                (m == 4 && len > (1 << 20))) {
                continue;
            }
            uint32_t c = cpu_crc32c_method(m, buf.data(), len, 0);
            const double t0 = now();
            for (int l = 0; l < iters; ++l) {
                c ^= cpu_crc32c_method(m, buf.data(), len, 0);
            }
            const double ns = (now() - t0) * 1e9 / iters;
            printf(", \"%s_ns\": %.1f, \"%s_crc\": %u", kName[m], ns, kName[m], c);
        }
        printf("}\n");
        fflush(stdout);
    }
    return 0;
}
