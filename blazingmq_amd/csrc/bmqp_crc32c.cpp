// bmqp_crc32c.cpp -- bmqp::Crc32c over the bmqcrc C ABI.
// Reference: /root/reference/src/groups/bmq/bmqp/bmqp_crc32c.cpp:39-67.
#include "bmqp_crc32c.h"

#include <stdint.h>
#include <vector>

namespace BloombergLP {
namespace bmqp {
namespace {

// The GPU itself is unusable (no device, no device memory, a HIP error): the
// reference's interface has no error channel (bmqp_crc32c.h:240-243), so the
// batch overloads then finish on the host, bit-exact, with the library's own
// SSE4.2 CRC.  Argument errors (BMQCRC_EINVAL) are returned as they are.
// Every fallback is recorded (bmqcrc_host_fallbacks); a fault (EIO) is also
// reported on stderr once.
bool gpuFailure(int rc)
{
    if (rc == BMQCRC_ENODEV || rc == BMQCRC_ENOMEM || rc == BMQCRC_EIO) {
        bmqcrc_note_host_fallback(rc);
        return true;
    }
    return false;
}

}  // close unnamed namespace

const unsigned int Crc32c::k_NULL_CRC32C = BMQCRC_NULL_CRC32C;

unsigned int Crc32c::calculate(const void* data, unsigned int length, unsigned int crc)
{
    return bmqcrc_crc32c(data, length, crc);
}

unsigned int Crc32c::calculate(const bdlbb::Blob& blob, unsigned int crc)
{
    // Same chaining as the reference: every buffer but the last in full, the
    // last up to lastDataBufferLength(); no buffers -> crc unchanged.
    const int numBuffers = blob.numDataBuffers();
    if (numBuffers == 0) {
        return crc;
    }
    for (int i = 0; i < numBuffers - 1; ++i) {
        const bdlbb::BlobBuffer& buffer = blob.buffer(i);
        crc = calculate(buffer.data(), static_cast<unsigned int>(buffer.size()), crc);
    }
    return calculate(blob.buffer(numBuffers - 1).data(),
                     static_cast<unsigned int>(blob.lastDataBufferLength()), crc);
}

int Crc32c::calculateBatch(const void* arena,
                           unsigned long long arenaBytes,
                           const unsigned long long* offsets,
                           const unsigned int* lengths,
                           const unsigned int* seeds,
                           unsigned int* crcs,
                           unsigned long long count,
                           const bmqcrc_opts* opts)
{
    static_assert(sizeof(unsigned long long) == sizeof(uint64_t), "u64");
    static_assert(sizeof(unsigned int) == sizeof(uint32_t), "u32");
    const int rc = bmqcrc_crc32c_batch(arena, arenaBytes,
                                       reinterpret_cast<const uint64_t*>(offsets), lengths, seeds,
                                       crcs, count, opts);
    if (!gpuFailure(rc) || (opts && (opts->flags & BMQCRC_F_DEVICE_PTRS))) {
        return rc;  // device-resident inputs cannot be read on the host
    }
    for (unsigned long long i = 0; i < count; ++i) {
        if (offsets[i] > arenaBytes || lengths[i] > arenaBytes - offsets[i]) {
            return BMQCRC_EINVAL;
        }
    }
    const char* base = static_cast<const char*>(arena);
    for (unsigned long long i = 0; i < count; ++i) {
        crcs[i] = calculate(base + offsets[i], lengths[i], seeds ? seeds[i] : k_NULL_CRC32C);
    }
    return 0;
}

int Crc32c::calculateBatch(const bdlbb::Blob* blobs,
                           unsigned int       count,
                           const unsigned int* seeds,
                           unsigned int*      crcs,
                           const bmqcrc_opts* opts)
{
    // Same buffer selection as calculate(const Blob&): every buffer but the
    // last in full, the last up to lastDataBufferLength().  The buffers stay
    // where they are; bmqcrc_crc32c_gather copies them once, through a pinned
    // staging ring, straight to the device.
    std::vector<const void*> ptr;
    std::vector<uint32_t> len;
    std::vector<uint64_t> first(1, 0);
    for (unsigned int b = 0; b < count; ++b) {
        const int nb = blobs[b].numDataBuffers();
        for (int i = 0; i < nb; ++i) {
            const int n = (i + 1 < nb) ? blobs[b].buffer(i).size() : blobs[b].lastDataBufferLength();
            ptr.push_back(blobs[b].buffer(i).data());
            len.push_back(static_cast<uint32_t>(n));
        }
        first.push_back(ptr.size());
    }
    const int rc = bmqcrc_crc32c_gather(ptr.data(), len.data(), len.size(), first.data(), seeds,
                                        crcs, count, opts);
    if (!gpuFailure(rc)) {
        return rc;
    }
    for (unsigned int b = 0; b < count; ++b) {
        crcs[b] = calculate(blobs[b], seeds ? seeds[b] : k_NULL_CRC32C);
    }
    return 0;
}

}  // namespace bmqp
}  // namespace BloombergLP
