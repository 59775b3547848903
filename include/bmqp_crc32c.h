// bmqp_crc32c.h -- drop-in replacement for BlazingMQ's bmqp::Crc32c with a
// batched MI355X path.
//
// Keeps the exact reference interface
//   /root/reference/src/groups/bmq/bmqp/bmqp_crc32c.h:225-257
// (k_NULL_CRC32C, calculate(const void*, unsigned, unsigned),
//  calculate(const bdlbb::Blob&, unsigned)) with identical results, and adds
// calculateBatch(), the entry the per-message callers (PutEventBuilder,
// FileStore::recoverMessages) use to CRC thousands of payloads in one GPU
// launch.  Thread safe, like the reference (bmqp_crc32c.h:40-42).
#ifndef INCLUDED_BMQP_CRC32C
#define INCLUDED_BMQP_CRC32C

#include "bmqcrc.h"

#ifdef BMQCRC_WITH_BDE
#include <bdlbb_blob.h>
#else
#include "bdlbb_blob_standin.h"
#endif

namespace BloombergLP {
namespace bmqp {

struct Crc32c {
    /// CRC32-C value for a 0 length input (bmqp_crc32c.h:233).
    static const unsigned int k_NULL_CRC32C;

    /// CRC32-C of `length` bytes at `data`, continuing from `crc` (the CRC of
    /// the preceding bytes).  `data` may be 0 only if `length` is 0.
    static unsigned int calculate(const void* data,
                                  unsigned int length,
                                  unsigned int crc = k_NULL_CRC32C);

    /// CRC32-C over the data buffers of `blob` in order, continuing from `crc`.
    static unsigned int calculate(const bdlbb::Blob& blob, unsigned int crc = k_NULL_CRC32C);

    /// Batched: `crcs[i] = calculate(arena + offsets[i], lengths[i],
    /// seeds ? seeds[i] : 0)` for `i < count`, computed on an MI355X in one
    /// launch (`opts` selects device/stream/pointer kind, may be 0).  Returns
    /// 0 on success or a negative BMQCRC_E* code.  Like the reference's
    /// calls it has no GPU failure mode: with host buffers and no usable GPU
    /// (BMQCRC_ENODEV/ENOMEM/EIO from the batch) it finishes on the host
    /// with the scalar path, bit-exact; device-resident inputs return the code.
    static int calculateBatch(const void* arena,
                              unsigned long long arenaBytes,
                              const unsigned long long* offsets,
                              const unsigned int* lengths,
                              const unsigned int* seeds,
                              unsigned int* crcs,
                              unsigned long long count,
                              const bmqcrc_opts* opts = 0);

    /// Batched Blob overload: `crcs[i] = calculate(blobs[i], seeds ? seeds[i] :
    /// 0)` for `i < count`, computed on an MI355X (bmqcrc_crc32c_gather: the
    /// blobs' buffers are copied once, through a pinned staging ring, into
    /// HBM, and every blob is folded as one message).  Returns 0 or a
    /// negative BMQCRC_E* code; without a usable GPU it finishes on the host
    /// like the overload above.
    static int calculateBatch(const bdlbb::Blob* blobs,
                              unsigned int       count,
                              const unsigned int* seeds,
                              unsigned int*      crcs,
                              const bmqcrc_opts* opts = 0);
};

}  // namespace bmqp
}  // namespace BloombergLP

#endif
