/* bmqcrc.h -- C ABI of the MI355X CRC32C library (libbmqcrc.so).
 *
 * Drop-in boundary for BlazingMQ's per-message CRC32C path.  Every entry point
 * takes plain pointers and sizes; no HIP or torch types cross the ABI.
 *
 * Reference interfaces replaced (paths relative to /root/reference):
 *   bmqcrc_crc32c        bmqp::Crc32c::calculate(const void*, unsigned, unsigned)
 *                        src/groups/bmq/bmqp/bmqp_crc32c.h:244-246, .cpp:41-45
 *   bmqcrc_crc32c_blob   bmqp::Crc32c::calculate(const bdlbb::Blob&, unsigned)
 *                        src/groups/bmq/bmqp/bmqp_crc32c.h:255-256, .cpp:47-67
 *   BMQCRC_NULL_CRC32C   bmqp::Crc32c::k_NULL_CRC32C (bmqp_crc32c.h:233, .cpp:39)
 *   bmqcrc_crc32c_batch  the per-message loops that call the above once per
 *                        message: PutEventBuilder::packMessage
 *                        (src/groups/bmq/bmqp/bmqp_puteventbuilder.cpp:302,320,400,413)
 *                        and FileStore::recoverMessages
 *                        (src/groups/mqb/mqbs/mqbs_filestore.cpp:2603-2624);
 *                        one call CRCs a whole batch on an MI355X.
 *   bmqcrc_combine       GF(2) shift-combine crc(A||B) from crc(A), crc(B), |B|
 *                        (used to stitch segments; no reference equivalent).
 *
 * Semantics of every CRC entry point are those of bmqp::Crc32c: reflected
 * CRC-32C (Castagnoli, 0x1EDC6F41), `crc` is the finalised CRC of the
 * preceding bytes (0 = k_NULL_CRC32C), calculate(p, 0, crc) == crc.
 *
 * Scalar entry points run on the host CPU (like the reference: one small
 * buffer per call is latency-bound; a GPU round trip would be ~10^4 x slower).
 * The batch entry points run ONLY on the GPU: they never fall back to the CPU
 * and return BMQCRC_ENODEV when no MI355X is usable.
 */
#ifndef BMQCRC_H
#define BMQCRC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BMQCRC_NULL_CRC32C 0u

/* Return codes: 0 on success, negative errno-style values on failure. */
#define BMQCRC_OK 0
#define BMQCRC_EIO (-5)
#define BMQCRC_ENOMEM (-12)
#define BMQCRC_ENODEV (-19)
#define BMQCRC_EINVAL (-22)

/* bmqcrc_opts.flags */
#define BMQCRC_F_DEVICE_PTRS 0x1u /* arena/offsets/lengths/seeds/out are device pointers */
#define BMQCRC_F_ASYNC 0x2u       /* device ptrs only: return after enqueueing on stream */
#define BMQCRC_F_TIME_KERNEL 0x4u /* record HIP events around the fold kernel (see bmqcrc_kernel_timing) */
/* Fold every message in one lane: no segmentation, no planner launches (one
 * kernel per batch).  For batches of small messages (PUT events, small
 * journal records): correct for any lengths, but a long message keeps its
 * whole wave busy for its full length. */
#define BMQCRC_F_WHOLE_MESSAGES 0x8u
/* ABI 2.2.  Plan this batch (planner launches before the fold) instead of
 * launching it on the guess that it has the previous batch's shape on the same
 * (device, stream); see bmqcrc_last_launch.  What a caller whose batch shapes
 * alternate pays per batch. */
#define BMQCRC_F_PLAN 0x10u

typedef struct bmqcrc_opts {
    uint32_t struct_size; /* sizeof(bmqcrc_opts); 0 reads the ABI 2.0 fields only (device,
                             stream, flags, seg_bytes) and never touches the bytes
                             after them, so a 2.0 caller's 24-byte struct is safe:
                             set it to use anything later (ABI 2.1-2.4 read the
                             whole struct when it was 0; such callers must set it) */
    int32_t device;       /* HIP device ordinal; -1 = current device */
    void* stream;         /* hipStream_t; NULL = that device's default (null) stream */
    uint32_t flags;       /* BMQCRC_F_* */
    uint32_t seg_bytes;   /* segment size in bytes, multiple of 128 in [256, 2^30]; 0 = automatic
                             from the batch's size (256 B - 64 KiB) */
    /* ABI 2.1.  Host-buffer calls only (bmqcrc_crc32c_batch, bmqcrc_crc32c_verify
     * and the format walks of bmqcrc_protocol.h: recovery verify, PUT-event
     * fill/verify, ledger validate): with ndevices > 1 the input is split over
     * ndevices devices, each copying its part over its own PCIe link.  The
     * batch splits the messages byte-balanced (bmqcrc_crc32c_batch_multi);
     * verify and the walks cut the buffer into contiguous byte ranges, copied
     * while the calling thread walks the format, each device verifies the
     * messages lying in its range and the few that straddle a cut are done by
     * the first device.  Results are identical to the single-device call.  devices == NULL means
     * 0..ndevices-1; a device may be listed more than once (each listing gets
     * a library-owned stream); `device` and `stream` are then ignored.
     * ndevices 0 or 1: the single device above.  Callers built against ABI
     * 2.0 (smaller struct_size) get 0. */
    uint32_t ndevices;
    const int32_t* devices;
    /* ABI 2.4.  bmqcrc_crc32c_batch with BMQCRC_F_DEVICE_PTRS: the caller's
     * upper bound on every lengths[i] (0 = none declared).  When it fits one
     * segment the batch is ONE fold launch with no planner, whatever the
     * previous batch on (device, stream) looked like -- the device-resident
     * counterpart of what a host-buffer batch gets from its seen lengths (a
     * broker knows its maximum PUT payload; its lengths live in HBM).  A
     * message longer than the bound is still computed exactly (its wave folds
     * it in a second pass), only slower.  BMQCRC_F_PLAN takes precedence.
     * Callers built against ABI <= 2.3 (smaller struct_size) get 0. */
    uint32_t max_len;
    /* ABI 2.5.  With max_len: the caller's lower bound on every lengths[i]
     * (0 = none).  When every length in [min_len, max_len] has the same u
     * segments and u divides 64 (1k x 4 KiB at 256-byte segments: u = 16),
     * the batch is likewise one launch (the speculative uniform form, known
     * instead of guessed); a message outside the range stays exact. */
    uint32_t min_len;
} bmqcrc_opts;

/* ---- scalar (host CPU) -------------------------------------------------- */

/* bmqp::Crc32c::calculate(data, length, crc).  data may be NULL iff length==0. */
uint32_t bmqcrc_crc32c(const void* data, uint32_t length, uint32_t crc);

/* bmqp::Crc32c::calculate(blob, crc): CRC of the concatenation of nbuf
 * buffers, chained from crc.  nbuf == 0 returns crc. */
uint32_t bmqcrc_crc32c_blob(const void* const* bufs, const uint32_t* lens, uint32_t nbuf,
                            uint32_t crc);

/* crc(A||B) given crc(A), crc(B) (both finalised, seed 0 for B) and |B|. */
uint32_t bmqcrc_combine(uint32_t crcA, uint32_t crcB, uint64_t lenB);

/* ---- batch (MI355X) ----------------------------------------------------- */

/* out[i] = calculate(arena + offsets[i], lengths[i], seeds ? seeds[i] : 0)
 * for i < n.  Messages may sit anywhere in [arena, arena + arena_bytes) at any
 * byte alignment and may overlap.  With BMQCRC_F_DEVICE_PTRS all five arrays
 * are device memory of opts->device (inputs "device resident"); otherwise they
 * are host memory and the library stages them through HBM.  Returns 0,
 * BMQCRC_EINVAL, BMQCRC_ENODEV, BMQCRC_ENOMEM or BMQCRC_EIO. */
int bmqcrc_crc32c_batch(const void* arena, uint64_t arena_bytes, const uint64_t* offsets,
                        const uint32_t* lengths, const uint32_t* seeds, uint32_t* out,
                        uint64_t n, const bmqcrc_opts* opts);

/* Batched verification (journal recovery, mqbs_filestore.cpp:2603-2624):
 * computes the CRC of every message exactly like bmqcrc_crc32c_batch (seed 0)
 * and compares it on the device with expected[i].  *n_bad receives the number
 * of mismatches; the min(n_bad, bad_cap) LOWEST mismatching indices are
 * written to bad_idx in ascending order (bad_idx may be NULL when bad_cap is 0).  Pointer kinds follow opts->flags
 * (n_bad/bad_idx are always host memory).  GPU only. */
int bmqcrc_crc32c_verify(const void* arena, uint64_t arena_bytes, const uint64_t* offsets,
                         const uint32_t* lengths, const uint32_t* expected, uint64_t n,
                         uint64_t* n_bad, uint64_t* bad_idx, uint64_t bad_cap,
                         const bmqcrc_opts* opts);

/* bmqp::Crc32c::calculate(const bdlbb::Blob&, crc) (bmqp_crc32c.cpp:47-67) for
 * n blobs at once.  Blob m is the concatenation of buffers
 * [msg_first_buf[m], msg_first_buf[m+1]) of (buf_offsets, buf_lengths) in
 * the arena (msg_first_buf has n+1 entries); out[m] = its CRC chained from
 * seeds ? seeds[m] : 0.  Per-buffer CRCs are combined on the device with
 * crc(A||B) = crc(A) * x^(8|B|) ^ crc0(B).  GPU only. */
int bmqcrc_crc32c_blobs(const void* arena, uint64_t arena_bytes, const uint64_t* buf_offsets,
                        const uint32_t* buf_lengths, uint64_t nbuf,
                        const uint64_t* msg_first_buf, const uint32_t* seeds, uint32_t* out,
                        uint64_t n, const bmqcrc_opts* opts);

/* The same Blob CRCs when the buffers are scattered in host memory (a
 * bdlbb::Blob's data buffers, as Crc32c::calculateBatch(const Blob*) passes
 * them): message m is the concatenation of bufs[msg_first_buf[m] ..
 * msg_first_buf[m+1]) with their buf_lengths, out[m] = its CRC chained from
 * seeds ? seeds[m] : 0.  Host pointers only (BMQCRC_F_DEVICE_PTRS and
 * BMQCRC_F_ASYNC are EINVAL), synchronous.  The buffers are gathered by
 * several host threads through a pinned staging ring whose chunks go to HBM
 * while the next ones are gathered (one host copy, no pageable staging), then
 * CRC'd as one batch on the device.  A message may be at most 2^32-1 bytes.
 * GPU only. */
int bmqcrc_crc32c_gather(const void* const* bufs, const uint32_t* buf_lengths, uint64_t nbuf,
                         const uint64_t* msg_first_buf, const uint32_t* seeds, uint32_t* out,
                         uint64_t n, const bmqcrc_opts* opts);

/* Host-pointer batch sharded over `ndev` devices: messages are split into
 * contiguous byte-balanced slices, one per device, each on its own stream,
 * with no inter-device communication.  devices==NULL means 0..ndev-1. */
int bmqcrc_crc32c_batch_multi(const void* arena, uint64_t arena_bytes, const uint64_t* offsets,
                              const uint32_t* lengths, const uint32_t* seeds, uint32_t* out,
                              uint64_t n, const int* devices, int ndev, uint32_t seg_bytes);

/* Pre-size the device workspace of (device, stream) for batches of up to
 * n_msgs messages over arena_bytes bytes, so later calls allocate nothing
 * (required before capturing bmqcrc_crc32c_batch into a hipGraph). */
int bmqcrc_reserve(int device, void* stream, uint64_t n_msgs, uint64_t arena_bytes,
                   uint32_t seg_bytes);

/* Fill nbytes of device memory with bytes [begin, begin + nbytes) of the
 * deterministic synthetic payload stream `seed` used by the benchmarks
 * (splitmix64 counter stream; begin must be a multiple of 8). */
int bmqcrc_fill_synthetic(void* dev_dst, uint64_t nbytes, uint64_t seed, uint64_t begin,
                          const bmqcrc_opts* opts);

/* Sum and count of fold-kernel durations (ms, HIP events on the launch
 * stream) recorded by calls with BMQCRC_F_TIME_KERNEL on (device, stream)
 * since the previous query; waits for those events, then resets. */
int bmqcrc_kernel_timing(int device, void* stream, double* total_ms, uint32_t* count);

/* ABI 2.2.  Launch plan of the previous batch CRC'd on (device, stream):
 * *kernels = kernels it launched (1: the fold alone; 2: planner + fold, the
 * planner being the single-pass size-class map for large ragged batches
 * (ABI 2.3); 3: planner, size-class sort, fold), *spec = the segments per message its single
 * launch assumed (0: planned; 1 also for BMQCRC_F_WHOLE_MESSAGES), *seg_bytes =
 * the segment size used.  Any pointer may be NULL. */
int bmqcrc_last_launch(int device, void* stream, uint32_t* kernels, uint32_t* spec,
                       uint32_t* seg_bytes);

/* ABI 2.7.  Whether the previous planned batch on (device, stream) had its
 * size-class map built (*map = 1: k_plan_map, or k_plan + k_plan_sort) or
 * was planned by the light k_plan alone, whose fold searches the
 * per-message segment offsets (*map = 0; also for single-launch batches).
 * A batch captured into a graph always gets the map. */
int bmqcrc_last_plan(int device, void* stream, uint32_t* map);

/* ABI 2.2.  Drop the batch-shape prediction of (device, stream): the next
 * batch there is planned (k_plan runs) instead of being launched on the guess
 * that it has the previous batch's shape.  For callers that know their next
 * batch differs; a batch still in flight may set the prediction again. */
int bmqcrc_forget_shape(int device, void* stream);

/* ABI 2.3.  Longest time (microseconds) the blocks of the single-pass
 * planner (ragged batches) wait for each other on (device, stream) before
 * giving up the size-class map of that batch; default 100 (1000 before round
 * 4's final build: eight processes sharing one GPU then spun up to 1 ms per
 * planner launch).  The planner's
 * blocks meet once, grid-wide, and its grid never exceeds what the device
 * holds at once; when the GPU still cannot run them all together (other
 * streams or processes hold the CUs) a block that waited this long gives the
 * map up, blocks that find it given up leave at once, and the fold maps that
 * batch's segments by searching the per-message segment offsets instead of
 * the size-class order (ABI 2.5; before, one lane per message) -- results are
 * exact either way, only slower.  0 gives every map up before the first poll
 * (a test hook for that path).  *voided (may be NULL) receives how many
 * planned batches on (device, stream) gave up their map so far; asking for it
 * waits for the work already enqueued on that stream. */
int bmqcrc_plan_wait(int device, void* stream, uint64_t wait_us, uint64_t* voided);

/* Zero-copy input: page-lock `bytes` of ordinary host memory at `host` and map
 * it into the GPU address space (hipHostRegister, mapped + portable).
 * *dev_ptr receives the device-side address of `host`; pass it as the arena
 * of a BMQCRC_F_DEVICE_PTRS batch and the kernels read the broker's blob
 * buffers over PCIe in place, with no staging copy (SURVEY.md 8(d),
 * end-to-end).  Undo with bmqcrc_host_unregister(host).  GPU only. */
int bmqcrc_host_register(void* host, uint64_t bytes, int device, void** dev_ptr);
int bmqcrc_host_unregister(void* host);

/* Number of usable HIP devices (0 when none). */
int bmqcrc_device_count(void);

/* Message for the last failing call on this thread ("" if none). */
const char* bmqcrc_last_error(void);

/* ABI 2.2.  The C++ spellings at the reference's call sites
 * (bmqp::Crc32c::calculateBatch, the bmqcrc_protocol.h wrappers) finish on the
 * host when a batch call fails with BMQCRC_ENODEV, ENOMEM or EIO, because the
 * reference's interface has no error channel.  Each such fallback is recorded
 * here: bmqcrc_host_fallbacks returns how many happened in this process and
 * stores the last failing code in *last_rc (may be NULL).  The first EIO (a
 * kernel fault or a sticky HIP error, as opposed to a missing device) is also
 * printed once on stderr with its HIP error, so a broken GPU context is never
 * hidden behind correct host results. */
void bmqcrc_note_host_fallback(int32_t rc);
uint64_t bmqcrc_host_fallbacks(int32_t* last_rc);

/* ABI version: (major << 16) | minor (2.6). */
uint32_t bmqcrc_version(void);

#ifdef __cplusplus
}
#endif

#endif /* BMQCRC_H */
