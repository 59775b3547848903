// bmqcrc_internal.h -- shared between the host dispatcher and the HIP kernels.
#pragma once
#include <stdint.h>

namespace bmqcrc {

// One wave owns 64 segments; per round each segment advances one 128-byte
// line (= 32 dwords = one full turn of the 32-word fold ring).
constexpr int kLine = 128;
constexpr int kWaveLanes = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kSlots = 2;                                  // LDS ring depth per wave
constexpr int kSlotBytes = kWaveLanes * kLine;             // 8 KiB per round per wave
constexpr int kLdsBytes = kWavesPerBlock * kSlots * kSlotBytes;  // 64 KiB per block
constexpr int kTabBytes = 8 * 256 * 4;  // remainder-reduction slicing tables (LDS)
constexpr int kXbBytes = 4 * 256 * 4;   // move factors x^(8 b 256^i) (LDS)
constexpr uint32_t kDefaultSegBytes = 16384;
constexpr int kPlanBlock = 1024;
constexpr int kPlanMaxBlocks = 256;  // planner grids: contiguous message ranges
constexpr int kSyncFlags = 16;       // BatchArgs::plan_sync: first arrival flag

constexpr int kBuckets = 16;            // segment size classes: floor(log2(lines))

// Experiment knobs for same-box A/B builds (tools/build_variant.sh
// -DBMQCRC_TUNE_BITS=...); the product is built with 0.  bit0 disables the
// non-temporal LDS-DMA loads, bit1 forces a 1-block/CU k_fold grid, bit3
// forces 2, bit4 always builds the size-class map (no shape prediction),
// bit5 reads one- and two-line groups non-temporally too, bit7 plans ragged
// batches with the round-2 pair k_plan<true> + k_plan_sort instead of the
// single-pass k_plan_map, bit9 gives planner blocks whole tiles, bit10 keeps
// two 4-wave k_fold blocks per CU with static group shares (round 3's schedule)
// instead of one 8-wave block claiming groups dynamically (A/B), bit11
// launches BMQCRC_F_PLAN batches as the speculative one-segment kernel instead
// of planning them (the cost of speculating on a stream with no history),
// bit12 plans every batch that is planned at all with k_plan_map (round 4)
// instead of the light k_plan when nothing says it is ragged.
#ifndef BMQCRC_TUNE_BITS
#define BMQCRC_TUNE_BITS 0u
#endif
constexpr uint32_t kTuneBits = BMQCRC_TUNE_BITS;
constexpr bool kShortDefaultPolicy = (kTuneBits & 32u) == 0;
// bit8 turns off the remainder-step skip of one-line groups (A/B).
constexpr bool kHornerSkip = (kTuneBits & 256u) == 0;
// Streams right-aligned at piece granularity when that saves a line or the
// stream is at most this many lines; longer streams otherwise keep a 128-byte
// aligned start, whose lines are whole cache lines (right-aligning every
// stream cost Zipf's k_fold 2.3 %, one line 0.5 %: profiles/r03/ab/ab3_*).
#ifndef BMQCRC_RIGHT_ALIGN_LINES
#define BMQCRC_RIGHT_ALIGN_LINES 1u
#endif
constexpr uint32_t kRightAlignLines = BMQCRC_RIGHT_ALIGN_LINES;
#ifndef BMQCRC_RIGHT_ALIGN
#define BMQCRC_RIGHT_ALIGN 1
#endif
constexpr bool kRightAlign = BMQCRC_RIGHT_ALIGN != 0;  // 0: round 2's 128-byte aligned streams

struct BatchArgs {
    const uint8_t* arena;      // device
    const uint64_t* offsets;   // device, n
    const uint32_t* lengths;   // device, n
    const uint32_t* seeds;     // device, n, or nullptr (all zero)
    uint32_t* out;             // device, n
    uint32_t* seg_first;       // workspace, n: block-local exclusive prefix of segment counts
    uint32_t* block_sum;       // workspace, 3 * nblocks, per k_plan block: [segments |
                               // messages with != 1 segment | segments per message if equal
                               // for all the block's messages, else ~0]
    uint32_t* seginfo;         // workspace, max_segs: segments in size-class order, one word
                               // each (message, | kSegLast for its last segment)
    uint32_t* firstk;          // workspace, max_segs / 64 + 1: k of each group's first entry
    unsigned long long* gdesc; // workspace, max_segs / 64 + 2 (round 4): (epoch << 32) | message
    uint32_t* grec;            // workspace, 8 words per group (round 6): the prefix record
                               // {epoch, message, lanes, 0} and the suffix record, a long
                               // run's tail and head in the group (k_plan_map)
                               // for a group whose 64 seginfo slots are all full segments of
                               // one message (k_plan_map writes this instead of the 64 entries)
    uint32_t* bhist;           // workspace, kBuckets * nblocks: per-block size-class histogram
    uint64_t n;
    uint64_t max_segs;
    uint64_t per_msg;          // messages per planner block (multiple of kPlanBlock)
    uint32_t seg_bytes;
    uint32_t nblocks;          // planner blocks (<= kPlanMaxBlocks)
    uint32_t whole;            // 1: BMQCRC_F_WHOLE_MESSAGES (one segment per message, no planner)
    uint32_t blocks_per_cu;    // k_fold grid: 1 (large messages) or 2 blocks per CU
    uint32_t tune;             // experiment knobs, fixed at build time (BMQCRC_TUNE_BITS below)
    uint32_t map_planned;      // 1: k_plan builds the size-class histogram and k_plan_sort
                               //    runs before k_fold; 0: skipped (the previous batch on this
                               //    workspace was closed-form) and a ragged batch maps segments
                               //    by binary search instead -- slower, never wrong
    uint32_t* shape_hint;      // host-mapped words or nullptr: k_fold writes [0] kHintIdentity,
                               // kHintClosed or kHintRagged, the host reads it when planning
                               // the next batch; [1] the epoch of the last launch whose
                               // k_plan_map gave its map up (sticky)
    // Speculative single launch (spec = u > 0): the previous batch on this
    // workspace had u segments per message (u = 1, or u dividing 64), so no
    // planner runs and k_fold folds segment k of message m in slot m*u + k
    // (a group holds 64/u whole messages).  A message with another segment
    // count is skipped there and folded by the same wave afterwards, 64
    // segments at a time -- correct for any batch, only slower when the
    // guess was wrong.
    uint32_t spec;
    // Single-pass planner (k_plan_map): [1] the device-side launch tag of
    // graph-captured batches, [2] the epoch of a launch whose map
    // was given up (k_fold then searches seg_first), [3] how many
    // launches gave theirs up, [kSyncFlags + b] block b's arrival flag (the
    // epoch of the launch it last arrived in), then kPlanMaxBlocks x
    // (kBuckets + 3) epoch-tagged words the blocks exchange.  Zeroed once
    // when allocated.
    unsigned long long* plan_sync;
    uint32_t plan_epoch;       // k_plan_map launch tag on this workspace, in [1, 2^31); 0: the
                               // tag is plan_sync[1], advanced on the device (graph capture)
    uint64_t map_wait_ticks;   // k_plan_map's grid-wide wait limit (100 MHz wall clock)
    uint32_t class_desc;       // k_plan_map: size classes in descending order (short schedules)
    // 1: plan this ragged batch with the meeting-free pair k_plan<true> +
    // k_plan_sort instead of k_plan_map (the host does so for a while after
    // a map on this workspace was given up: the GPU is shared, kPairAfterVoid)
    uint32_t pair;
    // set by the launcher: a batch of fewer groups than 4-wave blocks x CUs
    // runs its groups one per block first (group k * gridDim.x + blockIdx.x
    // for claim k) over every CU, instead of filling 4-wave blocks on a
    // quarter of them
    uint32_t spread;
};

// Ragged batches planned with the pair after k_fold reports a given-up map
// on the workspace (shape_hint[1] = that launch's epoch), before the
// single-pass planner is tried again.
constexpr uint32_t kPairAfterVoid = 16;

// k_fold groups per wave below which k_plan_map orders the size classes
// largest first: the schedule's tail is then one-line groups instead of a
// row of the largest ones.  Measured on Zipf shards (profiles/r03/ab/
// class_order_*.jsonl, k_fold us, ascending -> descending): 1/16 shard 278 ->
// 272, 1/8 531 -> 525, 1/4 1,036 -> 1,040, 1/2 2,051 -> 2,073, whole 4,082
// -> 4,162; the crossover lies between ~15 and ~30 groups per wave.
constexpr uint64_t kClassDescGroupsPerWave = 24;

constexpr uint32_t kPlanV = 4;  // planner: messages per thread per tile (kPlanBlock * kPlanV)
constexpr uint32_t kSegLast = 0x80000000u;  // seginfo: the entry is its message's last segment

// Ragged batches (map_planned): the single-pass k_plan_map (TUNE bit 7: the
// round-2 pair k_plan<true> + k_plan_sort instead; the pair was kept for
// single-tile blocks until the round-3 planner work made k_plan_map faster
// there too: 19.7 against 24.2 us on the 1/8 Zipf shard,
// profiles/r03/ab/planner_stamps/).
inline bool single_pass_planner(const BatchArgs& a)
{
    return !(a.tune & 128u) && !a.pair;
}

constexpr uint32_t kHintUnknown = 0;
constexpr uint32_t kHintClosed = 1;  // uniform segment counts (> 1); | (u << 8) when u divides 64
constexpr uint32_t kHintRagged = 2;
constexpr uint32_t kHintIdentity = 3;  // one segment per message

}  // namespace bmqcrc

// Launchers (crc32c_kernels.hip).  All asynchronous on `stream`.
extern "C" __attribute__((visibility("hidden"))) int bmqcrc_launch_batch(const bmqcrc::BatchArgs* a, void* stream, int num_cus,
                                   void* ev_start, void* ev_stop);
// k_plan_map blocks one CU holds at once (hipOccupancyMaxActiveBlocksPerMultiprocessor).
extern "C" __attribute__((visibility("hidden"))) int bmqcrc_plan_map_occupancy(int* blocks_per_cu);
extern "C" __attribute__((visibility("hidden"))) int bmqcrc_launch_compare(const uint32_t* got, const uint32_t* expected, uint64_t n,
                                     uint32_t* bad_count, uint32_t* bad_idx, uint32_t bad_cap,
                                     void* stream);
extern "C" __attribute__((visibility("hidden"))) int bmqcrc_launch_blob_combine(const uint32_t* buf_crc, const uint32_t* buf_len,
                                         const uint64_t* msg_first_buf, const uint32_t* seeds,
                                         uint32_t* out, uint64_t n, void* stream);
extern "C" __attribute__((visibility("hidden"))) int bmqcrc_launch_fill(uint8_t* dst, uint64_t nbytes, uint64_t seed, uint64_t begin,
                                  void* stream);
// Ordered mismatch list: pass 0 writes per-block counts to block_cnt, pass 1
// reads the exclusive prefix from block_cnt and writes the mismatching indices
// of ranks [skip, skip + bad_cap) in index order to bad_idx (ascending).
extern "C" __attribute__((visibility("hidden"))) int bmqcrc_launch_compare_ordered(const uint32_t* got, const uint32_t* expected,
                                            uint64_t n, uint32_t* block_cnt, uint32_t nblocks,
                                            uint32_t* bad_idx, uint32_t skip, uint32_t bad_cap,
                                            int pass, void* stream);
// Host-buffer verify with the descriptor walk overlapped (bmqcrc_host.cpp):
// `prepare` runs on the calling thread while the arena is copied to the device
// on a helper thread; it returns 0 and the (offset, length, expected CRC)
// arrays of n messages, or a BMQCRC_E* code with the error already set.
typedef int (*bmqcrc_prepare_fn)(void* ctx, const uint64_t** offsets, const uint32_t** lengths,
                                 const uint32_t** expected, uint64_t* n);
// `bad` receives the lowest min(*n_bad, bad_cap) mismatching indices, like
// bmqcrc_crc32c_verify; *n_written (if non-null) = how many were written.
// With `crcs` non-null the call computes instead of verifying: crcs = the n
// CRCs (expected, n_bad and bad are then unused).  C++ only.
#ifdef __cplusplus
#include <vector>
struct bmqcrc_opts;
__attribute__((visibility("hidden"))) int bmqcrc_verify_host_overlapped(
    const void* arena, uint64_t arena_bytes, bmqcrc_prepare_fn prepare, void* pctx,
    uint64_t* n_bad, std::vector<uint64_t>* bad, uint64_t bad_cap, const bmqcrc_opts* opts,
    std::vector<uint32_t>* crcs = nullptr, uint64_t* n_written = nullptr);
#endif
// Thread-local error message shared by every C-ABI source (bmqcrc_last_error).
extern "C" __attribute__((visibility("hidden"))) int bmqcrc_set_error(int rc, const char* msg);
extern "C" __attribute__((visibility("hidden"))) void bmqcrc_clear_error(void);
