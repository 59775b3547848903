// bmqcrc_host.cpp -- C ABI implementation (include/bmqcrc.h).
//
// Device context, per-(device, stream) workspaces, host<->device staging and
// multi-GPU sharding around the HIP kernels in crc32c_kernels.hip.  The batch
// path is GPU-only: with no usable device it returns BMQCRC_ENODEV and never
// computes on the CPU.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/bmqcrc.h"
#include "bmqcrc_internal.h"

namespace bmqcrc {
uint32_t cpu_crc32c(const void* data, uint32_t length, uint32_t crc);
uint32_t cpu_combine(uint32_t crcA, uint32_t crcB, uint64_t lenB);
}  // namespace bmqcrc

using namespace bmqcrc;

namespace {

thread_local std::string t_err;

int fail(int rc, const std::string& msg)
{
    t_err = msg;
    return rc;
}

#define HIP_TRY(expr)                                                                       \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess) {                                                             \
            return fail(e_ == hipErrorOutOfMemory ? BMQCRC_ENOMEM : BMQCRC_EIO,             \
                        std::string(#expr ": ") + hipGetErrorString(e_));                   \
        }                                                                                   \
    } while (0)

// Restores the calling thread's current HIP device on scope exit: the library
// selects the device a call targets, and a drop-in must not retarget the
// caller's later HIP/torch work on that thread.
struct DeviceGuard {
    int prev = -1;
    DeviceGuard()
    {
        if (hipGetDevice(&prev) != hipSuccess) {
            prev = -1;
        }
    }
    ~DeviceGuard()
    {
        if (prev >= 0) {
            (void)hipSetDevice(prev);
        }
    }
    DeviceGuard(const DeviceGuard&) = delete;
    DeviceGuard& operator=(const DeviceGuard&) = delete;
};

struct DevBuf {
    void* p = nullptr;
    uint64_t bytes = 0;
    bool fresh = false;  // set when ensure() (re)allocated
    int ensure(uint64_t want)
    {
        fresh = false;
        if (want <= bytes) {
            return 0;
        }
        fresh = true;
        if (p) {
            (void)hipFree(p);
            p = nullptr;
            bytes = 0;
        }
        want = std::max<uint64_t>(want, 256);
        HIP_TRY(hipMalloc(&p, want));
        bytes = want;
        return 0;
    }
    ~DevBuf()
    {
        if (p) {
            (void)hipFree(p);
        }
    }
};

// Planner + staging scratch for one (device, stream).
struct Workspace {
    std::mutex mu;
    DevBuf seg_first, block_sum, seginfo, firstk, gdesc, grec, bhist, plan_sync;
    uint32_t plan_epoch = 0;  // k_plan_map launches on this workspace (BatchArgs::plan_epoch)
    uint64_t map_wait_ticks = 10000;  // 100 us (bmqcrc_plan_wait)

    // host-pointer staging
    DevBuf arena, offsets, lengths, seeds, out;
    // verify / blobs
    DevBuf expected, vcount, vidx, vblock, buf_crc, first_buf;
    // BMQCRC_F_TIME_KERNEL: event pairs around k_fold not yet reported
    std::vector<std::pair<hipEvent_t, hipEvent_t>> timing, spare;
    // Shape of the last batch planned on this workspace, written by k_fold
    // into host-mapped memory (kHint*): after a closed-form batch the next
    // one skips the size-class histogram and the k_plan_sort launch.  A wrong guess only
    // costs speed (k_fold then maps segments by binary search).
    uint32_t* hint_host = nullptr;
    uint32_t* hint_dev = nullptr;
    // Launch plan of the last batch (bmqcrc_last_launch).
    uint32_t last_kernels = 0, last_spec = 0, last_seg = 0, last_map = 0;
    // Given-up planner maps (hint_host[1], written by k_fold): the last epoch
    // seen, and how many more ragged batches take the meeting-free pair.
    uint32_t void_seen = 0, pair_left = 0;
    // Pinned staging ring for gathered host buffers (bmqcrc_crc32c_gather):
    // kGatherSlots chunks of kGatherChunk bytes, each reusable once the event
    // recorded after its H2D copy has completed.
    uint8_t* pin = nullptr;
    hipEvent_t pin_ev[16] = {};
    bool pin_used[16] = {};
    ~Workspace()
    {
        if (hint_host) {
            (void)hipHostFree(hint_host);
        }
        if (pin) {
            (void)hipHostFree(pin);
        }
        for (hipEvent_t e : pin_ev) {
            if (e) {
                (void)hipEventDestroy(e);
            }
        }
        for (auto& v : {timing, spare}) {
            for (auto& e : v) {
                (void)hipEventDestroy(e.first);
                (void)hipEventDestroy(e.second);
            }
        }
    }
};

struct DeviceState {
    int num_cus = 0;
    // k_plan_map blocks the device holds at once (occupancy x CUs, at most
    // kPlanMaxBlocks): its grid never exceeds this, so on an idle GPU every
    // block is resident for the grid-wide meeting (a partitioned or smaller
    // part gets fewer, fuller blocks instead of a wait that must give up)
    uint32_t plan_resident = kPlanMaxBlocks;
};

std::mutex g_mu;
std::map<std::pair<int, void*>, std::unique_ptr<Workspace>> g_ws;
std::map<int, DeviceState> g_dev;

int device_count_raw()
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        return 0;
    }
    return n;
}

int resolve_device(int dev, int* out)
{
    const int n = device_count_raw();
    if (n <= 0) {
        return fail(BMQCRC_ENODEV, "no HIP device available (batch CRC32C runs only on the GPU)");
    }
    if (dev < 0) {
        HIP_TRY(hipGetDevice(&dev));
    }
    if (dev >= n) {
        return fail(BMQCRC_EINVAL, "device ordinal out of range");
    }
    *out = dev;
    return 0;
}

int device_state(int dev, DeviceState** st)
{
    std::lock_guard<std::mutex> g(g_mu);
    DeviceState& s = g_dev[dev];
    if (s.num_cus == 0) {
        hipDeviceProp_t prop;
        HIP_TRY(hipGetDeviceProperties(&prop, dev));
        if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
            return fail(BMQCRC_ENODEV, std::string("device is ") + prop.gcnArchName +
                                           ", this library is built for gfx950 (MI355X) only");
        }
        HIP_TRY(hipSetDevice(dev));
        int per = 0;
        if (bmqcrc_plan_map_occupancy(&per) != 0 || per <= 0) {
            return fail(BMQCRC_EIO, "k_plan_map occupancy query failed");
        }
        s.plan_resident = (uint32_t)std::min<uint64_t>(
            (uint64_t)per * (uint64_t)std::max(prop.multiProcessorCount, 1), kPlanMaxBlocks);
        s.num_cus = prop.multiProcessorCount;
    }
    *st = &s;
    return 0;
}

Workspace* workspace(int dev, void* stream)
{
    std::lock_guard<std::mutex> g(g_mu);
    auto& w = g_ws[std::make_pair(dev, stream)];
    if (!w) {
        w.reset(new Workspace());
    }
    return w.get();
}

uint64_t max_segs_for(uint64_t n, uint64_t arena_bytes, uint32_t seg)
{
    // Sum over messages of ceil(len/seg) <= n + total_len/seg.  For
    // non-overlapping messages total_len <= arena_bytes; segments past this
    // bound (overlapping batches) are resolved by binary search in-kernel.
    return n + arena_bytes / seg + 64;
}

// Contiguous ranges of whole kPlanBlock tiles, at most kPlanMaxBlocks blocks.
// (As many blocks as possible: the planners are latency-bound per block.
// Fewer, fuller blocks -- at least 8 tiles each, so that the 1/8 Zipf shard
// takes the single-pass planner -- traced 36.8 against 26.3 us there,
// profiles/r03/ab/planner_block_sizing/.)
static void split_ranges(uint64_t items, uint64_t* per, uint32_t* blocks,
                         uint32_t max_blocks = kPlanMaxBlocks)
{
    const uint64_t tiles = std::max<uint64_t>((items + kPlanBlock - 1) / kPlanBlock, 1);
    const uint64_t nb = std::min<uint64_t>(
        tiles, std::max<uint32_t>(1u, std::min<uint32_t>(max_blocks, kPlanMaxBlocks)));
    uint64_t tiles_per = (tiles + nb - 1) / nb;
    if (kTuneBits & 512u) {  // A/B: whole planner tiles (kPlanV x kPlanBlock) per block
        tiles_per = (tiles_per + kPlanV - 1) / kPlanV * kPlanV;
    }
    *per = tiles_per * kPlanBlock;
    *blocks = (uint32_t)((tiles + tiles_per - 1) / tiles_per);
}

int plan_ws(Workspace* w, hipStream_t s, uint64_t n, uint64_t arena_bytes, uint32_t seg,
            BatchArgs* a, const DeviceState& st)
{
    const int num_cus = st.num_cus;
    const uint64_t max_segs = max_segs_for(n, arena_bytes, seg);
    // k_plan_map's blocks meet grid-wide: never more than the GPU holds
    split_ranges(n, &a->per_msg, &a->nblocks, st.plan_resident);
    int rc;
    if ((rc = w->seg_first.ensure(4 * std::max<uint64_t>(n, 1))) ||
        (rc = w->block_sum.ensure(12ull * kPlanMaxBlocks)) ||
        (rc = w->seginfo.ensure(4 * max_segs)) ||
        (rc = w->firstk.ensure(4 * (max_segs / 64 + 2))) ||
        (rc = w->gdesc.ensure(8 * (max_segs / 64 + 2))) ||
        (rc = w->grec.ensure(32 * (max_segs / 64 + 2))) ||
        (rc = w->bhist.ensure(4ull * kBuckets * kPlanMaxBlocks)) ||
        (rc = w->plan_sync.ensure(8ull * (kSyncFlags + kPlanMaxBlocks +
                                          kPlanMaxBlocks * (kBuckets + 3))))) {
        return rc;
    }
    if (w->plan_sync.fresh) {  // zero counters, no given-up epoch (stream-ordered)
        HIP_TRY(hipMemsetAsync(w->plan_sync.p, 0, w->plan_sync.bytes, s));
    }
    if (w->grec.fresh) {  // no run record of any epoch either
        HIP_TRY(hipMemsetAsync(w->grec.p, 0, w->grec.bytes, s));
    }
    if (w->gdesc.fresh) {  // no group descriptor of any epoch (epochs start at 1)
        HIP_TRY(hipMemsetAsync(w->gdesc.p, 0, w->gdesc.bytes, s));
    }
    // host tags stay in [1, 2^31): a batch captured into a graph takes its
    // tags from the device instead (0x80000000 | count, k_epoch_advance)
    w->plan_epoch = w->plan_epoch % 0x7fffffffu + 1u;
    a->plan_sync = (unsigned long long*)w->plan_sync.p;
    a->plan_epoch = w->plan_epoch;
    a->map_wait_ticks = w->map_wait_ticks;
    if (!w->hint_host) {
        void* h = nullptr;
        HIP_TRY(hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocPortable |
                                          hipHostMallocCoherent));
        ((volatile uint32_t*)h)[0] = kHintUnknown;
        ((volatile uint32_t*)h)[1] = 0;  // no given-up map yet
        void* d = nullptr;
        const hipError_t e = hipHostGetDevicePointer(&d, h, 0);
        if (e != hipSuccess) {
            (void)hipHostFree(h);
            return fail(BMQCRC_EIO, std::string("hipHostGetDevicePointer: ") + hipGetErrorString(e));
        }
        w->hint_host = (uint32_t*)h;
        w->hint_dev = (uint32_t*)d;
    }
    a->shape_hint = w->hint_dev;
    {
        // expected k_fold groups per wave (max_segs bounds the segments)
        const uint64_t waves = (uint64_t)(num_cus > 0 ? num_cus : 256) * a->blocks_per_cu *
                               kWavesPerBlock;
        a->class_desc = (max_segs / 64) < kClassDescGroupsPerWave * waves ? 1u : 0u;
    }
    // seginfo entries hold 31-bit message indices (bit 31 marks a last
    // segment): larger batches map their segments by binary search
    a->map_planned = n < (1ull << 31) ? 1u : 0u;
    a->seg_first = (uint32_t*)w->seg_first.p;
    a->firstk = (uint32_t*)w->firstk.p;
    a->gdesc = (unsigned long long*)w->gdesc.p;
    a->grec = (uint32_t*)w->grec.p;
    a->block_sum = (uint32_t*)w->block_sum.p;
    a->seginfo = (uint32_t*)w->seginfo.p;
    a->bhist = (uint32_t*)w->bhist.p;
    a->max_segs = max_segs;
    return 0;
}

// 0 = automatic (auto_shape, per batch); otherwise validated here.
int check_seg(uint32_t* seg)
{
    if (*seg == 0) {
        return 0;
    }
    if (*seg % kLine != 0 || *seg < 256 || *seg > (1u << 30)) {
        return fail(BMQCRC_EINVAL, "seg_bytes must be a multiple of 128 in [256, 2^30]");
    }
    return 0;
}

struct Ctx {
    int dev = 0;
    DeviceState* st = nullptr;
    hipStream_t s = nullptr;
    Workspace* w = nullptr;
};

int open_ctx(int dev, void* user_stream, Ctx* c)
{
    int rc = device_state(dev, &c->st);
    if (rc) {
        return rc;
    }
    HIP_TRY(hipSetDevice(dev));
    c->dev = dev;
    c->s = (hipStream_t)user_stream;  // NULL: the device's default (null) stream, as in HIP
    c->w = workspace(dev, user_stream);
    return 0;
}

// A speculative single launch (BatchArgs::spec) is used only when every
// k_fold wave owns at least one group of 64 messages: a message longer than
// one segment is then folded by the wave that met it, and no wave is idle
// while another folds one.
bool spec_eligible(const Ctx& c, uint64_t n, uint32_t blocks_per_cu)
{
    const uint32_t per_cu = (kTuneBits & 2u) ? 1u : (kTuneBits & 8u) ? 2u : blocks_per_cu;
    const uint64_t waves = (uint64_t)(c.st->num_cus > 0 ? c.st->num_cus : 256) * per_cu *
                           kWavesPerBlock;
    return (n + 63) / 64 >= waves;
}

// Enqueue planner + fold on device pointers (caller holds c.w->mu).
// Segment size (when the caller left it at 0) and k_fold blocks per CU, from
// the batch's average message size and total bytes.  Measured on MI355X
// (profiles/r01/sweeps/, profiles/r02/seg_sweep_*.jsonl):
//  * >= 4 GiB of >= 16 KiB messages: 64 KiB segments, one 4-wave block per CU
//    (64k x 64 KiB: 620 us, the fastest shape);
//  * otherwise two blocks per CU; messages averaging >= 16 KiB get 16 KiB
//    segments when that still gives every wave slot a group of 64 (2 GiB of
//    64 KiB messages);
//  * everything else: the longest of 2 KiB, 1 KiB, 512 B, 256 B that gives
//    every wave two groups.  Segments of 4 and 8 KiB are never chosen: a wave
//    whose 64 segments start 4 or 8 KiB apart (uniform messages of those
//    sizes) streams at 0.71-0.75 of the roofline against 0.83-0.84 with
//    2 KiB segments, and Zipf 4M is within 2 % at 2, 4 and 16 KiB.
void auto_shape(uint64_t n, uint64_t arena_bytes, int num_cus, uint32_t* seg,
                uint32_t* blocks_per_cu)
{
    const uint64_t cus = (uint64_t)(num_cus > 0 ? num_cus : 256);
    const uint64_t wave_segs = (uint64_t)kWavesPerBlock * kWaveLanes;  // per block
    const bool large = n > 0 && arena_bytes / n >= kDefaultSegBytes;
    if (large && arena_bytes / (4 * kDefaultSegBytes) >= cus * wave_segs) {
        *blocks_per_cu = 1;
        if (*seg == 0) {
            *seg = 4 * kDefaultSegBytes;
        }
        return;
    }
    *blocks_per_cu = 2;
    if (*seg == 0) {
        const uint64_t slots = cus * 2 * wave_segs;
        if (large && arena_bytes / kDefaultSegBytes >= slots) {
            *seg = kDefaultSegBytes;
            return;
        }
        *seg = 256;
        for (uint32_t s : {2048u, 1024u, 512u}) {
            if (arena_bytes / s >= 2 * slots) {
                *seg = s;
                break;
            }
        }
    }
}

uint64_t max_length(const uint32_t* lengths, uint64_t n)
{
    uint32_t m = 0;
    for (uint64_t i = 0; i < n; ++i) {
        m = std::max(m, lengths[i]);
    }
    return m;
}

uint64_t min_length(const uint32_t* lengths, uint64_t n)
{
    uint32_t m = n ? UINT32_MAX : 0u;
    for (uint64_t i = 0; i < n; ++i) {
        m = std::min(m, lengths[i]);
    }
    return m;
}

// host_max_len: the longest message when the lengths were seen on the host, or
// the caller's declared bound for device lengths (bmqcrc_opts.max_len: a
// message over it is still exact, folded by its wave's second pass)
// (host-buffer calls), UINT64_MAX when they live on the device.
int run_batch(Ctx& c, uint32_t flags, uint32_t seg, const void* arena, uint64_t arena_bytes,
              const uint64_t* offsets, const uint32_t* lengths, const uint32_t* seeds,
              uint32_t* out, uint64_t n, uint64_t host_max_len = UINT64_MAX,
              uint64_t host_min_len = 0)
{
    Workspace* w = c.w;
    BatchArgs a;
    memset(&a, 0, sizeof(a));
    a.n = n;
    auto_shape(n, arena_bytes, c.st->num_cus, &seg, &a.blocks_per_cu);
    a.seg_bytes = seg;
    a.tune = kTuneBits;
    int rc;
    if (flags & BMQCRC_F_WHOLE_MESSAGES) {
        a.whole = 1;  // identity map over messages: no planner workspace
        a.max_segs = n;
    } else if ((rc = plan_ws(w, c.s, n, arena_bytes, seg, &a, *c.st))) {
        return rc;
    } else if (!(kTuneBits & 16u) && !(flags & BMQCRC_F_PLAN)) {
        const uint32_t hint = __atomic_load_n(w->hint_host, __ATOMIC_RELAXED);
        const uint32_t shape = hint & 0xffu, hint_u = hint >> 8;
        if (shape == kHintClosed || shape == kHintIdentity) {
            a.map_planned = 0;  // last batch was closed-form: predict this one is too
        }
        if (shape == kHintIdentity && spec_eligible(c, n, a.blocks_per_cu)) {
            a.spec = 1;  // ... and one segment per message: one launch, no planner
        } else if (shape == kHintClosed && hint_u >= 2u && hint_u <= 64u && 64u % hint_u == 0u &&
                   (uint64_t)n * hint_u <= 0xFFFFFF00ull) {
            // ... and the same u segments per message, u dividing 64: every
            // group holds 64/u whole messages, so one launch needs no planner
            // and no cross-group combine (a message of another count is folded
            // by its wave's second pass, and the next batch is planned again)
            a.spec = hint_u;
        }
    }
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    const bool capturing = hipStreamIsCapturing(c.s, &cap) == hipSuccess &&
                           cap == hipStreamCaptureStatusActive;
    // A captured launch is replayed as recorded: the light planner's "the
    // next batch gets the map" never happens inside a graph, so a capture
    // keeps the map whatever the history
    if (!(kTuneBits & (16u | 4096u)) && !capturing && !a.whole && !a.spec && a.map_planned &&
        w->hint_host &&
        (__atomic_load_n(w->hint_host, __ATOMIC_RELAXED) & 0xffu) != kHintRagged &&
        !(host_max_len != UINT64_MAX && host_max_len > a.seg_bytes &&
          (host_min_len == 0 || (host_min_len - 1) / a.seg_bytes != (host_max_len - 1) / a.seg_bytes))) {
        // Planned with no evidence that the batch is ragged -- no shape
        // history on the stream, or BMQCRC_F_PLAN after a closed-form batch
        // (segment counts seen on the host decide for host batches): the
        // light k_plan (counts and closed forms, no size-class map).  A
        // ragged batch is then folded by searching seg_first, and k_fold
        // records its shape, so the stream's next batch gets the map
        // (planned steps: 1M x 256 B 0.055 against 0.066 ms, 1k x 4 KiB 0.013
        // against 0.017; a ragged first batch 1.09x: Zipf 4.45 against 4.07;
        // profiles/r05/ab/light_planner.jsonl; TUNE bit 12 restores round 4)
        a.map_planned = 0;
    }
    if ((kTuneBits & 2048u) && !a.whole && (flags & BMQCRC_F_PLAN) &&
        spec_eligible(c, n, a.blocks_per_cu)) {
        // A/B only (TUNE bit 11): a batch with no shape history launched as
        // the speculative one-segment kernel instead of being planned (its
        // second pass folds the longer messages); bench.py's planned leg
        // then prices that choice
        a.spec = 1;
    } else if (!a.whole && host_max_len <= a.seg_bytes && !(flags & BMQCRC_F_PLAN)) {
        a.spec = 1;  // known, not guessed: every message is one segment
    } else if (!a.whole && host_min_len > 0 && host_max_len != UINT64_MAX &&
               !(flags & BMQCRC_F_PLAN)) {
        // every length in [min, max] has the same u segments, u dividing 64:
        // the speculative uniform launch, known instead of guessed
        const uint64_t u = (host_max_len - 1) / a.seg_bytes + 1;
        if ((host_min_len - 1) / a.seg_bytes + 1 == u && u >= 2 && u <= 64 && 64 % u == 0 &&
            (uint64_t)n * u <= 0xFFFFFF00ull) {
            a.spec = (uint32_t)u;
        }
    }
    if (!a.whole && !a.spec && a.map_planned && w->hint_host && w->map_wait_ticks != 0) {
        // (a zero limit is the test hook that gives every map up: no switch)
        // a map given up since the last look (k_fold's sticky epoch word):
        // the GPU is shared with other streams or processes, whose resident
        // kernels keep k_plan_map's blocks from meeting, so the next
        // kPairAfterVoid ragged batches here are planned by the pair, which
        // needs no co-residency (Zipf 4M: ~76 against ~54 us)
        const uint32_t voided = __atomic_load_n(w->hint_host + 1, __ATOMIC_RELAXED);
        if (voided != w->void_seen) {
            w->void_seen = voided;
            w->pair_left = kPairAfterVoid;
        }
        if (w->pair_left) {
            a.pair = 1;
            --w->pair_left;
        }
    }
    if (!a.whole && !a.spec && a.map_planned) {
        // inside a graph capture every replay must tag its planner words
        // afresh: the tag then lives on the device (BatchArgs::plan_epoch 0)
        if (capturing) {
            a.plan_epoch = 0;
        }
    }
    a.arena = (const uint8_t*)arena;
    a.offsets = offsets;
    a.lengths = lengths;
    a.seeds = seeds;
    a.out = out;
    void* ev0 = nullptr;
    void* ev1 = nullptr;
    if (flags & BMQCRC_F_TIME_KERNEL) {
        std::pair<hipEvent_t, hipEvent_t> ev;
        if (!w->spare.empty()) {
            ev = w->spare.back();
            w->spare.pop_back();
        } else {
            HIP_TRY(hipEventCreate(&ev.first));
            HIP_TRY(hipEventCreate(&ev.second));
        }
        w->timing.push_back(ev);
        ev0 = (void*)ev.first;
        ev1 = (void*)ev.second;
    }
    if (bmqcrc_launch_batch(&a, (void*)c.s, c.st->num_cus, ev0, ev1) != 0) {
        return fail(BMQCRC_EIO, std::string("kernel launch failed: ") +
                                    hipGetErrorString(hipGetLastError()));
    }
    w->last_spec = a.whole ? 1u : a.spec;
    w->last_seg = a.seg_bytes;
    w->last_kernels = n == 0                 ? 0u
                      : (a.whole || a.spec)  ? 1u
                      : !a.map_planned       ? 2u
                      : single_pass_planner(a) ? 2u
                                             : 3u;
    w->last_map = n != 0 && !a.whole && !a.spec && a.map_planned ? 1u : 0u;
    return 0;
}

// Stage host arrays into workspace buffers (async on c.s).
int stage(Ctx& c, DevBuf& buf, const void* host, uint64_t bytes)
{
    int rc = buf.ensure(bytes + 16);
    if (rc) {
        return rc;
    }
    if (bytes) {
        HIP_TRY(hipMemcpyAsync(buf.p, host, bytes, hipMemcpyHostToDevice, c.s));
    }
    return 0;
}

// declared_max / declared_min: the caller's bounds on every length of a
// device-resident batch (bmqcrc_opts.max_len / min_len, 0 = none); host
// batches use the lengths they hold.
int batch_one(int dev, void* user_stream, uint32_t flags, uint32_t seg, const void* arena,
              uint64_t arena_bytes, const uint64_t* offsets, const uint32_t* lengths,
              const uint32_t* seeds, uint32_t* out, uint64_t n, uint32_t declared_max = 0,
              uint32_t declared_min = 0)
{
    Ctx c;
    int rc = open_ctx(dev, user_stream, &c);
    if (rc) {
        return rc;
    }
    Workspace* w = c.w;
    std::lock_guard<std::mutex> g(w->mu);
    const bool dev_ptrs = (flags & BMQCRC_F_DEVICE_PTRS) != 0;
    if (dev_ptrs) {
        if ((rc = run_batch(c, flags, seg, arena, arena_bytes, offsets, lengths, seeds, out, n,
                            declared_max ? (uint64_t)declared_max : UINT64_MAX,
                            declared_max ? std::min(declared_min, declared_max) : 0u))) {
            return rc;
        }
        if (!(flags & BMQCRC_F_ASYNC)) {
            HIP_TRY(hipStreamSynchronize(c.s));
        }
        return 0;
    }
    if ((rc = stage(c, w->arena, arena, arena_bytes)) ||
        (rc = stage(c, w->offsets, offsets, 8 * n)) || (rc = stage(c, w->lengths, lengths, 4 * n)) ||
        (seeds && (rc = stage(c, w->seeds, seeds, 4 * n))) || (rc = w->out.ensure(4 * n))) {
        return rc;
    }
    if ((rc = run_batch(c, flags, seg, w->arena.p, arena_bytes, (const uint64_t*)w->offsets.p,
                        (const uint32_t*)w->lengths.p,
                        seeds ? (const uint32_t*)w->seeds.p : nullptr, (uint32_t*)w->out.p, n,
                        max_length(lengths, n), min_length(lengths, n)))) {
        return rc;
    }
    HIP_TRY(hipMemcpyAsync(out, w->out.p, 4 * n, hipMemcpyDeviceToHost, c.s));
    HIP_TRY(hipStreamSynchronize(c.s));
    return 0;
}

int parse_opts(const bmqcrc_opts* opts, bmqcrc_opts* o, uint32_t* seg, int* dev)
{
    memset(o, 0, sizeof(*o));
    o->device = -1;
    if (opts) {
        // struct_size 0 reads only the ABI 2.0 fields: a caller that never set
        // it may be built against any earlier, shorter layout
        // (ABI 2.7: nothing past offsetof(ndevices) is read then, not even to
        // check it -- a 2.0 caller's struct ends there)
        const size_t given = opts->struct_size ? opts->struct_size : offsetof(bmqcrc_opts, ndevices);
        memcpy(o, opts, std::min<size_t>(sizeof(*o), given));
        o->struct_size = sizeof(*o);
    }
    *seg = o->seg_bytes;
    const uint32_t known = BMQCRC_F_DEVICE_PTRS | BMQCRC_F_ASYNC | BMQCRC_F_TIME_KERNEL |
                           BMQCRC_F_WHOLE_MESSAGES | BMQCRC_F_PLAN;
    if (o->flags & ~known) {
        return fail(BMQCRC_EINVAL, "unknown bmqcrc_opts.flags bits");
    }
    int rc;
    if ((rc = check_seg(seg)) || (rc = resolve_device(o->device, dev))) {
        return rc;
    }
    return 0;
}

int check_ranges(const uint64_t* offsets, const uint32_t* lengths, uint64_t n,
                 uint64_t arena_bytes)
{
    for (uint64_t i = 0; i < n; ++i) {
        if (offsets[i] > arena_bytes || lengths[i] > arena_bytes - offsets[i]) {
            return fail(BMQCRC_EINVAL,
                        "message " + std::to_string(i) + " lies outside [arena, arena+arena_bytes)");
        }
    }
    return 0;
}

// Device mismatch-index list of a verify: 4 Mi entries (16 MiB) at most.
constexpr uint64_t kVerifyListCap = 1ull << 22;

int verify_locked(Ctx& c, Workspace* w, const bmqcrc_opts& o, uint32_t seg, bool arena_staged,
                  const void* arena, uint64_t arena_bytes, const uint64_t* offsets,
                  const uint32_t* lengths, const uint32_t* expected, uint64_t n, uint64_t* n_bad,
                  uint64_t* bad_idx, uint64_t bad_cap, uint64_t* n_written);

int verify_host_multi(const void* arena, uint64_t arena_bytes, bmqcrc_prepare_fn prepare,
                      void* pctx, uint64_t* n_bad, std::vector<uint64_t>* bad, uint64_t bad_cap,
                      const bmqcrc_opts& o, uint32_t seg, std::vector<uint32_t>* crcs,
                      uint64_t* n_written);

// The message arrays of a plain verify call, handed to verify_host_multi as
// an already finished "walk".
struct GivenArrays {
    const uint64_t* off;
    const uint32_t* len;
    const uint32_t* exp;
    uint64_t n;
};

int given_arrays(void* ctx, const uint64_t** off, const uint32_t** len, const uint32_t** exp,
                 uint64_t* n)
{
    const GivenArrays* g = (const GivenArrays*)ctx;
    *off = g->off;
    *len = g->len;
    *exp = g->exp;
    *n = g->n;
    return 0;
}

}  // namespace

extern "C" int bmqcrc_set_error(int rc, const char* msg)
{
    return fail(rc, msg ? msg : "");
}

extern "C" void bmqcrc_clear_error(void)
{
    t_err.clear();
}

extern "C" {

// bmqcrc_crc32c, bmqcrc_crc32c_blob and bmqcrc_combine: crc32c_cpu.cpp

int bmqcrc_crc32c_batch(const void* arena, uint64_t arena_bytes, const uint64_t* offsets,
                        const uint32_t* lengths, const uint32_t* seeds, uint32_t* out,
                        uint64_t n, const bmqcrc_opts* opts)
{
    t_err.clear();
    DeviceGuard keep_device;
    if (n == 0) {
        return 0;
    }
    if (!offsets || !lengths || !out || (!arena && arena_bytes)) {
        return fail(BMQCRC_EINVAL, "null pointer argument");
    }
    if (n > 0xFFFFFFFFull) {
        return fail(BMQCRC_EINVAL, "at most 2^32-1 messages per batch");
    }
    bmqcrc_opts o;
    uint32_t seg;
    int dev, rc;
    if ((rc = parse_opts(opts, &o, &seg, &dev))) {
        return rc;
    }
    if (!(o.flags & BMQCRC_F_DEVICE_PTRS) && (rc = check_ranges(offsets, lengths, n, arena_bytes))) {
        return rc;  // device arrays are trusted
    }
    if (!(o.flags & BMQCRC_F_DEVICE_PTRS) && o.ndevices > 1) {  // one byte range per device
        return bmqcrc_crc32c_batch_multi(arena, arena_bytes, offsets, lengths, seeds, out, n,
                                         o.devices, (int)o.ndevices, seg);
    }
    return batch_one(dev, o.stream, o.flags, seg, arena, arena_bytes, offsets, lengths, seeds,
                     out, n, (o.flags & BMQCRC_F_DEVICE_PTRS) ? o.max_len : 0u,
                     (o.flags & BMQCRC_F_DEVICE_PTRS) ? o.min_len : 0u);
}

int bmqcrc_crc32c_verify(const void* arena, uint64_t arena_bytes, const uint64_t* offsets,
                         const uint32_t* lengths, const uint32_t* expected, uint64_t n,
                         uint64_t* n_bad, uint64_t* bad_idx, uint64_t bad_cap,
                         const bmqcrc_opts* opts)
{
    t_err.clear();
    DeviceGuard keep_device;
    if (!n_bad) {
        return fail(BMQCRC_EINVAL, "n_bad is required");
    }
    *n_bad = 0;
    if (n == 0) {
        return 0;
    }
    if (!offsets || !lengths || !expected || (!arena && arena_bytes) || (bad_cap && !bad_idx)) {
        return fail(BMQCRC_EINVAL, "null pointer argument");
    }
    if (n > 0xFFFFFFFFull) {
        return fail(BMQCRC_EINVAL, "at most 2^32-1 messages per batch");
    }
    bmqcrc_opts o;
    uint32_t seg;
    int dev, rc;
    if ((rc = parse_opts(opts, &o, &seg, &dev))) {
        return rc;
    }
    const bool dev_ptrs = (o.flags & BMQCRC_F_DEVICE_PTRS) != 0;
    if (!dev_ptrs && (rc = check_ranges(offsets, lengths, n, arena_bytes))) {
        return rc;
    }
    if (!dev_ptrs && o.ndevices > 1) {  // one byte range per device, merged in index order
        GivenArrays ga = {offsets, lengths, expected, n};
        std::vector<uint64_t> bad;
        uint64_t written = 0;
        if ((rc = verify_host_multi(arena, arena_bytes, given_arrays, &ga, n_bad, &bad, bad_cap, o,
                                    seg, nullptr, &written))) {
            return rc;
        }
        std::copy(bad.begin(), bad.begin() + written, bad_idx);
        return 0;
    }
    Ctx c;
    if ((rc = open_ctx(dev, o.stream, &c))) {
        return rc;
    }
    Workspace* w = c.w;
    std::lock_guard<std::mutex> g(w->mu);
    return verify_locked(c, w, o, seg, false, arena, arena_bytes, offsets, lengths, expected, n,
                         n_bad, bad_idx, bad_cap, nullptr);
}

}  // extern "C"

namespace {

// The verify pipeline after the workspace lock: stage (host buffers; the
// arena may already be staged), fold, compare on the device, collect the
// lowest mismatching indices.
int verify_locked(Ctx& c, Workspace* w, const bmqcrc_opts& o, uint32_t seg, bool arena_staged,
                  const void* arena, uint64_t arena_bytes, const uint64_t* offsets,
                  const uint32_t* lengths, const uint32_t* expected, uint64_t n, uint64_t* n_bad,
                  uint64_t* bad_idx, uint64_t bad_cap, uint64_t* n_written)
{
    int rc;
    const bool dev_ptrs = (o.flags & BMQCRC_F_DEVICE_PTRS) != 0;
    // The device list holds at most kVerifyListCap indices (16 MiB), whatever
    // bad_cap is; a longer answer is taken in windows of that size, so exactly
    // min(n_bad, bad_cap) indices are still written.
    const uint64_t want = std::min<uint64_t>(bad_cap, n);
    const uint32_t cap = (uint32_t)std::min<uint64_t>(want, kVerifyListCap);
    if (n_written) {
        *n_written = 0;
    }
    if ((rc = w->out.ensure(4 * n)) || (rc = w->vcount.ensure(4)) ||
        (rc = w->vidx.ensure(4ull * std::max<uint32_t>(cap, 1)))) {
        return rc;
    }
    const void* d_arena = arena;
    const uint64_t* d_off = offsets;
    const uint32_t* d_len = lengths;
    const uint32_t* d_exp = expected;
    if (!dev_ptrs) {
        if ((!arena_staged && (rc = stage(c, w->arena, arena, arena_bytes))) ||
            (rc = stage(c, w->offsets, offsets, 8 * n)) ||
            (rc = stage(c, w->lengths, lengths, 4 * n)) ||
            (rc = stage(c, w->expected, expected, 4 * n))) {
            return rc;
        }
        d_arena = w->arena.p;
        d_off = (const uint64_t*)w->offsets.p;
        d_len = (const uint32_t*)w->lengths.p;
        d_exp = (const uint32_t*)w->expected.p;
    }
    if ((rc = run_batch(c, o.flags, seg, d_arena, arena_bytes, d_off, d_len, nullptr,
                        (uint32_t*)w->out.p, n,
                        dev_ptrs ? UINT64_MAX : max_length(lengths, n)))) {
        return rc;
    }
    HIP_TRY(hipMemsetAsync(w->vcount.p, 0, 4, c.s));
    if (bmqcrc_launch_compare((const uint32_t*)w->out.p, d_exp, n, (uint32_t*)w->vcount.p,
                              (uint32_t*)w->vidx.p, cap, (void*)c.s)) {
        return fail(BMQCRC_EIO, "compare launch failed");
    }
    uint32_t cnt = 0;
    HIP_TRY(hipMemcpyAsync(&cnt, w->vcount.p, 4, hipMemcpyDeviceToHost, c.s));
    HIP_TRY(hipStreamSynchronize(c.s));
    *n_bad = cnt;
    const uint64_t take = std::min<uint64_t>(cnt, want);
    if (take && cnt <= cap) {
        // the single pass kept every mismatch: sort the short list
        std::vector<uint32_t> idx(take);
        HIP_TRY(hipMemcpyAsync(idx.data(), w->vidx.p, 4ull * take, hipMemcpyDeviceToHost, c.s));
        HIP_TRY(hipStreamSynchronize(c.s));
        std::sort(idx.begin(), idx.end());
        for (uint64_t k = 0; k < take; ++k) {
            bad_idx[k] = idx[k];
        }
    } else if (take) {
        // more mismatches than device slots: the single pass kept an arbitrary
        // subset, so rebuild the list in index order, one window at a time
        const uint32_t nb = (uint32_t)std::min<uint64_t>((n + 255) / 256, 4096);
        if ((rc = w->vblock.ensure(4ull * nb))) {
            return rc;
        }
        uint32_t* d_blk = (uint32_t*)w->vblock.p;
        if (bmqcrc_launch_compare_ordered((const uint32_t*)w->out.p, d_exp, n, d_blk, nb,
                                          nullptr, 0, cap, 0, (void*)c.s)) {
            return fail(BMQCRC_EIO, "ordered compare launch failed");
        }
        std::vector<uint32_t> blk(nb);
        HIP_TRY(hipMemcpyAsync(blk.data(), d_blk, 4ull * nb, hipMemcpyDeviceToHost, c.s));
        HIP_TRY(hipStreamSynchronize(c.s));
        uint64_t run = 0;
        for (uint32_t b = 0; b < nb; ++b) {
            const uint32_t k = blk[b];
            blk[b] = (uint32_t)std::min<uint64_t>(run, 0xFFFFFFFFu);
            run += k;
        }
        HIP_TRY(hipMemcpyAsync(d_blk, blk.data(), 4ull * nb, hipMemcpyHostToDevice, c.s));
        std::vector<uint32_t> idx(cap);
        for (uint64_t skip = 0; skip < take; skip += cap) {
            const uint32_t m = (uint32_t)std::min<uint64_t>(cap, take - skip);
            if (bmqcrc_launch_compare_ordered((const uint32_t*)w->out.p, d_exp, n, d_blk, nb,
                                              (uint32_t*)w->vidx.p, (uint32_t)skip, m, 1,
                                              (void*)c.s)) {
                return fail(BMQCRC_EIO, "ordered compare launch failed");
            }
            HIP_TRY(hipMemcpyAsync(idx.data(), w->vidx.p, 4ull * m, hipMemcpyDeviceToHost, c.s));
            HIP_TRY(hipStreamSynchronize(c.s));  // also: blk is read by the async H2D copy
            for (uint32_t k = 0; k < m; ++k) {
                bad_idx[skip + k] = idx[k];
            }
        }
    }
    if (n_written) {
        *n_written = take;
    }
    return 0;
}

// Library-owned stream k of a device (a device listed twice in
// bmqcrc_opts.devices gets two streams, hence two workspaces).
int internal_stream(int dev, int k, hipStream_t* out)
{
    static std::map<std::pair<int, int>, hipStream_t> streams;
    std::lock_guard<std::mutex> g(g_mu);
    hipStream_t& s = streams[std::make_pair(dev, k)];
    if (!s) {
        HIP_TRY(hipSetDevice(dev));
        HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    }
    *out = s;
    return 0;
}

// bmqcrc_verify_host_overlapped over several devices (bmqcrc_opts.ndevices >
// 1): the arena is cut into ndevices contiguous byte ranges; one thread per
// range copies it to its device over that device's PCIe link while the
// calling thread walks the format, then verifies (or computes) the messages
// lying wholly inside its range.  The few messages that straddle a cut are
// gathered into a small arena and done by the first range's thread
// afterwards.  Results are merged in message order: n_bad is the sum, `bad`
// the lowest min(n_bad, bad_cap) indices overall.
int verify_host_multi(const void* arena, uint64_t arena_bytes, bmqcrc_prepare_fn prepare,
                      void* pctx, uint64_t* n_bad, std::vector<uint64_t>* bad, uint64_t bad_cap,
                      const bmqcrc_opts& o, uint32_t seg, std::vector<uint32_t>* crcs,
                      uint64_t* n_written)
{
    const uint32_t nd = o.ndevices;
    if (nd > 64) {
        return fail(BMQCRC_EINVAL, "at most 64 device listings");
    }
    const int have = device_count_raw();
    std::vector<int> devs(nd);
    for (uint32_t d = 0; d < nd; ++d) {
        devs[d] = o.devices ? o.devices[d] : (int)d;
        if (devs[d] < 0 || (have > 0 && devs[d] >= have)) {
            return fail(BMQCRC_EINVAL, "device ordinal out of range");
        }
    }
    const uint64_t* off = nullptr;
    const uint32_t* len = nullptr;
    const uint32_t* exp = nullptr;
    uint64_t n = 0;
    if (have <= 0) {
        // no usable device: a malformed input is still reported first
        const int prc = prepare(pctx, &off, &len, &exp, &n);
        if (prc || n == 0) {
            return prc;
        }
        return fail(BMQCRC_ENODEV, "no HIP device available (batch CRC32C runs only on the GPU)");
    }
    std::vector<uint64_t> cut(nd + 1, arena_bytes);
    cut[0] = 0;
    for (uint32_t d = 1; d < nd; ++d) {
        cut[d] = (arena_bytes / nd * d) & ~127ull;
    }
    std::vector<int> rcs(nd, 0);
    std::vector<std::string> errs(nd);
    std::vector<uint64_t> nb(nd, 0);
    std::vector<std::vector<uint64_t>> bads(nd);
    std::vector<uint32_t> owner;  // per message: its range, or nd (straddles a cut)
    std::mutex mu;
    std::condition_variable cv;
    bool walked = false, walk_ok = false;
    auto slice = [&](uint32_t t) {
        const int dev = devs[t];
        hipStream_t st = nullptr;
        Ctx c;
        int rc = internal_stream(dev, (int)t, &st);
        if (!rc) {
            rc = open_ctx(dev, (void*)st, &c);
        }
        std::unique_lock<std::mutex> lk;
        if (!rc) {
            lk = std::unique_lock<std::mutex>(c.w->mu);
            rc = stage(c, c.w->arena, (const uint8_t*)arena + cut[t], cut[t + 1] - cut[t]);
        }
        if (!rc && hipStreamSynchronize(c.s) != hipSuccess) {
            rc = fail(BMQCRC_EIO, "staging the arena range failed");
        }
        {
            std::unique_lock<std::mutex> wl(mu);
            cv.wait(wl, [&] { return walked; });
        }
        if (rc || !walk_ok) {
            rcs[t] = rc;
            errs[t] = t_err;
            return;
        }
        // this range's messages (and, for range 0, then the straddlers)
        for (uint32_t pass = 0; pass < (t == 0 ? 2u : 1u) && !rc; ++pass) {
            const uint32_t want = pass == 0 ? t : nd;
            std::vector<uint64_t> gi, lo;
            std::vector<uint32_t> ll, le;
            std::vector<uint8_t> packed;
            for (uint64_t i = 0; i < n; ++i) {
                if (owner[i] != want) {
                    continue;
                }
                gi.push_back(i);
                ll.push_back(len[i]);
                le.push_back(exp ? exp[i] : 0u);
                if (pass == 0) {
                    lo.push_back(off[i] - cut[t]);
                } else {
                    lo.push_back(packed.size());
                    packed.insert(packed.end(), (const uint8_t*)arena + off[i],
                                  (const uint8_t*)arena + off[i] + len[i]);
                }
            }
            if (gi.empty()) {
                continue;
            }
            const uint64_t m = gi.size();
            const bool staged = pass == 0;
            const void* abase = staged ? (const void*)((const uint8_t*)arena + cut[t])
                                       : (const void*)packed.data();
            const uint64_t abytes = staged ? cut[t + 1] - cut[t] : packed.size();
            if (crcs) {
                std::vector<uint32_t> part(m);
                if ((!staged && (rc = stage(c, c.w->arena, abase, abytes))) ||
                    (rc = stage(c, c.w->offsets, lo.data(), 8 * m)) ||
                    (rc = stage(c, c.w->lengths, ll.data(), 4 * m)) ||
                    (rc = c.w->out.ensure(4 * m)) ||
                    (rc = run_batch(c, o.flags, seg, c.w->arena.p, abytes,
                                    (const uint64_t*)c.w->offsets.p,
                                    (const uint32_t*)c.w->lengths.p, nullptr,
                                    (uint32_t*)c.w->out.p, m, max_length(ll.data(), m)))) {
                    break;
                }
                if (hipMemcpyAsync(part.data(), c.w->out.p, 4 * m, hipMemcpyDeviceToHost, c.s) !=
                        hipSuccess ||
                    hipStreamSynchronize(c.s) != hipSuccess) {
                    rc = fail(BMQCRC_EIO, "copying the CRCs back failed");
                    break;
                }
                for (uint64_t k = 0; k < m; ++k) {
                    (*crcs)[gi[k]] = part[k];
                }
                continue;
            }
            uint64_t nbad = 0, nw = 0;
            std::vector<uint64_t> lb(std::min<uint64_t>(bad_cap, m));
            if ((rc = verify_locked(c, c.w, o, seg, staged, abase, abytes, lo.data(), ll.data(),
                                    le.data(), m, &nbad, lb.data(), lb.size(), &nw))) {
                break;
            }
            nb[t] += nbad;
            for (uint64_t k = 0; k < nw; ++k) {
                bads[t].push_back(gi[lb[k]]);
            }
        }
        rcs[t] = rc;
        errs[t] = t_err;
    };
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < nd; ++t) {
        th.emplace_back(slice, t);
    }
    const int prc = prepare(pctx, &off, &len, &exp, &n);
    int rc = prc;
    if (!rc && n > 0xFFFFFFFFull) {
        rc = fail(BMQCRC_EINVAL, "at most 2^32-1 messages per batch");
    }
    if (!rc) {
        rc = check_ranges(off, len, n, arena_bytes);
    }
    if (!rc) {
        owner.resize(n);
        for (uint64_t i = 0; i < n; ++i) {
            uint32_t t = (uint32_t)(std::upper_bound(cut.begin(), cut.end(), off[i]) - cut.begin());
            t = std::min(t == 0 ? 0u : t - 1u, nd - 1);
            owner[i] = off[i] + len[i] <= cut[t + 1] ? t : nd;
        }
        if (crcs) {
            crcs->assign(n, 0);
        }
    }
    const std::string walk_err = t_err;
    {
        std::lock_guard<std::mutex> wl(mu);
        walked = true;
        walk_ok = rc == 0;
    }
    cv.notify_all();
    for (auto& t : th) {
        t.join();
    }
    if (rc) {  // the walk's error (malformed input) takes precedence
        t_err = walk_err;
        return rc;
    }
    for (uint32_t t = 0; t < nd; ++t) {
        if (rcs[t]) {
            return fail(rcs[t], "device " + std::to_string(devs[t]) + ": " + errs[t]);
        }
    }
    if (crcs) {
        return 0;
    }
    uint64_t total_bad = 0;
    std::vector<uint64_t> all;
    for (uint32_t t = 0; t < nd; ++t) {
        total_bad += nb[t];
        all.insert(all.end(), bads[t].begin(), bads[t].end());
    }
    std::sort(all.begin(), all.end());
    const uint64_t take = std::min<uint64_t>(all.size(), bad_cap);
    bad->assign(std::min(bad_cap, n), 0);
    std::copy(all.begin(), all.begin() + take, bad->begin());
    *n_bad = total_bad;
    if (n_written) {
        *n_written = take;
    }
    return 0;
}

}  // namespace

int bmqcrc_verify_host_overlapped(const void* arena, uint64_t arena_bytes,
                                  bmqcrc_prepare_fn prepare, void* pctx, uint64_t* n_bad,
                                  std::vector<uint64_t>* bad, uint64_t bad_cap,
                                  const bmqcrc_opts* opts, std::vector<uint32_t>* crcs,
                                  uint64_t* n_written)
{
    if (n_written) {
        *n_written = 0;
    }
    t_err.clear();
    DeviceGuard keep_device;
    if (!prepare || (!crcs && (!n_bad || !bad)) || (!arena && arena_bytes)) {
        return fail(BMQCRC_EINVAL, "null pointer argument");
    }
    if (n_bad) {
        *n_bad = 0;
    }
    bmqcrc_opts o;
    uint32_t seg;
    int dev = 0, rc;
    const uint64_t* off = nullptr;
    const uint32_t* len = nullptr;
    const uint32_t* exp = nullptr;
    uint64_t n = 0;
    rc = parse_opts(opts, &o, &seg, &dev);
    if (rc && rc != BMQCRC_ENODEV) {
        return rc;
    }
    if (o.flags & (BMQCRC_F_DEVICE_PTRS | BMQCRC_F_ASYNC)) {
        return fail(BMQCRC_EINVAL, "overlapped verify takes host buffers, synchronously");
    }
    if (o.ndevices > 1) {
        return verify_host_multi(arena, arena_bytes, prepare, pctx, n_bad, bad, bad_cap, o, seg,
                                 crcs, n_written);
    }
    Ctx c;
    if (rc || (rc = open_ctx(dev, o.stream, &c))) {
        // no usable device: a malformed input is still reported first
        const std::string why = t_err;
        const int prc = prepare(pctx, &off, &len, &exp, &n);
        if (prc || n == 0) {  // nothing to verify needs no device
            return prc;
        }
        return fail(rc, why);
    }
    Workspace* w = c.w;
    std::lock_guard<std::mutex> g(w->mu);
    // The arena's H2D copy runs on a helper thread while the caller's walk
    // produces the descriptors on this one (its errors stay in this thread's
    // bmqcrc_last_error).
    int src = 0;
    std::thread copier([&] {
        if (hipSetDevice(dev) != hipSuccess) {
            src = BMQCRC_EIO;
            return;
        }
        src = stage(c, w->arena, arena, arena_bytes);
        if (!src && hipStreamSynchronize(c.s) != hipSuccess) {
            src = BMQCRC_EIO;
        }
    });
    const int prc = prepare(pctx, &off, &len, &exp, &n);
    copier.join();
    if (prc) {
        return prc;
    }
    if (src) {
        return fail(src, "staging the arena to the device failed");
    }
    if (n == 0) {
        return 0;
    }
    if (n > 0xFFFFFFFFull) {
        return fail(BMQCRC_EINVAL, "at most 2^32-1 messages per batch");
    }
    if ((rc = check_ranges(off, len, n, arena_bytes))) {
        return rc;
    }
    if (crcs) {  // compute: stage the descriptors, fold, copy the CRCs back
        crcs->assign(n, 0);
        if ((rc = stage(c, w->offsets, off, 8 * n)) || (rc = stage(c, w->lengths, len, 4 * n)) ||
            (rc = w->out.ensure(4 * n))) {
            return rc;
        }
        if ((rc = run_batch(c, o.flags, seg, w->arena.p, arena_bytes,
                            (const uint64_t*)w->offsets.p, (const uint32_t*)w->lengths.p, nullptr,
                            (uint32_t*)w->out.p, n, max_length(len, n)))) {
            return rc;
        }
        HIP_TRY(hipMemcpyAsync(crcs->data(), w->out.p, 4 * n, hipMemcpyDeviceToHost, c.s));
        HIP_TRY(hipStreamSynchronize(c.s));
        return 0;
    }
    bad->assign(std::min<uint64_t>(bad_cap, n), 0);
    return verify_locked(c, w, o, seg, true, arena, arena_bytes, off, len, exp, n, n_bad,
                         bad->data(), bad->size(), n_written);
}

extern "C" {

int bmqcrc_crc32c_blobs(const void* arena, uint64_t arena_bytes, const uint64_t* buf_offsets,
                        const uint32_t* buf_lengths, uint64_t nbuf,
                        const uint64_t* msg_first_buf, const uint32_t* seeds, uint32_t* out,
                        uint64_t n, const bmqcrc_opts* opts)
{
    t_err.clear();
    DeviceGuard keep_device;
    if (n == 0) {
        return 0;
    }
    if (!msg_first_buf || !out || (nbuf && (!buf_offsets || !buf_lengths)) ||
        (!arena && arena_bytes)) {
        return fail(BMQCRC_EINVAL, "null pointer argument");
    }
    if (nbuf > 0xFFFFFFFFull || n > 0xFFFFFFFFull) {
        return fail(BMQCRC_EINVAL, "at most 2^32-1 buffers and blobs per call");
    }
    bmqcrc_opts o;
    uint32_t seg;
    int dev, rc;
    if ((rc = parse_opts(opts, &o, &seg, &dev))) {
        return rc;
    }
    const bool dev_ptrs = (o.flags & BMQCRC_F_DEVICE_PTRS) != 0;
    if (!dev_ptrs) {
        if ((rc = check_ranges(buf_offsets, buf_lengths, nbuf, arena_bytes))) {
            return rc;
        }
        for (uint64_t m = 0; m < n; ++m) {
            if (msg_first_buf[m] > msg_first_buf[m + 1] || msg_first_buf[m + 1] > nbuf) {
                return fail(BMQCRC_EINVAL, "msg_first_buf must be non-decreasing and <= nbuf");
            }
        }
    }
    Ctx c;
    if ((rc = open_ctx(dev, o.stream, &c))) {
        return rc;
    }
    Workspace* w = c.w;
    std::lock_guard<std::mutex> g(w->mu);
    if ((rc = w->buf_crc.ensure(4 * std::max<uint64_t>(nbuf, 1)))) {
        return rc;
    }
    const void* d_arena = arena;
    const uint64_t* d_off = buf_offsets;
    const uint32_t* d_len = buf_lengths;
    const uint64_t* d_first = msg_first_buf;
    const uint32_t* d_seeds = seeds;
    uint32_t* d_out = out;
    if (!dev_ptrs) {
        if ((rc = stage(c, w->arena, arena, arena_bytes)) ||
            (rc = stage(c, w->offsets, buf_offsets, 8 * nbuf)) ||
            (rc = stage(c, w->lengths, buf_lengths, 4 * nbuf)) ||
            (rc = stage(c, w->first_buf, msg_first_buf, 8 * (n + 1))) ||
            (seeds && (rc = stage(c, w->seeds, seeds, 4 * n))) || (rc = w->out.ensure(4 * n))) {
            return rc;
        }
        d_arena = w->arena.p;
        d_off = (const uint64_t*)w->offsets.p;
        d_len = (const uint32_t*)w->lengths.p;
        d_first = (const uint64_t*)w->first_buf.p;
        d_seeds = seeds ? (const uint32_t*)w->seeds.p : nullptr;
        d_out = (uint32_t*)w->out.p;
    }
    if (nbuf && (rc = run_batch(c, o.flags, seg, d_arena, arena_bytes, d_off, d_len, nullptr,
                                (uint32_t*)w->buf_crc.p, nbuf,
                                dev_ptrs ? UINT64_MAX : max_length(buf_lengths, nbuf)))) {
        return rc;
    }
    if (bmqcrc_launch_blob_combine((const uint32_t*)w->buf_crc.p, d_len, d_first, d_seeds, d_out,
                                   n, (void*)c.s)) {
        return fail(BMQCRC_EIO, "blob combine launch failed");
    }
    if (!dev_ptrs) {
        HIP_TRY(hipMemcpyAsync(out, d_out, 4 * n, hipMemcpyDeviceToHost, c.s));
        HIP_TRY(hipStreamSynchronize(c.s));
    } else if (!(o.flags & BMQCRC_F_ASYNC)) {
        HIP_TRY(hipStreamSynchronize(c.s));
    }
    return 0;
}

// Scattered host buffers (a bdlbb::Blob's data buffers) -> one contiguous
// device arena, through the workspace's pinned ring: kGatherThreads host
// threads each copy their chunks into pinned slots and enqueue the slot's H2D
// copy at once, so gathering chunk k+1 overlaps the PCIe transfer of chunk k
// (no pageable staging copy, no second host copy).  Message m is then the
// contiguous range of its buffers and the whole batch is one fold launch.
constexpr uint64_t kGatherChunk = 4ull << 20;
constexpr int kGatherSlots = 16;
constexpr int kGatherThreads = 8;

int bmqcrc_crc32c_gather(const void* const* bufs, const uint32_t* buf_lengths, uint64_t nbuf,
                         const uint64_t* msg_first_buf, const uint32_t* seeds, uint32_t* out,
                         uint64_t n, const bmqcrc_opts* opts)
{
    t_err.clear();
    DeviceGuard keep_device;
    if (n == 0) {
        return 0;
    }
    if (!msg_first_buf || !out || (nbuf && (!bufs || !buf_lengths))) {
        return fail(BMQCRC_EINVAL, "null pointer argument");
    }
    if (nbuf > 0xFFFFFFFFull || n > 0xFFFFFFFFull) {
        return fail(BMQCRC_EINVAL, "at most 2^32-1 buffers and messages per call");
    }
    for (uint64_t m = 0; m < n; ++m) {
        if (msg_first_buf[m] > msg_first_buf[m + 1] || msg_first_buf[m + 1] > nbuf) {
            return fail(BMQCRC_EINVAL, "msg_first_buf must be non-decreasing and <= nbuf");
        }
    }
    // Arena layout: buffers [b0, b1) back to back, in order.
    const uint64_t b0 = msg_first_buf[0], b1 = msg_first_buf[n];
    std::vector<uint64_t> boff(b1 - b0 + 1, 0);
    for (uint64_t b = b0; b < b1; ++b) {
        if (buf_lengths[b] && !bufs[b]) {
            return fail(BMQCRC_EINVAL, "buffer " + std::to_string(b) + " is NULL with a length");
        }
        boff[b - b0 + 1] = boff[b - b0] + buf_lengths[b];
    }
    const uint64_t total = boff.back();
    std::vector<uint64_t> moff(n);
    std::vector<uint32_t> mlen(n);
    uint64_t maxlen = 0;
    for (uint64_t m = 0; m < n; ++m) {
        moff[m] = boff[msg_first_buf[m] - b0];
        const uint64_t len = boff[msg_first_buf[m + 1] - b0] - moff[m];
        if (len > 0xFFFFFFFFull) {
            return fail(BMQCRC_EINVAL, "message " + std::to_string(m) + " is longer than 2^32-1");
        }
        mlen[m] = (uint32_t)len;
        maxlen = std::max(maxlen, len);
    }
    // argument errors above are reported before a missing device
    bmqcrc_opts o;
    uint32_t seg;
    int dev, rc;
    if ((rc = parse_opts(opts, &o, &seg, &dev))) {
        return rc;
    }
    if (o.flags & (BMQCRC_F_DEVICE_PTRS | BMQCRC_F_ASYNC)) {
        return fail(BMQCRC_EINVAL, "gather takes host buffers, synchronously");
    }
    Ctx c;
    if ((rc = open_ctx(dev, o.stream, &c))) {
        return rc;
    }
    Workspace* w = c.w;
    std::lock_guard<std::mutex> g(w->mu);
    if ((rc = w->arena.ensure(total + 16))) {
        return rc;
    }
    if (total && !w->pin) {
        void* h = nullptr;
        HIP_TRY(hipHostMalloc(&h, kGatherSlots * kGatherChunk, hipHostMallocPortable));
        w->pin = (uint8_t*)h;
        for (int sl = 0; sl < kGatherSlots; ++sl) {
            HIP_TRY(hipEventCreateWithFlags(&w->pin_ev[sl], hipEventDisableTiming));
        }
    }
    const uint64_t nchunks = (total + kGatherChunk - 1) / kGatherChunk;
    const int nthreads = (int)std::min<uint64_t>(kGatherThreads, nchunks);
    std::vector<int> trc(std::max(nthreads, 1), 0);
    std::vector<std::string> terr(trc.size());
    auto worker = [&](int t) {
        if (hipSetDevice(dev) != hipSuccess) {
            trc[t] = BMQCRC_EIO;
            terr[t] = "hipSetDevice failed in a gather thread";
            return;
        }
        const int per = kGatherSlots / nthreads;  // slots t, t + nthreads, ... are thread t's
        for (uint64_t ch = (uint64_t)t; ch < nchunks; ch += (uint64_t)nthreads) {
            const int sl = t + nthreads * (int)((ch / (uint64_t)nthreads) % (uint64_t)per);
            hipError_t e = hipSuccess;
            if (w->pin_used[sl]) {
                e = hipEventSynchronize(w->pin_ev[sl]);  // the slot's previous copy is done
            }
            const uint64_t lo = ch * kGatherChunk, hi = std::min(total, lo + kGatherChunk);
            uint8_t* dst = w->pin + (uint64_t)sl * kGatherChunk;
            size_t k = (size_t)(std::upper_bound(boff.begin(), boff.end(), lo) - boff.begin()) - 1;
            for (uint64_t pos = lo; e == hipSuccess && pos < hi;) {
                if (boff[k + 1] <= pos) {
                    ++k;  // empty buffers and buffers that end at pos
                    continue;
                }
                const uint64_t take = std::min(hi, boff[k + 1]) - pos;
                memcpy(dst + (pos - lo), (const uint8_t*)bufs[b0 + k] + (pos - boff[k]), take);
                pos += take;
            }
            if (e == hipSuccess) {
                e = hipMemcpyAsync((uint8_t*)w->arena.p + lo, dst, hi - lo, hipMemcpyHostToDevice,
                                   c.s);
            }
            if (e == hipSuccess) {
                e = hipEventRecord(w->pin_ev[sl], c.s);
            }
            if (e != hipSuccess) {
                trc[t] = e == hipErrorOutOfMemory ? BMQCRC_ENOMEM : BMQCRC_EIO;
                terr[t] = std::string("gather staging: ") + hipGetErrorString(e);
                return;
            }
            w->pin_used[sl] = true;
        }
    };
    if (nthreads == 1) {
        worker(0);
    } else if (nthreads > 1) {
        std::vector<std::thread> th;
        for (int t = 0; t < nthreads; ++t) {
            th.emplace_back(worker, t);
        }
        for (auto& t : th) {
            t.join();
        }
    }
    for (size_t t = 0; t < trc.size(); ++t) {
        if (trc[t]) {
            (void)hipStreamSynchronize(c.s);  // no copy may still read a slot we hand back
            return fail(trc[t], terr[t]);
        }
    }
    if ((rc = stage(c, w->offsets, moff.data(), 8 * n)) ||
        (rc = stage(c, w->lengths, mlen.data(), 4 * n)) ||
        (seeds && (rc = stage(c, w->seeds, seeds, 4 * n))) || (rc = w->out.ensure(4 * n))) {
        return rc;
    }
    if ((rc = run_batch(c, o.flags, seg, w->arena.p, total, (const uint64_t*)w->offsets.p,
                        (const uint32_t*)w->lengths.p,
                        seeds ? (const uint32_t*)w->seeds.p : nullptr, (uint32_t*)w->out.p, n,
                        maxlen))) {
        return rc;
    }
    HIP_TRY(hipMemcpyAsync(out, w->out.p, 4 * n, hipMemcpyDeviceToHost, c.s));
    HIP_TRY(hipStreamSynchronize(c.s));
    return 0;
}

int bmqcrc_crc32c_batch_multi(const void* arena, uint64_t arena_bytes, const uint64_t* offsets,
                              const uint32_t* lengths, const uint32_t* seeds, uint32_t* out,
                              uint64_t n, const int* devices, int ndev, uint32_t seg_bytes)
{
    t_err.clear();
    if (n == 0) {
        return 0;
    }
    if (ndev < 1 || !offsets || !lengths || !out || !arena) {
        return fail(BMQCRC_EINVAL, "bad arguments");
    }
    uint32_t seg = seg_bytes;
    int rc = check_seg(&seg);
    if (rc) {
        return rc;
    }
    const int have = device_count_raw();
    if (have <= 0) {
        return fail(BMQCRC_ENODEV, "no HIP device available");
    }
    std::vector<int> devs(ndev);
    for (int d = 0; d < ndev; ++d) {
        devs[d] = devices ? devices[d] : d;
        if (devs[d] < 0 || devs[d] >= have) {
            return fail(BMQCRC_EINVAL, "device ordinal out of range");
        }
    }
    uint64_t total = 0;
    for (uint64_t i = 0; i < n; ++i) {
        if (offsets[i] > arena_bytes || lengths[i] > arena_bytes - offsets[i]) {
            return fail(BMQCRC_EINVAL, "message outside arena");
        }
        total += lengths[i];
    }
    // Contiguous byte-balanced message slices; each device gets its own
    // copy of the arena range its slice touches.
    std::vector<uint64_t> cut(ndev + 1, n);
    cut[0] = 0;
    {
        uint64_t acc = 0, i = 0;
        for (int d = 1; d < ndev; ++d) {
            const uint64_t target = total * (uint64_t)d / (uint64_t)ndev;
            while (i < n && acc < target) {
                acc += lengths[i++];
            }
            cut[d] = i;
        }
    }
    std::vector<int> rcs(ndev, 0);
    std::vector<std::string> errs(ndev);
    std::vector<std::thread> th;
    for (int d = 0; d < ndev; ++d) {
        th.emplace_back([&, d]() {
            const uint64_t lo = cut[d], hi = cut[d + 1];
            if (lo >= hi) {
                return;
            }
            uint64_t amin = UINT64_MAX, amax = 0;
            for (uint64_t i = lo; i < hi; ++i) {
                amin = std::min(amin, offsets[i]);
                amax = std::max(amax, offsets[i] + lengths[i]);
            }
            if (amin > amax) {
                amin = amax = 0;
            }
            std::vector<uint64_t> rel(hi - lo);
            for (uint64_t i = lo; i < hi; ++i) {
                rel[i - lo] = offsets[i] - amin;
            }
            rcs[d] = batch_one(devs[d], nullptr, 0, seg, (const uint8_t*)arena + amin, amax - amin,
                               rel.data(), lengths + lo, seeds ? seeds + lo : nullptr, out + lo,
                               hi - lo);
            errs[d] = t_err;
        });
    }
    for (auto& t : th) {
        t.join();
    }
    for (int d = 0; d < ndev; ++d) {
        if (rcs[d]) {
            return fail(rcs[d], "device " + std::to_string(devs[d]) + ": " + errs[d]);
        }
    }
    return 0;
}

int bmqcrc_reserve(int device, void* stream, uint64_t n_msgs, uint64_t arena_bytes,
                   uint32_t seg_bytes)
{
    t_err.clear();
    DeviceGuard keep_device;
    int dev, rc;
    if ((rc = check_seg(&seg_bytes)) || (rc = resolve_device(device, &dev))) {
        return rc;
    }
    DeviceState* st = nullptr;
    if ((rc = device_state(dev, &st))) {
        return rc;
    }
    HIP_TRY(hipSetDevice(dev));
    Workspace* w = workspace(dev, stream);
    std::lock_guard<std::mutex> g(w->mu);
    BatchArgs a;
    memset(&a, 0, sizeof(a));
    auto_shape(n_msgs, arena_bytes, st->num_cus, &seg_bytes, &a.blocks_per_cu);  // as the batch call will
    return plan_ws(w, (hipStream_t)stream, n_msgs, arena_bytes, seg_bytes, &a, *st);
}

int bmqcrc_fill_synthetic(void* dev_dst, uint64_t nbytes, uint64_t seed, uint64_t begin,
                          const bmqcrc_opts* opts)
{
    t_err.clear();
    DeviceGuard keep_device;
    int dev, rc;
    if ((rc = resolve_device(opts ? opts->device : -1, &dev))) {
        return rc;
    }
    if (((uintptr_t)dev_dst & 7u) || (begin & 7u)) {
        return fail(BMQCRC_EINVAL, "destination and begin must be 8-byte aligned");
    }
    DeviceState* st = nullptr;
    if ((rc = device_state(dev, &st))) {
        return rc;
    }
    HIP_TRY(hipSetDevice(dev));
    hipStream_t s = opts ? (hipStream_t)opts->stream : nullptr;
    if (bmqcrc_launch_fill((uint8_t*)dev_dst, nbytes, seed, begin, (void*)s)) {
        return fail(BMQCRC_EIO, "fill launch failed");
    }
    if (!(opts && (opts->flags & BMQCRC_F_ASYNC))) {
        HIP_TRY(hipStreamSynchronize(s));
    }
    return 0;
}

int bmqcrc_kernel_timing(int device, void* stream, double* total_ms, uint32_t* count)
{
    t_err.clear();
    DeviceGuard keep_device;
    int dev, rc;
    if ((rc = resolve_device(device, &dev))) {
        return rc;
    }
    HIP_TRY(hipSetDevice(dev));
    Workspace* w = workspace(dev, stream);
    std::lock_guard<std::mutex> g(w->mu);
    double tot = 0;
    uint32_t cnt = 0;
    for (auto& e : w->timing) {
        HIP_TRY(hipEventSynchronize(e.second));
        float ms = 0;
        HIP_TRY(hipEventElapsedTime(&ms, e.first, e.second));
        tot += ms;
        ++cnt;
        w->spare.push_back(e);
    }
    w->timing.clear();
    if (total_ms) {
        *total_ms = tot;
    }
    if (count) {
        *count = cnt;
    }
    return 0;
}

int bmqcrc_last_launch(int device, void* stream, uint32_t* kernels, uint32_t* spec,
                       uint32_t* seg_bytes)
{
    t_err.clear();
    DeviceGuard keep_device;
    int dev, rc;
    if ((rc = resolve_device(device, &dev))) {
        return rc;
    }
    Workspace* w = workspace(dev, stream);
    std::lock_guard<std::mutex> g(w->mu);
    if (kernels) {
        *kernels = w->last_kernels;
    }
    if (spec) {
        *spec = w->last_spec;
    }
    if (seg_bytes) {
        *seg_bytes = w->last_seg;
    }
    return 0;
}

int bmqcrc_last_plan(int device, void* stream, uint32_t* map)
{
    t_err.clear();
    DeviceGuard keep_device;
    int dev, rc;
    if ((rc = resolve_device(device, &dev))) {
        return rc;
    }
    Workspace* w = workspace(dev, stream);
    std::lock_guard<std::mutex> g(w->mu);
    if (map) {
        *map = w->last_map;
    }
    return 0;
}

int bmqcrc_forget_shape(int device, void* stream)
{
    t_err.clear();
    DeviceGuard keep_device;
    int dev, rc;
    if ((rc = resolve_device(device, &dev))) {
        return rc;
    }
    Workspace* w = workspace(dev, stream);
    std::lock_guard<std::mutex> g(w->mu);
    if (w->hint_host) {
        __atomic_store_n(w->hint_host, kHintUnknown, __ATOMIC_RELAXED);
    }
    return 0;
}

int bmqcrc_plan_wait(int device, void* stream, uint64_t wait_us, uint64_t* voided)
{
    t_err.clear();
    DeviceGuard keep_device;
    int dev, rc;
    DeviceState* st = nullptr;
    if ((rc = resolve_device(device, &dev)) || (rc = device_state(dev, &st))) {
        return rc;
    }
    HIP_TRY(hipSetDevice(dev));
    Workspace* w = workspace(dev, stream);
    std::lock_guard<std::mutex> g(w->mu);
    w->map_wait_ticks = wait_us > (UINT64_MAX / 100) ? UINT64_MAX : wait_us * 100;
    if (voided) {
        // k_plan_map counts its launches that gave up their map (plan_sync[3])
        unsigned long long n = 0;
        if (w->plan_sync.p) {  // after the work already enqueued on this stream
            HIP_TRY(hipMemcpyAsync(&n, (const uint8_t*)w->plan_sync.p + 24, 8,
                                   hipMemcpyDeviceToHost, (hipStream_t)stream));
            HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
        }
        *voided = n;
    }
    return 0;
}

int bmqcrc_host_register(void* host, uint64_t bytes, int device, void** dev_ptr)
{
    t_err.clear();
    DeviceGuard keep_device;
    if (!host || !bytes || !dev_ptr) {
        return fail(BMQCRC_EINVAL, "host, bytes and dev_ptr are required");
    }
    int dev, rc;
    DeviceState* st = nullptr;
    if ((rc = resolve_device(device, &dev)) || (rc = device_state(dev, &st))) {
        return rc;
    }
    HIP_TRY(hipSetDevice(dev));
    HIP_TRY(hipHostRegister(host, bytes, hipHostRegisterMapped | hipHostRegisterPortable));
    void* d = nullptr;
    const hipError_t e = hipHostGetDevicePointer(&d, host, 0);
    if (e != hipSuccess) {
        (void)hipHostUnregister(host);
        return fail(BMQCRC_EIO, std::string("hipHostGetDevicePointer: ") + hipGetErrorString(e));
    }
    *dev_ptr = d;
    return 0;
}

int bmqcrc_host_unregister(void* host)
{
    t_err.clear();
    if (!host) {
        return fail(BMQCRC_EINVAL, "null host pointer");
    }
    if (device_count_raw() <= 0) {
        return fail(BMQCRC_ENODEV, "no HIP device available");
    }
    HIP_TRY(hipHostUnregister(host));
    return 0;
}

int bmqcrc_device_count(void)
{
    return device_count_raw();
}

const char* bmqcrc_last_error(void)
{
    return t_err.c_str();
}

// Host fallbacks of the C++ spellings (bmqcrc.h).  A fault (EIO) is never
// silent: the first one in the process is printed with its HIP error.
static std::atomic<uint64_t> g_fallbacks{0};
static std::atomic<int32_t> g_fallback_rc{0};
static std::atomic<bool> g_eio_reported{false};

void bmqcrc_note_host_fallback(int32_t rc)
{
    g_fallbacks.fetch_add(1, std::memory_order_relaxed);
    g_fallback_rc.store(rc, std::memory_order_relaxed);
    if (rc == BMQCRC_EIO && !g_eio_reported.exchange(true)) {
        fprintf(stderr,
                "libbmqcrc: GPU batch failed with BMQCRC_EIO (%s); finishing on the host "
                "(bmqcrc_host_fallbacks counts every such call)\n",
                t_err.c_str());
    }
}

uint64_t bmqcrc_host_fallbacks(int32_t* last_rc)
{
    if (last_rc) {
        *last_rc = g_fallback_rc.load(std::memory_order_relaxed);
    }
    return g_fallbacks.load(std::memory_order_relaxed);
}

uint32_t bmqcrc_version(void)
{
    return (2u << 16) | 7u;
}

}  // extern "C"
