#!/usr/bin/env python3
"""Device-resident CRC32C GiB/s over batched payloads on 1/2/4/8 MI355X.

Metric and configs: BASELINE.json.  A "step" is one bmqcrc_crc32c_batch call
(planner kernels + fold kernel) over one resident batch.  Default workload
(N=1) is configs[2]: 65,536 messages x 64 KiB of synthetic random payload
(splitmix64 stream, seed 2) -- the headline HBM-bound regime.

--gpus N runs one process per GPU.  Under torchrun (WORLD_SIZE set) it must
equal WORLD_SIZE; without it, bench.py starts `torch.distributed.run
--nproc-per-node N` itself as a child process (before touching a GPU) and
exits with its status.  Every rank CRCs its own 64k x 64 KiB slice of an
N-times larger batch (weak scaling, no data-path collective; a gloo barrier
brackets the timed region and the time is the max over ranks).  For N > 1
the line also carries "strong_scaling": BASELINE configs[3] (Zipf 4M, one
batch split byte-balanced over the N ranks) timed across the ranks and, in
the same run, the whole batch on rank 0's GPU alone -- the measured speed-up.

Output: one JSON line on rank 0 (see README/DESIGN.md for fields).
"""
import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md

# BASELINE.json configs (configs[0] is the reference's CPU-only case).
#   name: (description, lengths(rank, world) -> (np.uint32 lengths, stream begin), payload seed, scaling)
ZIPF_N = 4 << 20


def _uniform(n, size):
    def gen(rank, world):
        import numpy as np
        return np.full(n, size, dtype=np.uint32), rank * n * size
    return gen


def _zipf(rank, world):
    """configs[3]: 4M msgs, size = 64*r, r in [1,16384], P(r) ~ r^-1.5 (seed 3),
    one global batch sharded byte-balanced across the ranks (no collective)."""
    import numpy as np
    from blazingmq_amd.shard import rank_slice
    rng = np.random.default_rng(3)
    r = np.arange(1, 16385, dtype=np.float64)
    p = r ** -1.5
    p /= p.sum()
    lens = (64 * rng.choice(16384, size=ZIPF_N, p=p) + 64).astype(np.uint32)
    lo, hi = rank_slice(lens, rank, world)
    begin = int(lens[:lo].sum(dtype=np.uint64))
    return lens[lo:hi], begin


CONFIGS = {
    "1k_x_4KiB": ("1,000 msgs x 4 KiB (configs[0], the reference's CPU-only case; launch-bound "
                  "on the GPU)", _uniform(1000, 4096), 0xB1A2E5, "weak"),
    "64k_x_64KiB": ("65,536 msgs x 64 KiB per GPU (configs[2], HBM-bound headline)",
                    _uniform(65536, 65536), 2, "weak"),
    "1M_x_256B": ("1,048,576 msgs x 256 B per GPU (configs[1], small-message regime)",
                  _uniform(1 << 20, 256), 1, "weak"),
    "zipf_4M": ("4M msgs, Zipf 64 B-1 MiB (r^-1.5), one batch sharded across GPUs (configs[3])",
                _zipf, 4, "strong"),
    "16_x_256MiB": ("16 msgs x 256 MiB per GPU (configs[4], multi-chunk fold + combine)",
                    _uniform(16, 256 << 20), 5, "weak"),
}

UNIFORM_SIZES = {"1k_x_4KiB": 4096, "64k_x_64KiB": 65536, "1M_x_256B": 256,
                 "16_x_256MiB": 256 << 20}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--config", default=None, choices=list(CONFIGS),
                   help="default 64k_x_64KiB (the headline); --cpu-table: all configs")
    p.add_argument("--seg-bytes", type=int, default=0)
    p.add_argument("--whole-messages", action="store_true",
                   help="BMQCRC_F_WHOLE_MESSAGES: one lane per message, no planner launches")
    p.add_argument("--msg-bytes", type=int, default=0,
                   help="experiment: override the message size of a uniform config "
                        "(the line is then marked as not the BASELINE workload)")
    p.add_argument("--msgs", type=int, default=0,
                   help="experiment: override the message count of a uniform config "
                        "(the line is then marked as not the BASELINE workload)")
    p.add_argument("--align", type=int, default=0,
                   help="experiment: start every message at a multiple of this many bytes "
                        "(padding between messages, never read; Zipf over-fetch attribution: "
                        "128 leaves no 128-byte line shared by two messages); the line is "
                        "marked as not the BASELINE workload")
    p.add_argument("--shard", default="",
                   help="experiment 'i/N': time only shard i of an N-way split of the config on "
                        "this one GPU (a strong-scaling rank's work; the line is marked as not "
                        "the BASELINE workload)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=2.0,
                   help="approximate wall time of the CPU-baseline sample")
    p.add_argument("--check", type=int, default=256, help="messages checked against the oracle")
    p.add_argument("--settle-seconds", type=float, default=1.0,
                   help="untimed batch passes during setup, before the W warmup steps, so the "
                        "GPU reaches steady-state clocks (measured: a cold GPU reads ~6%% low)")
    p.add_argument("--no-kernel-timing", action="store_true",
                   help="skip the HIP-event pass around k_fold (for external profilers)")
    p.add_argument("--cpu-table", action="store_true",
                   help="CPU baseline table (DESIGN.md section 6): every config, the three "
                        "bdlde::Crc32c variants restated in oracle/, 1 and up to 16 threads")
    p.add_argument("--scalar", action="store_true",
                   help="the drop-in scalar bmqp::Crc32c::calculate (pointer and 4 KiB-buffer "
                        "Blob forms, tools/bin/scalar_ladder) on the reference's size ladder, "
                        "beside its published times and the oracle's SSE4.2 3-way and serial "
                        "crc32q loops; one JSON line per size (no GPU)")
    p.add_argument("--protocol", action="store_true",
                   help="measure the batch callers of SURVEY.md 8(f): partition recovery "
                        "verify, deferred PUT-event CRCs, Blob batches, ledger validation")
    p.add_argument("--e2e", action="store_true",
                   help="end-to-end mode: H2D from pinned host + CRC + D2H (for DESIGN.md)")
    p.add_argument("--no-strong-scaling", action="store_true",
                   help="N > 1: skip the strong-scaled Zipf object")
    p.add_argument("--rotate", type=int, default=None,
                   help="N > 1: every step (settle, warmup, timed, planned, declared, kernel "
                        "timing) takes the next of N copies of the batch (arena, offsets, "
                        "lengths, out), so a batch smaller than the 256 MiB Infinity Cache is "
                        "read from HBM rather than replayed from the cache.  Default: 4 for "
                        "1M_x_256B (configs[1], 272 MiB: 4 copies cycle 1.1 GiB, so its line "
                        "is an HBM figure; --rotate 1 replays one copy from the cache), 1 "
                        "otherwise")
    p.add_argument("--plan-wait-us", type=int, default=None,
                   help="bmqcrc_plan_wait limit for this run (default: the library's 100 us; "
                        "0 gives every ragged batch's size-class map up: the fallback's cost)")
    p.add_argument("--launch-check", action="store_true",
                   help="test hook: start the ranks, rendezvous over gloo and print the "
                        "world as rank 0 sees it, without touching a GPU")
    a = p.parse_args()
    a.config_given = a.config is not None
    if a.rotate is None:
        a.rotate = 4 if a.config == "1M_x_256B" else 1
    if a.config is None:
        a.config = "64k_x_64KiB"
    return a


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def host_threads():
    """This GPU's share of the host: the box's thread allotment
    (OMP_NUM_THREADS, 16 per GPU on the pool), else min(nproc, 16)."""
    try:
        return max(1, int(os.environ["OMP_NUM_THREADS"]))
    except (KeyError, ValueError):
        return min(os.cpu_count() or 1, 16)


# The reference's published default-CRC32C time per buffer (ns), 64-bit
# hardware-accelerated build (bmqp_crc32c.h:116,119,122,127,129), measured by
# its tight loop of 100,000 calls on one buffer (bmqp_crc32c.t.cpp:1116-1120).
REF_PUBLISHED_NS = {256: (30, "bmqp_crc32c.h:116"), 1024: (45, "bmqp_crc32c.h:119"),
                    4096: (176, "bmqp_crc32c.h:122"), 65536: (2858, "bmqp_crc32c.h:127"),
                    1 << 20: (50937, "bmqp_crc32c.h:129")}


def gpu_numa_node(device):
    """NUMA node of the GPU `device` (torch ordinal) from its PCI address,
    or None."""
    try:
        import torch
        p = torch.cuda.get_device_properties(device)
        addr = "%04x:%02x:%02x.0" % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
        with open("/sys/bus/pci/devices/%s/numa_node" % addr) as f:
            node = int(f.read().strip())
        return node if node >= 0 else None
    except Exception:
        return None


def cpu_baseline(lens_np, seed, seconds, device=0):
    """Reference-equivalent CPU CRC32C (oracle, SSE4.2 3-way; BDE 4.39 is not
    available offline) on a bounded sample (first ~256 MiB of messages) of the
    same synthetic workload.  Legs, each warm (one untimed pass) and timed
    for >= 0.3 s: the batch on one thread; on this GPU's share of the host's
    threads (created once, before the clock, each pinned to its own physical
    core; the test5 pattern, one thread per byte-balanced message slice;
    median of seven windows) both streamed from DRAM and cache-resident (the
    value: every thread re-CRCs its own copy of <= 2 MiB of the sample, the
    reference's loop methodology); and the reference's own
    benchmark loop (bmqp_crc32c.t.cpp:1116-1120: one message CRC'd up to
    100,000 times) for messages up to 1 MiB, beside its published figure."""
    import numpy as np
    import oracle
    threads = host_threads()
    csum = np.cumsum(lens_np, dtype=np.uint64)
    n = max(1, int(np.searchsorted(csum, 256 << 20, side="right")))
    lens = np.ascontiguousarray(lens_np[:n])
    offs = np.zeros(n, dtype=np.uint64)
    if n > 1:
        offs[1:] = csum[:n - 1]
    nbytes = int(lens.sum(dtype=np.uint64))
    # every thread pinned to its own physical core of the process's allowed
    # set, on the GPU's NUMA node first, idle cores first (round 6:
    # unpinned, 16 threads swung 2x between windows of one run);
    # the 1-thread leg on the first of them.  The sample is written while the
    # process runs on those cores, so its pages are theirs (first touch).
    node = gpu_numa_node(device)
    cpus = oracle.pick_cpus(threads, node)
    threads = len(cpus)
    saved_affinity = os.sched_getaffinity(0)
    try:
        os.sched_setaffinity(0, cpus)
    except OSError:
        pass
    arena = oracle.fill_payload(0, nbytes, seed)
    # a batch far below the sample size (configs[0]: 1,000 x 4 KiB = 4 MB)
    # is tiled to >= 64 MiB, so that a pass is milliseconds of CRC work, not
    # the pool's per-pass barrier (the multi-threaded windows swung 40 % on
    # 26-us passes, round 6)
    tiles = max(1, -(-(64 << 20) // max(nbytes, 1))) if nbytes < (64 << 20) else 1
    if tiles > 1:
        arena = np.tile(arena, tiles)
        offs = (offs[None, :] + (np.arange(tiles, dtype=np.uint64) * np.uint64(nbytes))[:, None]
                ).reshape(-1)
        lens = np.tile(lens, tiles)
        nbytes *= tiles
    try:
        os.sched_setaffinity(0, saved_affinity)
    except OSError:
        pass
    t1, reps1 = oracle.time_batch_for(arena, offs, lens, 1, "hw", 0.5, cpus=cpus)
    # the multi-threaded leg shares the box's host with other jobs: one
    # untimed window (clocks and caches settle), then seven timed windows,
    # the median reported with the min and max
    nwin = 7
    oracle.time_batch_for(arena, offs, lens, threads, "hw", max(0.3, seconds / nwin), cpus=cpus)
    legs = [oracle.time_batch_for(arena, offs, lens, threads, "hw", max(0.3, seconds / nwin),
                                  cpus=cpus)
            for _ in range(nwin)]
    gib = nbytes / 2**30
    rates = sorted(gib * r / tt for tt, r in legs)
    med = rates[nwin // 2]
    # The cache-resident leg (the value): the reference's own methodology --
    # a resident buffer CRC'd over and over (bmqp_crc32c.t.cpp:1116-1120) --
    # on every thread at once: thread t CRCs its own copy of the sample's
    # first messages (<= 2 MiB: its core's L2 and share of the L3) 32 times
    # per pass.  The streamed leg above reads 256 MiB from DRAM through the
    # CCDs' fabric links, which the host's other jobs share: its windows
    # swung 11-29 % within a run and 2x between boxes (round 6).
    win = max(1, int(np.searchsorted(csum, 2 << 20, side="right")))
    wl = np.ascontiguousarray(lens_np[:win], dtype=np.uint32)
    wo = np.zeros(win, dtype=np.uint64)
    if win > 1:
        wo[1:] = np.cumsum(wl[:-1], dtype=np.uint64)
    wb = int(wl.sum(dtype=np.uint64))
    stride = (wb + 4095) // 4096 * 4096
    rrep = max(1, (64 << 20) // max(wb, 1)) if wb < (64 << 20) else 1
    try:
        os.sched_setaffinity(0, cpus)
    except OSError:
        pass
    carena = oracle.fill_payload(0, stride * threads, seed)
    try:
        os.sched_setaffinity(0, saved_affinity)
    except OSError:
        pass
    coffs = (np.arange(threads, dtype=np.uint64)[:, None, None] * np.uint64(stride)
             + np.zeros((1, rrep, 1), dtype=np.uint64) + wo[None, None, :]).reshape(-1)
    clens = np.tile(wl, threads * rrep)
    cgib = float(clens.sum(dtype=np.uint64)) / 2**30
    oracle.time_batch_for(carena, coffs, clens, threads, "hw", max(0.3, seconds / nwin), cpus=cpus)
    clegs = [oracle.time_batch_for(carena, coffs, clens, threads, "hw", max(0.3, seconds / nwin),
                                   cpus=cpus)
             for _ in range(nwin)]
    crates = sorted(cgib * r / tt for tt, r in clegs)
    cmed = crates[nwin // 2]
    res = {
        "value": round(cmed, 3),
        "windows_GiBps": [round(cgib * r / tt, 3) for tt, r in clegs],
        "window_min_max": [round(crates[0], 3), round(crates[-1], 3)],
        "window_spread": round((crates[-1] - crates[0]) / cmed, 3),
        "streamed_value": round(med, 3),
        "streamed_windows_GiBps": [round(gib * r / tt, 3) for tt, r in legs],
        "streamed_window_spread": round((rates[-1] - rates[0]) / med, 3),
        "unit": "GiB/s",
        "cores": threads,
        "pinned_cpus": cpus,
        "gpu_numa_node": node,
        "kind": "port",
        "single_thread_value": round(gib * reps1 / t1, 3),
        "host_threads": os.cpu_count(),
        "not_measured": "nproc/8 (%d threads, one GPU's share of an 8-GPU node) and all %d "
                        "threads: a one-GPU job on this pool may use %d threads "
                        "(OMP_NUM_THREADS); the rest of the shared host is not ours to load"
                        % ((os.cpu_count() or 8) // 8, os.cpu_count() or 0, threads),
        "sample": "value: cache-resident, the reference's loop methodology on every thread -- "
                  "thread t CRCs its own copy of the batch's first %d msgs (%.2f MiB) %d times "
                  "per pass; streamed_value: first %d msgs (%.0f MiB%s) of the same synthetic "
                  "batch read from DRAM; %d threads (this "
                  "GPU's share of the host: OMP_NUM_THREADS, 16 per GPU on the pool), each "
                  "pinned to its own physical core (GPU NUMA node %s first, idle cores first; "
                  "the samples first-touched there), created once before the clock; per leg one "
                  "untimed window, then the median of %d windows of >= %.2f s; single "
                  "thread %d warm "
                  "passes (%.2f s) = %.2f GiB/s; SSE4.2 crc32q 3-way interleaved, lanes joined "
                  "by shift tables (bdlde::Crc32c default analogue, oracle/crc32c_oracle.c); "
                  "host %s, nproc %d"
                  % (win, wb / 2**20, rrep, n, gib * 1024,
                     ", the batch tiled %d times" % tiles if tiles > 1 else "",
                     threads, node, nwin, max(0.3, seconds / nwin), reps1, t1,
                     gib * reps1 / t1, cpu_model(), os.cpu_count()),
    }
    size = int(lens_np[0]) if lens_np.size else 0
    if 0 < size <= (1 << 20) and bool(np.all(lens == size)):
        buf = arena[:size]
        iters = 100000
        tr = oracle.time_repeat(buf, 1000)
        iters = int(min(100000, max(1000, 0.5 / max(tr / 1000, 1e-9))))
        tr = oracle.time_repeat(buf, iters)
        ref = {"ns_per_msg": round(1e9 * tr / iters, 1), "msg_bytes": size, "iters": iters,
               "GiBps": round(size * iters / tr / 2**30, 3),
               "method": "the reference's loop: one buffer CRC'd `iters` times on one thread "
                         "(bmqp_crc32c.t.cpp:1116-1120), oracle SSE4.2 3-way",
               "batch_ns_per_msg_1_thread": round(1e9 * t1 / reps1 / (n * tiles), 1)}
        if size in REF_PUBLISHED_NS:
            ns, where = REF_PUBLISHED_NS[size]
            ref.update({"reference_published_ns": ns, "reference_published_at": where,
                        "reference_published_host": "the reference's own (unnamed) 64-bit "
                                                    "build host"})
        # the drop-in scalar bmqp::Crc32c::calculate (the product's CPU path,
        # what unbatched callers link) in the same loop, same host
        try:
            import subprocess
            exe = os.path.join(ROOT, "tools", "bin", "scalar_ladder")
            line = subprocess.run([exe, str(size)], capture_output=True, text=True, timeout=60,
                                  check=True).stdout.splitlines()[-1]
            d = json.loads(line)
            ref["dropin_calculate_ns"] = d["calculate_ns"]
            ref["dropin_blob_4KiB_ns"] = d["blob_4KiB_ns"]
            ref["dropin_source"] = "tools/bin/scalar_ladder (libbmqcrc.so, csrc/crc32c_cpu.cpp)"
        except (OSError, subprocess.SubprocessError, ValueError, KeyError, IndexError) as e:
            ref["dropin_calculate_ns"] = None
            ref["dropin_error"] = str(e)[:200]
        res["reference_loop"] = ref
    return res


CPU_VARIANTS = {"hw": "SSE4.2 crc32q 3-way interleaved (bdlde::Crc32c::calculate default)",
                "hw_serial": "SSE4.2 crc32q serial (calculateHardwareSerial)",
                "sw": "slicing-by-8 software (calculateSoftware)"}


def cpu_table(args):
    """CPU baseline table: the reference-equivalent CPU CRC32C (oracle/'s
    restatement of bdlde::Crc32c, BDE 4.39 being unavailable offline), three
    variants, 1 and T threads (one per core over byte-balanced message slices,
    the reference's test5 pattern), each config sampled like the cpu_baseline
    leg (first messages up to ~256 MiB).  One JSON line per measurement."""
    import platform

    import numpy as np
    import oracle
    threads = host_threads()
    configs = [args.config] if args.config_given else list(CONFIGS)
    for cfg in configs:
        _, gen, seed, _ = CONFIGS[cfg]
        lens_all, begin = gen(0, 1)
        csum = np.cumsum(lens_all, dtype=np.uint64)
        n = max(1, int(np.searchsorted(csum, 256 << 20, side="right")))
        lens = np.ascontiguousarray(lens_all[:n])
        offs = np.zeros(n, dtype=np.uint64)
        if n > 1:
            offs[1:] = csum[:n - 1]
        nbytes = int(lens.sum(dtype=np.uint64))
        arena = oracle.fill_payload(begin, nbytes, seed)
        ref = oracle.batch(arena, offs, lens, nthreads=threads, variant="hw")
        for var in CPU_VARIANTS:
            assert np.array_equal(oracle.batch(arena, offs, lens, nthreads=threads,
                                               variant=var), ref), (cfg, var)
            for th in sorted({1, threads}):
                t, _ = oracle.time_batch(arena, offs, lens, th, var, 1)
                reps = max(1, int(args.cpu_seconds / 4 / max(t, 1e-6)))
                t, _ = oracle.time_batch(arena, offs, lens, th, var, reps)
                print(json.dumps({
                    "config": cfg, "variant": var, "variant_desc": CPU_VARIANTS[var],
                    "threads": th, "GiBps": round(nbytes / 2**30 * reps / t, 3),
                    "sample_msgs": n, "sample_MiB": round(nbytes / 2**20, 1), "passes": reps,
                    "host": cpu_model(), "nproc": os.cpu_count(),
                    "machine": platform.machine()}), flush=True)


# bmqp_crc32c.h:109-132: the reference's default (SSE4.2) time per call, ns,
# on its size ladder (bmqp_crc32c.t.cpp:95-118), 64-bit build
REF_LADDER_NS = {11: 9, 16: 9, 21: 10, 59: 13, 64: 12, 69: 13, 251: 30, 256: 30, 261: 37,
                 1019: 155, 1024: 45, 1029: 50, 4091: 299, 4096: 176, 4101: 190, 16379: 864,
                 16384: 724, 16389: 754, 65536: 2858, 262144: 11925, 1048576: 50937,
                 4194304: 198662, 16777216: 796534, 67108864: 9976933}


def scalar(args):
    """The drop-in scalar CRC (what every unbatched caller links) on the
    reference's size ladder: tools/bin/scalar_ladder times
    bmqp::Crc32c::calculate(ptr, len) and calculate(Blob of 4 KiB buffers)
    with the reference's loop (bmqp_crc32c.t.cpp:1116-1120); beside it the
    oracle's restatement of the reference's SSE4.2 3-way CRC and a serial
    crc32q chain, the same loop in C, and the published time."""
    import subprocess

    import numpy as np
    import oracle
    exe = os.path.join(ROOT, "tools", "bin", "scalar_ladder")
    out = subprocess.run([exe], capture_output=True, text=True, timeout=600, check=True).stdout
    rng = np.random.default_rng(0)
    buf = rng.integers(0, 256, size=64 << 20, dtype=np.uint8)
    host = {"host": cpu_model(), "nproc": os.cpu_count(), "threads": 1}
    for line in out.splitlines():
        rec = json.loads(line)
        size = rec["size"]
        sub = buf[:size]
        iters = max(20, min(100000, rec["iters"]))
        t_hw = oracle.time_repeat(sub, iters, "hw")
        t_ser = oracle.time_repeat(sub, iters, "hw_serial")
        rec.update({"published_ns": REF_LADDER_NS.get(size),
                    "published_at": "bmqp_crc32c.h:109-132",
                    "oracle_3way_ns": round(1e9 * t_hw / iters, 1),
                    "oracle_serial_crc32q_ns": round(1e9 * t_ser / iters, 1),
                    "oracle_iters": iters, **host})
        rec["calculate_over_serial"] = round(rec["calculate_ns"] / rec["oracle_serial_crc32q_ns"], 3)
        rec["calculate_over_published"] = (round(rec["calculate_ns"] / rec["published_ns"], 3)
                                           if rec["published_ns"] else None)
        print(json.dumps(rec), flush=True)
    return 0


def _wall(fn, reps):
    """Median wall time of reps synchronous calls (after one warm-up call)."""
    import time
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2]


def protocol(args):
    """The batch callers of SURVEY.md 8(f), each timed end to end through its
    C-ABI entry point on host buffers (host walk of the reference's format,
    staging through HBM, one batched GPU call, results back), beside the
    reference-equivalent CPU loop (host walk + one bdlde::Crc32c-equivalent
    call per message, oracle/, 1 and 16 threads).  Parity: every stored CRC
    verifies, planted corruptions are found, fills equal the CPU CRCs."""
    import ctypes

    import numpy as np
    import oracle
    import torch

    from blazingmq_amd import _native as N
    from blazingmq_amd import csl, put_event, storage, synth
    threads = host_threads()
    reps = max(3, args.steps // 4)

    def cpu_leg(buf, offs, lens, walk_s):
        out = {}
        for th in (1, threads):
            t, _ = oracle.time_batch(buf, offs, lens, th, "hw", 1)
            k = max(1, int(0.5 / max(t, 1e-6)))
            t, _ = oracle.time_batch(buf, offs, lens, th, "hw", k)
            out["t%d_s" % th] = round(walk_s + t / k, 6)
        return out

    def line(path, ref, n, nbytes, gpu_s, walk_s, cpu, parity, note):
        gib = nbytes / 2**30
        print(json.dumps({
            "path": path, "reference": ref, "messages": n, "payload_bytes": nbytes,
            "gpu": {"s": round(gpu_s, 6), "GiBps": round(gib / gpu_s, 2), "includes": note},
            "host_walk_s": round(walk_s, 6),
            "cpu_baseline": {"kind": "port", "threads": [1, threads],
                             "GiBps": [round(gib / cpu["t1_s"], 2),
                                       round(gib / cpu["t%d_s" % threads], 2)],
                             "what": "host walk + one SSE4.2 3-way CRC per message "
                                     "(oracle/, bdlde::Crc32c analogue)"},
            "speedup_vs_1_thread": round(cpu["t1_s"] / gpu_s, 2),
            "parity": parity, "host": cpu_model()}), flush=True)

    # 1. partition recovery (mqbs_filestore.cpp:2495-2624), 256K x 4000 B
    n = args.msgs or 262144
    journal, data, app_off, app_len = synth.partition(n, 4000)
    walk_s = _wall(lambda: storage.scan_partition(journal, data), reps)
    gpu_s = _wall(lambda: storage.verify_partition(journal, data), reps)
    res = storage.verify_partition(journal, data)
    bad = data.copy()
    planted = [0, n // 2, n - 1]
    for i in planted:
        bad[int(app_off[i]) + 17] ^= 0x5A
    found = storage.verify_partition(journal, bad)
    jrec0 = journal.size - n * storage.JOURNAL_RECORD_SIZE
    # alarms come in the reference's (backward) journal order
    exp_off = [jrec0 + i * storage.JOURNAL_RECORD_SIZE for i in reversed(planted)]
    parity = {"n_bad": res["n_bad"], "planted": len(planted),
              "found_exact": found["bad_record_offsets"].tolist() == exp_off}
    line("recovery_verify", "mqbs::FileStore::recoverMessages CRC check "
         "(mqbs_filestore.cpp:2495-2624)", n, int(app_len.sum(dtype=np.uint64)), gpu_s, walk_s,
         cpu_leg(data, app_off, app_len, walk_s), parity,
         "journal + DATA walk on the host, H2D of the DATA file, batched verify, D2H")
    del journal, data, bad

    # 2. deferred PUT-event CRCs (bmqp_puteventbuilder.cpp:302,320,400,413),
    #    one 64 MiB-class event of 1 KiB messages
    m = 60000
    event, ev_off, ev_len = synth.put_event(m, 1020)
    it = put_event.PutMessageIterator(event)
    walk_s = _wall(lambda: it.scan(), reps)
    opts = N.make_opts()
    work = event.copy()

    def fill():
        N.check_count(N.lib.bmqcrc_put_event_fill_crcs(ctypes.c_void_p(work.ctypes.data),
                                                       work.size, ctypes.byref(opts)))
    gpu_s = _wall(fill, reps)
    got = np.frombuffer(work.tobytes(), np.uint8)
    pos = ev_off - 8
    stored = (got[pos.astype(np.int64)[:, None] + np.arange(4)].astype(np.uint32)
              * np.array([1 << 24, 1 << 16, 1 << 8, 1], np.uint32)).sum(1).astype(np.uint32)
    exp = oracle.batch(event, ev_off, ev_len, nthreads=threads)
    nm, nb, _ = put_event.PutMessageIterator(work).verify_crcs()
    parity = {"fill_equals_cpu": bool(np.array_equal(stored, exp)), "verify_n_bad": nb}
    line("put_event_fill_crcs", "bmqp::PutEventBuilder::packMessage CRC "
         "(bmqp_puteventbuilder.cpp:302,320,400,413)", m, int(ev_len.sum()), gpu_s, walk_s,
         cpu_leg(event, ev_off, ev_len, walk_s), parity,
         "PUT walk on the host, H2D of the event, batched CRC, D2H, big-endian header writes")
    del event, work

    # 3. Blob batches (bmqp_crc32c.cpp:47-67): 16K blobs of 16 x 4 KiB buffers,
    #    device-resident (buffers already in HBM)
    dev = torch.device("cuda", 0)
    nblob, nbuf, bsz = 16384, 16, 4096
    total = nblob * nbuf * bsz
    arena = torch.empty(total + 64, dtype=torch.uint8, device=dev)
    from blazingmq_amd import fill_synthetic
    fill_synthetic(arena, 21)
    boff = torch.arange(nblob * nbuf, dtype=torch.int64, device=dev) * bsz
    blen = torch.full((nblob * nbuf,), bsz, dtype=torch.int32, device=dev)
    first = torch.arange(nblob + 1, dtype=torch.int64, device=dev) * nbuf
    out = torch.empty(nblob, dtype=torch.int32, device=dev)
    dopts = N.make_opts(flags=N.BMQCRC_F_DEVICE_PTRS)

    def blobs():
        N.check(N.lib.bmqcrc_crc32c_blobs(
            ctypes.c_void_p(arena.data_ptr()), arena.numel(), ctypes.c_void_p(boff.data_ptr()),
            ctypes.c_void_p(blen.data_ptr()), nblob * nbuf, ctypes.c_void_p(first.data_ptr()),
            None, ctypes.c_void_p(out.data_ptr()), nblob, ctypes.byref(dopts)))
        torch.cuda.synchronize(dev)
    gpu_s = _wall(blobs, reps)
    host = arena.cpu().numpy()
    bo = np.arange(nblob, dtype=np.uint64) * (nbuf * bsz)
    bl = np.full(nblob, nbuf * bsz, np.uint32)
    exp = oracle.batch(host, bo, bl, nthreads=threads)  # a blob = its buffers concatenated
    parity = {"equal": bool(np.array_equal(out.cpu().numpy().view(np.uint32), exp))}
    line("blobs_device", "bmqp::Crc32c::calculate(const bdlbb::Blob&) per blob "
         "(bmqp_crc32c.cpp:47-67)", nblob, total, gpu_s, 0.0, cpu_leg(host, bo, bl, 0.0), parity,
         "device-resident buffers: per-buffer CRCs + on-device combine, one synchronous call")

    # 3b. the same blobs with their buffers scattered in host memory (each a
    #     separate allocation, like a broker's 4 KiB blob buffers):
    #     Crc32c::calculateBatch(const Blob*) -> bmqcrc_crc32c_gather (pinned
    #     staging ring, gather overlapped with the H2D copies, one fold launch)
    hbufs = [np.array(host[i * bsz:(i + 1) * bsz]) for i in range(nblob * nbuf)]
    ptrs = (ctypes.c_void_p * len(hbufs))(*[b.ctypes.data for b in hbufs])
    hlen = np.full(len(hbufs), bsz, np.uint32)
    hfirst = np.arange(nblob + 1, dtype=np.uint64) * nbuf
    hout = np.zeros(nblob, np.uint32)
    hopts = N.make_opts()

    def gather():
        N.check(N.lib.bmqcrc_crc32c_gather(ptrs, hlen.ctypes.data, len(hbufs), hfirst.ctypes.data,
                                           None, hout.ctypes.data, nblob, ctypes.byref(hopts)))
    gpu_s = _wall(gather, reps)
    parity = {"equal": bool(np.array_equal(hout, exp))}
    line("blobs_host_gather", "bmqp::Crc32c::calculate(const bdlbb::Blob&) per blob "
         "(bmqp_crc32c.cpp:47-67)", nblob, total, gpu_s, 0.0, cpu_leg(host, bo, bl, 0.0), parity,
         "host buffers (one allocation each) gathered through the pinned ring and copied to HBM "
         "by %d threads, one fold launch, D2H of the CRCs; CPU leg on a contiguous copy" %
         min(8, (total + (4 << 20) - 1) // (4 << 20)))
    del arena, host, hbufs

    # 4. cluster state ledger validation (mqbc_clusterstateledgerutil.cpp:248-336)
    r = 32768
    rng = np.random.default_rng(13)
    adv = rng.integers(0, 256, size=(r, 1000), dtype=np.uint8)
    log = np.frombuffer(csl.file_header(b"BMQ01") + b"".join(
        csl.append_record(adv[i].tobytes(), sequence_number=i + 1) for i in range(r)),
        np.uint8).copy()
    wrc, end, roff, rlen, rcrc = csl.scan_log(log)
    walk_s = _wall(lambda: csl.scan_log(log), reps)
    gpu_s = _wall(lambda: csl.validate_log(log), reps)
    rc, off, _ = csl.validate_log(log)
    bad = log.copy()
    bad[int(roff[r // 3]) + 40] ^= 1
    rc_bad, _, first_bad = csl.validate_log(bad)
    parity = {"rc": rc, "end_offset_ok": off == log.size, "corrupt_rc": rc_bad,
              "first_bad_ok": first_bad == int(roff[r // 3])}
    line("csl_validate", "mqbc::ClusterStateLedgerUtil::validateLog "
         "(mqbc_clusterstateledgerutil.cpp:248-336)", r, int(np.asarray(rlen).sum()), gpu_s,
         walk_s, cpu_leg(log, np.asarray(roff, np.uint64), np.asarray(rlen, np.uint32), walk_s),
         parity, "ledger walk on the host, H2D, batched verify, D2H")


def pmc_traffic(config):
    """HBM bytes per k_fold launch from the newest committed rocprofv3 PMC
    summary of this config: read = 2 x FETCH_SIZE (gfx950 correction) +
    WRITE_SIZE, per MI355X_MICROARCH.md.  bench_traffic.json (repo root,
    written by tools/summarize_profiles.py) holds the newest figure per config
    with its source summary under profiles/rNN/ -- it travels to the GPU box,
    where ./profiles is not sent; the summaries themselves are the fallback."""
    try:
        with open(os.path.join(ROOT, "bench_traffic.json")) as f:
            t = json.load(f)[config]
        return int(t["traffic_bytes_per_launch"]), t["source"]
    except (OSError, ValueError, KeyError, TypeError):
        pass
    import glob
    # newest round first, and within a round its final/ set after the rest
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", config + "_summary.json")) +
                   glob.glob(os.path.join(ROOT, "profiles", "r*", "final", config + "_summary.json")))
    if not paths:
        return None, None
    with open(paths[-1]) as f:
        s = json.load(f)
    return int(s["traffic_bytes_per_launch"]), os.path.relpath(paths[-1], ROOT)


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def spawn_ranks(args):
    """--gpus N without torchrun: run N ranks under torch.distributed.run as a
    child process (this process has not touched a GPU) and return its status."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1",
           "--nproc-per-node", str(args.gpus), "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def launch_check(args, world, rank):
    """The rank plumbing of a GPU run (rendezvous, barrier, max over ranks)
    with no GPU: rank 0 prints what it sees."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
        dist.barrier()
        t = torch.tensor([float(rank)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        top = int(t[0])
        dist.destroy_process_group()
    else:
        top = 0
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "max_rank": top,
                          "gpus_arg": args.gpus}), flush=True)
    return 0


def main():
    args = parse()
    if args.cpu_table:
        return cpu_table(args)
    if args.scalar:
        return scalar(args)
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        return spawn_ranks(args)
    world = int(world_env or "1")
    if world != args.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world), file=sys.stderr)
        return 2
    if args.launch_check:
        return launch_check(args, world, int(os.environ.get("RANK", "0")))
    if args.protocol:
        import torch
        torch.cuda.set_device(0)
        return protocol(args)
    import numpy as np
    import torch
    import torch.distributed as dist

    import blazingmq_amd as bmq
    from blazingmq_amd import Crc32c

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    # BENCH_DEVICE pins every rank to one GPU: only for rehearsing the
    # multi-process path on a one-GPU box.  Such a line is marked
    # "rehearsal_single_gpu" and reports n_gpus 1, never a scaling point.
    rehearsal = "BENCH_DEVICE" in os.environ
    local = int(os.environ.get("BENCH_DEVICE", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    desc, gen, seed, scaling = CONFIGS[args.config]
    if args.msgs or args.msg_bytes:
        size = args.msg_bytes or UNIFORM_SIZES[args.config]  # KeyError: uniform configs only
        n_msgs = args.msgs or int(UNIFORM_SIZES[args.config] * len(gen(0, 1)[0]) // size)
        gen = _uniform(n_msgs, size)
        desc = "EXPERIMENT (not the BASELINE workload): %d msgs x %d B" % (n_msgs, size)
    if args.shard:
        if world > 1:
            raise SystemExit("--shard is a one-process experiment")
        si, sn = (int(x) for x in args.shard.split("/"))
        lens_np, begin = gen(si, sn)
        desc = "EXPERIMENT (not the BASELINE workload): shard %d of %d of %s" % (si, sn, desc)
    else:
        lens_np, begin = gen(rank, world)
    n = int(lens_np.size)
    offs_np = np.zeros(n, dtype=np.int64)
    span = lens_np.astype(np.int64)
    if args.align > 1:
        span = (span + args.align - 1) // args.align * args.align
        desc = "EXPERIMENT (not the BASELINE workload): %s, messages %d-byte aligned" % (
            desc, args.align)
    if n > 1:
        np.cumsum(span[:-1], dtype=np.int64, out=offs_np[1:])
    total_bytes = int(lens_np.sum(dtype=np.uint64))
    arena_bytes = int(offs_np[-1] + lens_np[-1]) if n else 0
    # This rank's messages are bytes [begin, begin + total) of synthetic stream
    # `seed`, generated in HBM; offsets are relative to the rank's arena.
    stream = torch.cuda.current_stream(dev)
    rotate = max(1, args.rotate)
    copies = []  # --rotate: N independent copies of the batch, one per step in turn
    for _ in range(rotate):
        arena = torch.empty(max(arena_bytes, 8), dtype=torch.uint8, device=dev)
        _fill_slice(bmq, arena, seed, begin)
        copies.append((arena, torch.from_numpy(offs_np).to(dev),
                       torch.from_numpy(lens_np.view(np.int32)).to(dev),
                       torch.empty(n, dtype=torch.int32, device=dev)))
    arena, offsets, lengths, out = copies[0]
    torch.cuda.synchronize(dev)

    if args.e2e:
        return e2e(args, dev, stream, arena, offs_np, lens_np, total_bytes, world, rank, dist,
                   desc)

    turn = [0]

    def step(timed, plan=False, max_len=0, min_len=0):
        nonlocal out
        arena_i, offsets_i, lengths_i, out = copies[turn[0] % rotate]
        turn[0] += 1
        Crc32c.calculate_batch(arena_i, offsets_i, lengths_i, None, out,
                               seg_bytes=args.seg_bytes, stream=stream, sync=False,
                               time_kernel=timed, whole_messages=args.whole_messages, plan=plan,
                               max_len=max_len, min_len=min_len)

    # setup: settle the GPU clocks under this exact load (not part of W or K)
    t_settle = time.perf_counter()
    while time.perf_counter() - t_settle < args.settle_seconds:
        step(False)
        torch.cuda.synchronize(dev)
    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize(dev)
    bmq.kernel_timing(local, stream)  # reset
    wait_us = 100 if args.plan_wait_us is None else args.plan_wait_us
    voided0 = bmq.plan_wait(local, stream, wait_us)  # given-up planner maps so far

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(False)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    launch = bmq.last_launch(local, stream)  # the steady-state step's launch plan
    voided1 = bmq.plan_wait(local, stream, wait_us)
    # The same K steps with the shape prediction off (BMQCRC_F_PLAN): what a
    # caller whose batch shapes alternate on one stream pays per batch.
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(False, plan=True)
    torch.cuda.synchronize(dev)
    planned = time.perf_counter() - t0
    planned_launch = bmq.last_launch(local, stream)
    voided2 = bmq.plan_wait(local, stream, wait_us)
    # ... and with the prediction dropped before every step but the batch's
    # length bounds declared (bmqcrc_opts.max_len / min_len, ABI 2.4 / 2.5): what a
    # caller that knows its message sizes pays when shapes alternate.
    max_len = int(lens_np.max()) if n else 0
    min_len = int(lens_np.min()) if n else 0
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        bmq.forget_shape(local, stream)
        step(False, max_len=max_len, min_len=min_len)
    torch.cuda.synchronize(dev)
    declared = time.perf_counter() - t0
    declared_launch = bmq.last_launch(local, stream)
    if world > 1:
        dist.barrier()
    step(False)  # back to the predicted shape
    # Second timed pass of the same K steps with HIP events recorded around
    # the dominant kernel (k_fold) on its launch stream: its average duration
    # prices the roofline (events add launch gaps, so `value` comes from the
    # clean pass above).
    if not args.no_kernel_timing:
        for _ in range(args.steps):
            step(True)
        torch.cuda.synchronize(dev)
    kern_ms, kern_cnt = bmq.kernel_timing(local, stream)
    del arena, copies  # the strong-scaling leg below needs the memory
    bytes_all = total_bytes
    kern_max = kern_ms / max(kern_cnt, 1)
    plan_voided = [voided1 - voided0, voided2 - voided1]
    if world > 1:
        vt = torch.tensor(plan_voided, dtype=torch.int64)
        dist.all_reduce(vt)
        plan_voided = [int(vt[0]), int(vt[1])]
        tt = torch.tensor([elapsed, kern_max, planned, declared], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed, kern_max, planned, declared = (float(tt[0]), float(tt[1]), float(tt[2]),
                                                float(tt[3]))
        bt = torch.tensor([total_bytes, n], dtype=torch.int64)
        dist.all_reduce(bt)
        bytes_all, n_all = int(bt[0]), int(bt[1])
    else:
        n_all = n

    # parity spot check against the CPU oracle (sampled messages)
    import oracle
    got = out.cpu().numpy().view(np.uint32)
    rng = np.random.default_rng(rank)
    idx = np.unique(np.concatenate([[0, n - 1], rng.integers(0, n, size=max(0, args.check - 2))]))
    budget = 256 << 20  # bytes of payload regenerated on the host for checking
    bad, checked = 0, 0
    for i in idx:
        ln = int(lens_np[i])
        if checked and ln > budget:
            continue
        budget -= ln
        exp = oracle.crc32c(oracle.fill_payload(begin + int(offs_np[i]), ln, seed), 0, "hw")
        bad += int(got[i] != exp)
        checked += 1
    if world > 1:
        bt = torch.tensor([bad, checked], dtype=torch.int64)
        dist.all_reduce(bt)
        bad, checked = int(bt[0]), int(bt[1])
    strong = None
    if world > 1 and not args.no_strong_scaling and not args.config_given:
        strong = strong_scaling(args, bmq, Crc32c, dev, stream, world, rank, dist)
        bad += strong.pop("_bad")

    if rank == 0:
        value = bytes_all / 2**30 * args.steps / elapsed
        avg_kern_s = kern_max / 1e3 if kern_cnt else float("nan")
        alg_bytes = total_bytes + 4 * n  # this GPU's payload read once + CRCs written
        achieved = alg_bytes / avg_kern_s / 1e9
        traffic, traffic_src = pmc_traffic(args.config)
        res = {
            "metric": "device-resident CRC32C GiB/s over batched payloads, 1/2/4/8 MI355X",
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": 1 if rehearsal else world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 4),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (splitmix64 random payload bytes generated in HBM)",
            "config": {"workload": args.config + ": " + desc
                       + ("; steps rotate over %d copies of the batch (%.0f MiB, past the "
                          "256 MiB Infinity Cache)" % (rotate, rotate * (total_bytes + 16 * n)
                                                       / 2**20) if rotate > 1 else ""),
                       "n_msgs_total": n_all, "payload_bytes_total": bytes_all,
                       "seg_bytes": args.seg_bytes or "auto",
                       "whole_messages": bool(args.whole_messages),
                       "parallelism": "dp%d (sharded batch, no collective)" % world},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": "k_fold", "kernel_avg_us": round(avg_kern_s * 1e6, 2),
                         "kernel_time_source": "HIP events around each k_fold launch on its "
                                               "stream, K extra steps (event-priced: includes "
                                               "the launch gap, so frac is a lower bound; the "
                                               "traced kernel time is in profiles/)",
                         "frac_per_step": round(alg_bytes / (elapsed / args.steps) / 1e9
                                                / HBM_PEAK_GBS, 4),
                         "alg_bytes_per_launch": alg_bytes},
            "parity": {"checked_msgs": checked, "mismatches": bad},
            "kernels_per_step": launch["kernels"],
            "speculative_segments_per_msg": launch["spec"],
            "planned_ms_per_step": round(1e3 * planned / args.steps, 4),
            "planned_value": round(bytes_all / 2**30 * args.steps / planned, 2),
            "planned_kernels_per_step": planned_launch["kernels"],
            # single-pass planner launches (all ranks) whose size-class map was
            # given up, in the K timed steps and in the K planned steps
            "plan_voided": plan_voided[0],
            "planned_plan_voided": plan_voided[1],
            "plan_wait_us": wait_us,
        }
        # the bounds buy one launch only when every length in them has the
        # same u segments, u dividing 64; otherwise an in-flight batch may
        # restore the dropped prediction mid-loop, so the leg is not reported
        sb = max(declared_launch["seg_bytes"], 1)
        u_hi, u_lo = (max_len - 1) // sb + 1, (max(min_len, 1) - 1) // sb + 1
        if max_len and (u_hi == 1 or (min_len and u_hi == u_lo and 64 % u_hi == 0)):
            res.update({"declared_max_len": max_len, "declared_min_len": min_len,
                        "declared_ms_per_step": round(1e3 * declared / args.steps, 4),
                        "declared_kernels_per_step": declared_launch["kernels"]})
        if rehearsal:
            res["rehearsal_single_gpu"] = True
            res["ranks_on_one_gpu"] = world
        if strong is not None:
            if rehearsal:  # N ranks on one GPU: not a scaling point
                strong["n_gpus"] = 1
                strong["ranks_on_one_gpu"] = world
            res["strong_scaling"] = strong
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(lens_np, seed, args.cpu_seconds, dev.index or 0)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 1 if bad else 0


def strong_scaling(args, bmq, Crc32c, dev, stream, world, rank, dist):
    """BASELINE configs[3] strong-scaled: the Zipf 4M
    batch split byte-balanced over the `world` ranks (no collective), K steps
    timed like the main line (barriers, max over ranks); then, in the same
    run, the whole batch on rank 0's GPU alone (the N=1 time) while the other
    ranks wait.  speedup = t(1 GPU) / t(N GPUs); targets >= 3.5x at 4, >= 7x
    at 8.  A sampled parity check of both legs against the oracle."""
    import numpy as np
    import oracle
    import torch
    _, gen, seed, _ = CONFIGS["zipf_4M"]

    def leg(lens_np, begin, active):
        n = int(lens_np.size)
        offs_np = np.zeros(n, dtype=np.int64)
        if n > 1:
            np.cumsum(lens_np[:-1], dtype=np.int64, out=offs_np[1:])
        total = int(lens_np.sum(dtype=np.uint64))
        elapsed, bad, checked = 0.0, 0, 0
        if active:
            arena = torch.empty(max(total, 8), dtype=torch.uint8, device=dev)
            _fill_slice(bmq, arena, seed, begin)
            offsets = torch.from_numpy(offs_np).to(dev)
            lengths = torch.from_numpy(lens_np.view(np.int32)).to(dev)
            out = torch.empty(n, dtype=torch.int32, device=dev)

            def step():
                Crc32c.calculate_batch(arena, offsets, lengths, None, out, stream=stream,
                                       sync=False)
            t_settle = time.perf_counter()
            while time.perf_counter() - t_settle < args.settle_seconds / 2:
                step()
                torch.cuda.synchronize(dev)
            for _ in range(args.warmup):
                step()
            torch.cuda.synchronize(dev)
        dist.barrier()
        if active:
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize(dev)
            elapsed = time.perf_counter() - t0
        dist.barrier()
        if active:
            got = out.cpu().numpy().view(np.uint32)
            rng = np.random.default_rng(100 + rank)
            for i in np.unique(np.concatenate([[0, n - 1], rng.integers(0, n, size=62)])):
                exp = oracle.crc32c(oracle.fill_payload(begin + int(offs_np[i]), int(lens_np[i]),
                                                        seed), 0, "hw")
                bad += int(got[i] != exp)
                checked += 1
            del arena, offsets, lengths, out
            torch.cuda.empty_cache()
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)       # the slowest rank's window
        tb = torch.tensor([total, bad, checked], dtype=torch.int64)
        dist.all_reduce(tb)                            # bytes and mismatches summed
        return float(t[0]), int(tb[1]), int(tb[0]), int(tb[2])

    lens_r, begin_r = gen(rank, world)
    t_n, bad_n, bytes_n, chk_n = leg(lens_r, begin_r, True)
    lens_1, begin_1 = gen(0, 1) if rank == 0 else (np.zeros(1, np.uint32), 0)
    t_1, bad_1, _, chk_1 = leg(lens_1, begin_1, rank == 0)
    gib = bytes_n / 2**30 * args.steps
    return {"config": "zipf_4M: " + CONFIGS["zipf_4M"][0], "scaling": "strong",
            "value": round(gib / t_n, 2), "unit": "GiB/s", "n_gpus": world,
            "ms_per_step": round(1e3 * t_n / args.steps, 4),
            "one_gpu_value": round(gib / t_1, 2),
            "one_gpu_ms_per_step": round(1e3 * t_1 / args.steps, 4),
            "speedup": round(t_1 / t_n, 3), "payload_bytes_total": bytes_n,
            "one_gpu_leg": "the whole batch on rank 0's GPU in the same run",
            "parity": {"checked_msgs": chk_n + chk_1, "mismatches": bad_n + bad_1},
            "_bad": bad_n + bad_1}


def e2e(args, dev, stream, arena_dev, offs_np, lens_np, total_bytes, world, rank, dist, desc):
    """End-to-end: the payload starts in host memory (broker blob buffers) and
    the CRCs end there.  Two ways in, both timed per step (K steps after W):
      staged    -- pinned host arena, H2D copy + batch CRC + D2H of the CRCs;
      zero_copy -- ordinary host memory registered with bmqcrc_host_register,
                   the kernels read it in place over PCIe, + D2H of the CRCs.
    Reported in DESIGN.md, never as the bench `value`."""
    import numpy as np
    import torch
    from blazingmq_amd import Crc32c, HostRegistration, calculate_batch_ptr
    n = lens_np.size
    host = torch.empty(arena_dev.numel(), dtype=torch.uint8, pin_memory=True)
    host.copy_(arena_dev)
    offsets = torch.from_numpy(offs_np).to(dev)
    lengths = torch.from_numpy(lens_np.view("int32")).to(dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    out_host = torch.empty(n, dtype=torch.int32, pin_memory=True)

    def timed(step):
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize(dev)
        return time.perf_counter() - t0

    def staged():
        arena_dev.copy_(host, non_blocking=True)
        Crc32c.calculate_batch(arena_dev, offsets, lengths, None, out, seg_bytes=args.seg_bytes,
                               stream=stream, sync=False)
        out_host.copy_(out, non_blocking=True)

    el = timed(staged)
    ref = out_host.numpy().copy()
    h2d = timed(lambda: arena_dev.copy_(host, non_blocking=True))

    pageable = np.empty(arena_dev.numel(), dtype=np.uint8)  # ordinary malloc'd host memory
    pageable[:] = host.numpy()
    with HostRegistration(pageable, device=dev.index) as reg:
        def zero_copy():
            calculate_batch_ptr(reg.dev_ptr, reg.nbytes, offsets, lengths, None, out,
                                seg_bytes=args.seg_bytes, stream=stream, sync=False)
            out_host.copy_(out, non_blocking=True)
        el_zc = timed(zero_copy)
    zc = out_host.numpy().copy()
    resident = Crc32c.calculate_batch(arena_dev, offsets, lengths, seg_bytes=args.seg_bytes,
                                      stream=stream).cpu().numpy()
    same = bool(np.array_equal(zc, ref))
    if not same:
        bad = np.nonzero(zc != ref)[0]
        print("e2e mismatch: %d of %d (first %s); staged vs resident %d, zero-copy vs resident %d"
              % (bad.size, n, bad[:8].tolist(), int((ref != resident).sum()),
                 int((zc != resident).sum())), file=sys.stderr, flush=True)
    gib = total_bytes / 2**30 * args.steps
    if rank == 0:
        print(json.dumps({
            "metric": "end-to-end CRC32C GiB/s, payload in host memory, CRCs back to host",
            "value": round(gib * world / el, 2), "unit": "GiB/s",
            "n_gpus": world, "steps": args.steps, "config": args.config + ": " + desc,
            "staged_pinned_GiBps": round(gib / el, 2),
            "h2d_only_GiBps": round(gib / h2d, 2),
            "zero_copy_GiBps": round(gib / el_zc, 2),
            "zero_copy_matches_staged": same,
            "ms_per_step": round(1e3 * el / args.steps, 3),
            "ms_per_step_zero_copy": round(1e3 * el_zc / args.steps, 3)}), flush=True)
    return 0 if same else 1


def _fill_slice(bmq, arena, seed, begin):
    """Fill `arena` with bytes [begin, begin+len) of synthetic stream `seed`."""
    bmq.fill_synthetic(arena, seed, begin=begin)


if __name__ == "__main__":
    sys.exit(main())
