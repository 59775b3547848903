#!/usr/bin/env python3
"""Device-resident CRC32C GiB/s over batched payloads on 1/2/4/8 MI355X.

Metric and configs: BASELINE.json.  A "step" is one bmqcrc_crc32c_batch call
(planner kernels + fold kernel) over one resident batch.  Default workload
(N=1) is configs[2]: 65,536 messages x 64 KiB of synthetic random payload
(splitmix64 stream, seed 2) -- the headline HBM-bound regime.  With
--gpus N (torchrun, one process per GPU) every rank CRCs its own 64k x 64 KiB
slice of an N-times larger batch (weak scaling, no data-path collective; a
gloo barrier brackets the timed region and the time is the max over ranks).

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

CONFIGS = {
    # name: (n_msgs, msg_bytes, seed)  -- BASELINE.json configs[1], [2], [4]
    "64k_x_64KiB": (65536, 65536, 2),
    "1M_x_256B": (1 << 20, 256, 1),
    "16_x_256MiB": (16, 256 << 20, 5),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--config", default="64k_x_64KiB", choices=sorted(CONFIGS))
    p.add_argument("--seg-bytes", type=int, default=0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=2.0,
                   help="approximate wall time of the CPU-baseline sample")
    p.add_argument("--check", type=int, default=256, help="messages checked against the oracle")
    return p.parse_args()


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def cpu_baseline(msg_bytes, seed, seconds):
    """Reference-equivalent CPU CRC32C (oracle, SSE4.2 3-way; BDE 4.39 is not
    available offline) on a bounded sample of the same synthetic workload."""
    import numpy as np
    import oracle
    threads = min(os.cpu_count() or 1, 16)
    n = max(1, (256 << 20) // msg_bytes)  # 256 MiB sample of the same stream
    arena = oracle.fill_payload(0, n * msg_bytes, seed)
    offs = np.arange(n, dtype=np.uint64) * msg_bytes
    lens = np.full(n, msg_bytes, dtype=np.uint32)
    t1, _ = oracle.time_batch(arena, offs, lens, 1, "hw", 1)          # single thread
    t, _ = oracle.time_batch(arena, offs, lens, threads, "hw", 1)      # calibrate
    reps = max(1, int(seconds / max(t, 1e-6)))
    t, _ = oracle.time_batch(arena, offs, lens, threads, "hw", reps)
    gib = n * msg_bytes / 2**30
    return {
        "value": round(gib * reps / t, 3),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": "%d msgs x %d B (%.0f MiB) of the same synthetic stream, %d passes; "
                  "SSE4.2 crc32q 3-way interleaved (bdlde::Crc32c default analogue); "
                  "single-thread %.2f GiB/s; host %s, nproc %d"
                  % (n, msg_bytes, gib * 1024, reps, gib / t1, cpu_model(), os.cpu_count()),
    }


def pmc_traffic(config):
    """HBM bytes per k_fold launch from the newest committed rocprofv3 PMC
    summary of this config (profiles/rNN/<config>_summary.json): read =
    2 x FETCH_SIZE (gfx950 correction) + WRITE_SIZE, per MI355X_MICROARCH.md."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", config + "_summary.json")))
    if not paths:
        return None, None
    with open(paths[-1]) as f:
        s = json.load(f)
    return int(s["traffic_bytes_per_launch"]), os.path.relpath(paths[-1], ROOT)


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    import blazingmq_amd as bmq
    from blazingmq_amd import Crc32c

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    n, msg_bytes, seed = CONFIGS[args.config]
    total_bytes = n * msg_bytes
    # rank r owns messages [r*n, (r+1)*n) of the global batch: its slice of the
    # synthetic stream starts at byte r*n*msg_bytes.
    arena = torch.empty(total_bytes, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    # device-side fill of the rank's slice (begin offset via seed stream index)
    _fill_slice(bmq, arena, seed, rank * total_bytes)
    offsets = torch.arange(n, dtype=torch.int64, device=dev) * msg_bytes
    lengths = torch.full((n,), msg_bytes, dtype=torch.int32, device=dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)

    def step(timed):
        Crc32c.calculate_batch(arena, offsets, lengths, None, out, seg_bytes=args.seg_bytes,
                               stream=stream, sync=False, time_kernel=timed)

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize(dev)
    bmq.kernel_timing(local, stream)  # reset

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    kern_ms, kern_cnt = bmq.kernel_timing(local, stream)
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    # parity spot check against the CPU oracle (sampled messages)
    import oracle
    got = out.cpu().numpy().view(np.uint32)
    rng = np.random.default_rng(rank)
    idx = np.unique(np.concatenate([[0, n - 1], rng.integers(0, n, size=max(0, args.check - 2))]))
    bad = 0
    for i in idx:
        begin = rank * total_bytes + int(i) * msg_bytes
        exp = oracle.crc32c(oracle.fill_payload(begin, msg_bytes, seed), 0, "hw")
        bad += int(got[i] != exp)
    if world > 1:
        bt = torch.tensor([bad], dtype=torch.int64)
        dist.all_reduce(bt)
        bad = int(bt.item())

    if rank == 0:
        gib_all = world * total_bytes / 2**30
        value = gib_all * args.steps / elapsed
        avg_kern_s = (kern_ms / 1e3 / kern_cnt) if kern_cnt else float("nan")
        alg_bytes = total_bytes + 4 * n  # payload read once + CRC written
        traffic, traffic_src = pmc_traffic(args.config)
        achieved = alg_bytes / avg_kern_s / 1e9
        res = {
            "metric": "device-resident CRC32C GiB/s over batched payloads, 1/2/4/8 MI355X",
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (splitmix64 random bytes, generated in HBM)",
            "config": {"workload": "%s: %d msgs x %d B per GPU (BASELINE configs)"
                       % (args.config, n, msg_bytes), "n_msgs_per_gpu": n,
                       "msg_bytes": msg_bytes, "seg_bytes": args.seg_bytes or 16384,
                       "parallelism": "dp%d (sharded batch, no collective)" % world},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": "k_fold", "kernel_avg_us": round(avg_kern_s * 1e6, 2),
                         "alg_bytes_per_launch": alg_bytes},
            "parity": {"checked_msgs": int(len(idx)) * world, "mismatches": bad},
        }
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(msg_bytes, seed, args.cpu_seconds)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 1 if bad else 0


def _fill_slice(bmq, arena, seed, begin):
    """Fill `arena` with bytes [begin, begin+len) of synthetic stream `seed`."""
    bmq.fill_synthetic(arena, seed, begin=begin)


if __name__ == "__main__":
    sys.exit(main())
