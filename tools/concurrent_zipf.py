#!/usr/bin/env python3
"""Concurrent ragged batches on one GPU: BASELINE configs[3] (Zipf 4M) split
byte-balanced into S parts, each part CRC'd on its own HIP stream (the
library keeps one workspace per (device, stream)), all S enqueued at once --
a broker recovering S partitions on S streams.  Against the same parts back
to back on one stream, and the whole batch on one stream with the planner's
map kept (default wait) and given up (plan_wait 0: the fallback's cost).

Per leg: wall time per step (K steps after W warm-up steps), the planner
launches whose size-class map was given up (bmqcrc_plan_wait's counter), and
every CRC compared with the whole-batch mapped result, which is itself
sample-checked against the oracle.  GPU box only; one JSON line per leg.

    python3 tools/concurrent_zipf.py [--streams 2,4] [--steps 10] [--warmup 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.environ.get("GRAFT_REPO_ROOT",
                      os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import blazingmq_amd as bmq  # noqa: E402
from blazingmq_amd import Crc32c  # noqa: E402
from blazingmq_amd.shard import rank_slice  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--streams", default="2,4")
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--seg-bytes", type=int, default=0, help="0: automatic")
    p.add_argument("--wait-us", default="100",
                   help="bmqcrc_plan_wait limits to run the concurrent legs with (comma list)")
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    _, gen, seed, _ = bench.CONFIGS["zipf_4M"]
    lens_np, begin = gen(0, 1)
    n = lens_np.size
    offs_np = np.zeros(n, dtype=np.int64)
    np.cumsum(lens_np[:-1], dtype=np.int64, out=offs_np[1:])
    total = int(lens_np.sum(dtype=np.uint64))
    arena = torch.empty(total, dtype=torch.uint8, device=dev)
    bmq.fill_synthetic(arena, seed, begin=begin)
    offs = torch.from_numpy(offs_np).to(dev)
    lens = torch.from_numpy(lens_np.view(np.int32)).to(dev)
    gib = total / 2**30

    def leg(name, parts, streams, wait_us):
        outs = [torch.empty(hi - lo, dtype=torch.int32, device=dev) for lo, hi in parts]
        for s in streams:
            bmq.plan_wait(0, s, wait_us)
        # each part is its own arena (a partition's DATA file): its bytes and
        # offsets relative to them, so the automatic shape sees the part's size
        views = []
        for lo, hi in parts:
            base = int(offs_np[lo]) if hi > lo else 0
            nb = int(offs_np[hi - 1]) + int(lens_np[hi - 1]) - base if hi > lo else 0
            views.append((arena[base:base + nb], offs[lo:hi] - base, lens[lo:hi]))

        def step():
            for (ar, of, ln), s, o in zip(views, streams, outs):
                Crc32c.calculate_batch(ar, of, ln, None, o, stream=s, sync=False,
                                       seg_bytes=a.seg_bytes)
        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize(dev)
        v0 = sum(bmq.plan_wait(0, s, wait_us) for s in set(streams))
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize(dev)
        dt = (time.perf_counter() - t0) / a.steps
        v1 = sum(bmq.plan_wait(0, s, wait_us) for s in set(streams))
        got = torch.cat(outs).cpu().numpy().view(np.uint32)
        return dt, v1 - v0, got

    one = torch.cuda.Stream(dev)
    waits = [int(x) for x in a.wait_us.split(",") if x]
    t_map, v_map, ref = leg("whole", [(0, n)], [one], waits[0])
    # the reference result: oracle-checked on a sample
    import oracle
    rng = np.random.default_rng(7)
    idx = np.unique(np.concatenate([[0, n - 1], rng.integers(0, n, size=254)]))
    bad = sum(int(ref[i] != oracle.crc32c(oracle.fill_payload(begin + int(offs_np[i]),
                                                              int(lens_np[i]), seed), 0, "hw"))
              for i in idx)

    def emit(leg_name, dt, voided, got, **kw):
        print(json.dumps(dict({
            "leg": leg_name, "ms_per_step": round(1e3 * dt, 4), "GiBps": round(gib / dt, 1),
            "plan_voided": voided, "steps": a.steps, "seg_bytes": a.seg_bytes or "auto",
            "equal_to_whole_mapped": bool(np.array_equal(got, ref))}, **kw)), flush=True)

    emit("whole_one_stream_mapped", t_map, v_map, ref, oracle_sample_mismatches=bad,
         oracle_sample=int(idx.size))
    t_void, v_void, got = leg("whole_void", [(0, n)], [one], 0)
    emit("whole_one_stream_map_given_up", t_void, v_void, got,
         ratio_to_mapped=round(t_void / t_map, 3))
    for S in [int(x) for x in a.streams.split(",") if x]:
        parts = [rank_slice(lens_np, r, S) for r in range(S)]
        streams = [torch.cuda.Stream(dev) for _ in range(S)]
        for w in waits:
            dt, v, got = leg("conc%d" % S, parts, streams, w)
            emit("%d_parts_%d_streams_at_once" % (S, S), dt, v, got, planner_launches=S * a.steps,
                 ratio_to_mapped=round(dt / t_map, 3), plan_wait_us=w)
        dt, v, got = leg("serial%d" % S, parts, [one] * S, waits[0])
        emit("%d_parts_one_stream" % S, dt, v, got, planner_launches=S * a.steps,
             ratio_to_mapped=round(dt / t_map, 3), plan_wait_us=waits[0])
    return 0


if __name__ == "__main__":
    sys.exit(main())
