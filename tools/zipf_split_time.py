#!/usr/bin/env python3
"""Zipf 4M split by message size (GPU box): the whole batch, then only its
messages <= S bytes and only those > S (same arena, same offsets), each
timed steady-state with HIP events around the call (planner + k_fold), to
see how Zipf's time divides between its many small and few large messages.

  usage: python3 tools/zipf_split_time.py [--seg B] [S=2048 ...]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import bench
    from blazingmq_amd import Crc32c, fill_synthetic
    dev = torch.device("cuda", 0)
    lens, _ = bench._zipf(0, 1)
    offs = np.zeros(lens.size, dtype=np.int64)
    np.cumsum(lens[:-1], dtype=np.int64, out=offs[1:])
    arena = torch.empty(int(lens.sum(dtype=np.uint64)) + 64, dtype=torch.uint8, device=dev)
    fill_synthetic(arena, 4)
    s = torch.cuda.Stream(dev)
    args = sys.argv[1:]
    seg = 0
    if args[:1] == ["--seg"]:
        seg, args = int(args[1]), args[2:]
    cuts = [int(x) for x in args] or [2048]
    kw = {"seg_bytes": seg} if seg else {}

    def timed(mask, tag):
        ln = lens[mask]
        o = torch.from_numpy(offs[mask]).to(dev)
        lt = torch.from_numpy(ln.view(np.int32)).to(dev)
        out = torch.empty(ln.size, dtype=torch.int32, device=dev)
        for _ in range(5):
            Crc32c.calculate_batch(arena, o, lt, None, out, stream=s, sync=False, **kw)
        s.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        e0.record(s)
        for _ in range(reps):
            Crc32c.calculate_batch(arena, o, lt, None, out, stream=s, sync=False, **kw)
        e1.record(s)
        s.synchronize()
        us = 1000.0 * e0.elapsed_time(e1) / reps
        b = int(ln.sum(dtype=np.uint64))
        print(json.dumps({"subset": tag, "seg_bytes": seg or "auto", "msgs": int(ln.size), "bytes": b, "us_per_call": round(us, 1),
                          "alg_frac_of_8TBps": round((b + 4 * ln.size) / us / 8e6, 4)}), flush=True)

    timed(np.ones(lens.size, bool), "whole")
    for c in cuts:
        timed(lens <= c, "len<=%d" % c)
        timed(lens > c, "len>%d" % c)


if __name__ == "__main__":
    main()
