#!/usr/bin/env python3
"""Per-block phase times of k_plan_map (GPU box, diagnostic build only).

Needs a library built with -DBMQCRC_PLAN_DIAG=3 or 4 (tools/build_variant.sh pd3
-DBMQCRC_PLAN_DIAG=3), swapped in as libbmqcrc.so by the caller.  Runs the
Zipf batch (or one shard of it) a few times, then reads the per-block
wall-clock stamps of the last planner launch (8 per block, see g_plan_trace;
100 MHz) and prints the spread of each phase over the blocks.

  usage: python3 tools/plan_trace_diag.py [i/N]
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import bench
    from blazingmq_amd import Crc32c, _native
    shard = sys.argv[1] if len(sys.argv) > 1 else "0/1"
    si, sn = (int(x) for x in shard.split("/"))
    lens, begin = bench._zipf(si, sn)
    n = lens.size
    offs = np.zeros(n, dtype=np.int64)
    np.cumsum(lens[:-1], dtype=np.int64, out=offs[1:])
    dev = torch.device("cuda", 0)
    arena = torch.empty(int(lens.sum(dtype=np.uint64)), dtype=torch.uint8, device=dev)
    import blazingmq_amd as bmq
    bench._fill_slice(bmq, arena, 4, begin)
    o = torch.from_numpy(offs).to(dev)
    ln = torch.from_numpy(lens.view(np.int32)).to(dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    for _ in range(8):
        Crc32c.calculate_batch(arena, o, ln, None, out, sync=False)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (256 * 8))()
    if _native.lib.bmqcrc_diag_plan_trace(buf) != 0:
        raise SystemExit("bmqcrc_diag_plan_trace failed")
    t = np.array(buf, dtype=np.float64).reshape(256, 8)
    t = t[t[:, 0] > 0]
    t0 = t[:, 0].min()
    us = (t - t0) / 100.0  # 100 MHz ticks -> microseconds
    res = {"shard": shard, "blocks": int(t.shape[0])}
    names = ["start", "loads_landed", "tile0_done", "phase1_done", "wait_done", "deferred_done",
             "bases_done", "end"]
    for k, name in enumerate(names):
        res[name + "_us"] = [round(float(us[:, k].min()), 2), round(float(np.median(us[:, k])), 2),
                             round(float(us[:, k].max()), 2)]
    for k in range(1, len(names)):
        res["d_" + names[k]] = [round(float(x), 2)
                                for x in np.percentile(us[:, k] - us[:, k - 1], [0, 50, 100])]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
