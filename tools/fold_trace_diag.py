#!/usr/bin/env python3
"""Per-wave phase times of k_fold (GPU box, diagnostic build only).

Needs a library built with -DBMQCRC_FOLD_DIAG=1 (tools/build_variant.sh fd1
-DBMQCRC_FOLD_DIAG=1), swapped in as libbmqcrc.so by the caller.  Runs a
uniform batch (bench.py's configs, optionally --msgs / --msg-bytes) several
times, then reads the per-wave wall-clock stamps (100 MHz) of the last
k_fold launch and prints the spread of each phase over the waves: when the
waves start, their prologue (tables, planner words), the first descriptors
-> DMA issue, the first group's data landing and fold, the loop, the last
group's remainder and combine, and where the launch ends.

  usage: python3 tools/fold_trace_diag.py <config | zipf_4M[:i/N]> [msgs] [msg_bytes] [raw.npy]
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
    import blazingmq_amd as bmq
    from blazingmq_amd import Crc32c, _native
    cfg = sys.argv[1] if len(sys.argv) > 1 else "1M_x_256B"
    dev = torch.device("cuda", 0)
    if cfg.startswith("zipf"):  # zipf_4M or zipf_4M:i/N (one strong-scaling shard)
        si, sn = (int(x) for x in (cfg.split(":")[1] if ":" in cfg else "0/1").split("/"))
        lens, begin = bench._zipf(si, sn)
        n, size = int(lens.size), 0
        offs = np.zeros(n, dtype=np.int64)
        np.cumsum(lens[:-1], dtype=np.int64, out=offs[1:])
        arena = torch.empty(int(lens.sum(dtype=np.uint64)) + 64, dtype=torch.uint8, device=dev)
        bmq.fill_synthetic(arena, 4, begin=begin)
        o = torch.from_numpy(offs).to(dev)
        ln = torch.from_numpy(lens.view(np.int32)).to(dev)
    else:
        size = int(sys.argv[3]) if len(sys.argv) > 3 else bench.UNIFORM_SIZES[cfg]
        n = int(sys.argv[2]) if len(sys.argv) > 2 else len(bench.CONFIGS[cfg][1](0, 1)[0])
        arena = torch.empty(n * size + 64, dtype=torch.uint8, device=dev)
        bmq.fill_synthetic(arena, 1)
        o = torch.arange(n, dtype=torch.int64, device=dev) * size
        ln = torch.full((n,), size, dtype=torch.int32, device=dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev)
    for _ in range(50 if size else 8):
        Crc32c.calculate_batch(arena, o, ln, None, out, stream=s, sync=False)
    torch.cuda.synchronize()
    kw = 4096
    buf = (ctypes.c_ulonglong * (kw * 8))()
    if _native.lib.bmqcrc_diag_fold_trace(buf) != 0:
        raise SystemExit("bmqcrc_diag_fold_trace failed (not a FOLD_DIAG build?)")
    t = np.array(buf, dtype=np.float64).reshape(kw, 8)
    if len(sys.argv) > 4:  # raw stamps (wave-major, 8 per wave, 100 MHz ticks) for analysis
        np.save(sys.argv[4], t)
    t = t[t[:, 0] > 0]
    t0 = t[:, 0].min()
    us = (t - t0) / 100.0  # 100 MHz ticks -> microseconds
    res = {"config": cfg, "msgs": n, "msg_bytes": size, "waves": int(t.shape[0]),
           "launch_us": round(float(us[:, 6].max()), 2)}
    names = ["entry", "prologue_done", "first_issue", "first_group_folded", "last_lines_folded",
             "loop_done", "end"]
    for k, name in enumerate(names):
        res[name + "_us"] = [round(float(x), 2) for x in np.percentile(us[:, k], [0, 50, 100])]
    for k in range(1, len(names)):
        res["d_" + names[k]] = [round(float(x), 2)
                                for x in np.percentile(us[:, k] - us[:, k - 1], [0, 50, 100])]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
