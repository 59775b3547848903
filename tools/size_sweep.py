#!/usr/bin/env python3
"""k_fold time and step rate vs message size at a fixed 256 MiB batch, planned
and BMQCRC_F_WHOLE_MESSAGES, one JSON line per point (GPU box)."""
import os, sys, json, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np, torch
import blazingmq_amd as bmq
from blazingmq_amd import Crc32c
dev = torch.device("cuda", 0)
total = 256 << 20
arena = torch.empty(total + 4096, dtype=torch.uint8, device=dev)
bmq.fill_synthetic(arena, 1)
s = torch.cuda.current_stream(dev)
for size in (64, 128, 256, 512, 1024, 2048, 4096, 16384, 65536):
    n = total // size
    offs = torch.arange(n, dtype=torch.int64, device=dev) * size
    lens = torch.full((n,), size, dtype=torch.int32, device=dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    for whole in (False, True):
        for _ in range(20):
            Crc32c.calculate_batch(arena, offs, lens, None, out, stream=s, sync=False, whole_messages=whole)
        torch.cuda.synchronize()
        bmq.kernel_timing(0, s)
        t0 = time.perf_counter()
        K = 30
        for _ in range(K):
            Crc32c.calculate_batch(arena, offs, lens, None, out, stream=s, sync=False, whole_messages=whole)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / K
        for _ in range(K):
            Crc32c.calculate_batch(arena, offs, lens, None, out, stream=s, sync=False, time_kernel=True, whole_messages=whole)
        torch.cuda.synchronize()
        ms, cnt = bmq.kernel_timing(0, s)
        kus = ms / cnt * 1e3
        print(json.dumps({"size": size, "n": n, "whole": whole, "step_us": round(el * 1e6, 2),
                          "GiBps": round(total / 2**30 / el, 1), "k_fold_us": round(kus, 2),
                          "k_fold_TBps": round((total + 4 * n) / kus / 1e6, 3)}), flush=True)
