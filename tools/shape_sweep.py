#!/usr/bin/env python3
"""k_fold time vs segment size and blocks per CU for a few batch shapes (GPU
box), one JSON line per point.  Explicit seg_bytes; the grid is forced to 1 / 2
blocks per CU by the variant builds variant_bpc1.so / variant_bpc2.so
(tools/build_variant.sh bpc1 -DBMQCRC_TUNE_BITS=2; bpc2 -DBMQCRC_TUNE_BITS=8),
swapped in as libbmqcrc.so for a child process per grid choice."""
import json
import os
import subprocess
import sys
import time

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SHAPES = [(4096, 65536), (65536, 4096), (16384, 16384), (1 << 18, 1024)]  # (n, size): 256 MiB
SEGS = [0, 1024, 2048, 4096, 8192, 16384, 65536]
if os.environ.get("SHAPE_SWEEP_LARGE"):  # 1 and 2 GiB of 64 KiB messages
    SHAPES = [(16384, 65536), (32768, 65536)]
    SEGS = [0, 2048, 4096, 8192, 16384, 32768, 65536]


def child(n, size, seg):
    sys.path.insert(0, ROOT)
    import torch
    import blazingmq_amd as bmq
    from blazingmq_amd import Crc32c
    dev = torch.device("cuda", 0)
    arena = torch.empty(n * size + 4096, dtype=torch.uint8, device=dev)
    bmq.fill_synthetic(arena, 1)
    s = torch.cuda.current_stream(dev)
    offs = torch.arange(n, dtype=torch.int64, device=dev) * size
    lens = torch.full((n,), size, dtype=torch.int32, device=dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    for _ in range(20):
        Crc32c.calculate_batch(arena, offs, lens, None, out, stream=s, sync=False, seg_bytes=seg)
    torch.cuda.synchronize()
    bmq.kernel_timing(0, s)
    for _ in range(30):
        Crc32c.calculate_batch(arena, offs, lens, None, out, stream=s, sync=False, seg_bytes=seg,
                               time_kernel=True)
    torch.cuda.synchronize()
    ms, cnt = bmq.kernel_timing(0, s)
    return ms / cnt * 1e3


if __name__ == "__main__":
    if len(sys.argv) > 1:
        n, size, seg = map(int, sys.argv[1:4])
        print(child(n, size, seg))
        sys.exit(0)
    import shutil
    lib = os.path.join(ROOT, "blazingmq_amd", "lib")
    base = os.path.join("/tmp", "shape_sweep_base.so")
    shutil.copy(os.path.join(lib, "libbmqcrc.so"), base)
    for n, size in SHAPES:
        for bpc in (1, 2):
            shutil.copy(os.path.join(lib, "variant_bpc%d.so" % bpc), os.path.join(lib, "libbmqcrc.so"))
            for seg in SEGS:
                r = subprocess.run([sys.executable, __file__, str(n), str(size), str(seg)],
                                   capture_output=True, text=True, timeout=120)
                if r.returncode != 0:
                    shutil.copy(base, os.path.join(lib, "libbmqcrc.so"))
                    print(json.dumps({"n": n, "size": size, "seg": seg, "error": r.stderr[-300:]}))
                    sys.exit(1)
                us = float(r.stdout.strip().splitlines()[-1])
                print(json.dumps({"n": n, "size": size, "blocks_per_cu": bpc,
                                  "seg": seg or "auto", "k_fold_us": round(us, 2),
                                  "TBps": round(n * size / us / 1e6, 3)}), flush=True)
    shutil.copy(base, os.path.join(lib, "libbmqcrc.so"))
