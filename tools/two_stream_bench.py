#!/usr/bin/env python3
"""Two batches in flight on two HIP streams of one process (the library keeps
one workspace per (device, stream)), against the same batches back to back on
one stream: how much of a single stream's step is batch-boundary idle time
(planner launch, k_fold ramp-up and drain).  Headline shape, 64k x 64 KiB per
batch.  GPU box only; prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import blazingmq_amd as bmq  # noqa: E402
from blazingmq_amd import Crc32c  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    n, size, steps = 65536, 65536, 40
    lens = torch.full((n,), size, dtype=torch.int32, device=dev)
    offs = torch.arange(n, dtype=torch.int64, device=dev) * size
    arenas = [torch.empty(n * size + 8, dtype=torch.uint8, device=dev) for _ in range(2)]
    for i, a in enumerate(arenas):
        bmq.fill_synthetic(a, 2 + i)
    outs = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(2)]
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]

    def run(two):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for k in range(steps):
            j = k % 2 if two else 0
            Crc32c.calculate_batch(arenas[k % 2], offs, lens, None, outs[k % 2],
                                   stream=streams[j], sync=False)
        torch.cuda.synchronize(dev)
        return time.perf_counter() - t0

    for two in (False, True):  # warm-up both paths
        run(two)
    res = {}
    for two in (False, True, False, True):
        t = run(two)
        key = "two_streams" if two else "one_stream"
        res.setdefault(key, []).append(round(steps * n * size / 2**30 / t, 1))
    ref = [Crc32c.calculate_batch(arenas[i], offs, lens, None).cpu() for i in range(2)]
    same = all(torch.equal(ref[i], outs[i].cpu()) for i in range(2))
    print(json.dumps({"shape": "64k x 64 KiB per batch", "steps": steps,
                      "GiBps_one_stream": res["one_stream"], "GiBps_two_streams": res["two_streams"],
                      "results_equal": same}))


if __name__ == "__main__":
    main()
