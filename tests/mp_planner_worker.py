"""One process of the shared-GPU planner test (started by
tests/test_gpu_runtime.py::test_processes_share_the_planner_on_one_gpu, never
collected by pytest).  It CRCs a ragged batch of more than 1.4M messages (the
single-pass planner's size; its blocks meet grid-wide) on GPU 0 with the
library's default planner wait limit, `steps` times after every process is
ready, checks every CRC of every step against the oracle and prints one JSON
line: the median and fastest step, the mismatches and how many planner maps
were given up (bmqcrc_plan_wait's count).

usage: mp_planner_worker.py <worker id> <steps> <sync dir>
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    wid, steps, sync = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    import numpy as np
    import torch

    import oracle
    from blazingmq_amd import Crc32c, plan_wait
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    rng = np.random.default_rng(500 + wid)
    n = 1_400_000 + 1000 * wid
    lens = np.concatenate([rng.integers(0, 300, size=n - 300),
                           rng.integers(0, 200_000, size=300)]).astype(np.uint32)
    rng.shuffle(lens)
    arena_np = rng.integers(0, 256, size=32 << 20, dtype=np.uint8)
    offs = (rng.random(n) * (arena_np.size - lens + 1)).astype(np.int64)
    exp = oracle.batch(arena_np, offs, lens, None, nthreads=4)
    arena = torch.from_numpy(arena_np).to(dev)
    d_offs = torch.from_numpy(offs).to(dev)
    d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    s = torch.cuda.Stream(dev)

    def step():
        Crc32c.calculate_batch(arena, d_offs, d_lens, None, out, stream=s, sync=False)
        s.synchronize()
        return int(np.count_nonzero(out.cpu().numpy().view(np.uint32) != exp))

    bad = step()  # warm: workspace, shape history
    v0 = plan_wait(0, s)
    open(os.path.join(sync, "ready_%d" % wid), "w").close()
    go = os.path.join(sync, "go")
    t_wait = time.time()
    while not os.path.exists(go):
        if time.time() - t_wait > 120:
            raise SystemExit("no go signal")
        time.sleep(0.001)
    times = []
    for _ in range(steps):
        t0 = time.perf_counter()
        Crc32c.calculate_batch(arena, d_offs, d_lens, None, out, stream=s, sync=False)
        s.synchronize()
        times.append(time.perf_counter() - t0)
        bad += int(np.count_nonzero(out.cpu().numpy().view(np.uint32) != exp))
    voided = plan_wait(0, s) - v0
    times.sort()
    print(json.dumps({"worker": wid, "msgs": n, "steps": steps, "median_ms": 1e3 * times[len(times) // 2],
                      "min_ms": 1e3 * times[0], "mismatches": bad, "plan_voided": voided}),
          flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
