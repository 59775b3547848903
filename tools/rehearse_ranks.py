#!/usr/bin/env python3
"""Rehearse `bench.py --gpus N` on a one-GPU box (every rank on GPU 0).

Starts `BENCH_DEVICE=0 python3 bench.py --gpus N ...` as a child process (it
starts its own N ranks), samples the host memory of the whole process tree
every 0.5 s, and writes one JSON summary: exit code, wall time, peak summed
RSS, and the bench line rank 0 printed.  The bench line says
"rehearsal_single_gpu": true and "ranks_on_one_gpu": N.

  usage (on the box): python3 tools/rehearse_ranks.py N OUT.json [bench args...]
"""
import json
import os
import subprocess
import sys
import time

import psutil


def tree_rss(proc):
    total = 0
    try:
        procs = [proc] + proc.children(recursive=True)
    except psutil.NoSuchProcess:
        return 0
    for p in procs:
        try:
            total += p.memory_info().rss
        except psutil.NoSuchProcess:
            pass
    return total


def main():
    n = int(sys.argv[1])
    out = sys.argv[2]
    extra = sys.argv[3:]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, BENCH_DEVICE="0")
    log = out + ".log"
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", str(n)] + extra
    t0 = time.time()
    peak = 0
    last_note = t0
    with open(log, "w") as f:
        child = subprocess.Popen(cmd, stdout=f, stderr=subprocess.STDOUT, env=env, cwd=root)
        ps = psutil.Process(child.pid)
        while child.poll() is None:
            peak = max(peak, tree_rss(ps))
            if time.time() - last_note > 30:
                last_note = time.time()
                print("rehearsal %d ranks: %.0f s, peak host RSS %.2f GiB"
                      % (n, last_note - t0, peak / 2**30), flush=True)
            time.sleep(0.5)
    wall = time.time() - t0
    line = None
    with open(log) as f:
        for ln in f:
            ln = ln.strip()
            if ln.startswith("{") and '"metric"' in ln:
                line = json.loads(ln)
    res = {"ranks": n, "rc": child.returncode, "wall_s": round(wall, 1),
           "peak_host_rss_gib": round(peak / 2**30, 2), "cmd": " ".join(cmd[1:]),
           "bench": line}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "bench"}))
    sys.exit(child.returncode)


if __name__ == "__main__":
    main()
