#!/usr/bin/env python3
"""CPU baseline table: the reference-equivalent CPU
CRC32C -- oracle/crc32c_oracle.c's restatement of bdlde::Crc32c, since BDE
4.39 is not available offline -- timed on this host for every BASELINE.json
config, three variants, one thread and T threads (one per core over
byte-balanced message slices, the reference's test5 pattern).

Each config is sampled like bench.py's cpu_baseline leg: its first messages up
to ~256 MiB (the whole batch when smaller), same synthetic bytes.  Prints one
JSON line per (config, variant, threads).

    python3 tools/cpu_baseline.py [--threads 16] [--seconds 0.5] [config ...]
"""
import argparse
import json
import os
import platform
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import bench  # noqa: E402
import oracle  # noqa: E402

VARIANTS = {"hw": "SSE4.2 crc32q 3-way interleaved (bdlde::Crc32c::calculate default)",
            "hw_serial": "SSE4.2 crc32q serial (calculateHardwareSerial)",
            "sw": "slicing-by-8 software (calculateSoftware)"}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--threads", type=int, default=min(os.cpu_count() or 1, 16))
    p.add_argument("--seconds", type=float, default=0.5, help="target wall time per measurement")
    p.add_argument("--sample-mib", type=int, default=256)
    p.add_argument("configs", nargs="*", default=list(bench.CONFIGS))
    a = p.parse_args()
    for cfg in a.configs:
        desc, gen, seed, _ = bench.CONFIGS[cfg]
        lens_all, begin = gen(0, 1)
        csum = np.cumsum(lens_all, dtype=np.uint64)
        n = max(1, int(np.searchsorted(csum, a.sample_mib << 20, side="right")))
        lens = np.ascontiguousarray(lens_all[:n])
        offs = np.zeros(n, dtype=np.uint64)
        if n > 1:
            offs[1:] = csum[:n - 1]
        nbytes = int(lens.sum(dtype=np.uint64))
        arena = oracle.fill_payload(begin, nbytes, seed)
        # parity before timing: the sampled CRCs of every variant agree
        ref = oracle.batch(arena, offs, lens, nthreads=a.threads, variant="hw")
        for var in VARIANTS:
            got = oracle.batch(arena, offs, lens, nthreads=a.threads, variant=var)
            assert np.array_equal(got, ref), (cfg, var)
            for th in sorted({1, a.threads}):
                t, _ = oracle.time_batch(arena, offs, lens, th, var, 1)
                reps = max(1, int(a.seconds / max(t, 1e-6)))
                t, _ = oracle.time_batch(arena, offs, lens, th, var, reps)
                print(json.dumps({
                    "config": cfg, "variant": var, "variant_desc": VARIANTS[var],
                    "threads": th, "GiBps": round(nbytes / 2**30 * reps / t, 3),
                    "sample_msgs": n, "sample_MiB": round(nbytes / 2**20, 1), "passes": reps,
                    "host": bench.cpu_model(), "nproc": os.cpu_count(),
                    "machine": platform.machine()}), flush=True)


if __name__ == "__main__":
    main()
