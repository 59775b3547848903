#!/usr/bin/env python3
"""Turn rocprofv3 output dirs (gpurun_out/<prefix>_<config>, <prefix>f_<config>,
<prefix>w_<config>) into committed summaries under profiles/<round>/:

  <config>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary
  <config>_pmc_fetch.csv      --pmc FETCH_SIZE per-dispatch counters
  <config>_pmc_write.csv      --pmc WRITE_SIZE per-dispatch counters
  <config>_summary.json       k_fold average duration, HBM bytes per launch
                              (read = 2 x FETCH_SIZE KB x 1024: gfx950 counts
                              half the bytes of a wide coalesced stream,
                              MI355X_MICROARCH.md HBM), algorithmic bytes.

Also records each config's traffic in bench_traffic.json (repo root), the
file bench.py's roofline.traffic reads on the GPU box.

usage: summarize_profiles.py <round dir> <prefix> <config>=<alg_bytes> ...
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


TRAFFIC = os.path.join(ROOT, "bench_traffic.json")


def record_traffic(cfg, s, summary_path):
    """bench_traffic.json (tracked, at the repo root so that it travels to
    the GPU box, where ./profiles is not sent): the newest PMC traffic per
    config, which bench.py's roofline.traffic reports with its source."""
    try:
        with open(TRAFFIC) as f:
            t = json.load(f)
    except (OSError, ValueError):
        t = {}
    t[cfg] = {"traffic_bytes_per_launch": int(s["traffic_bytes_per_launch"]),
              "alg_bytes_per_launch": int(s["alg_bytes_per_launch"]),
              "traffic_over_alg": round(s["traffic_over_alg"], 5),
              "source": os.path.relpath(summary_path, ROOT)}
    with open(TRAFFIC, "w") as f:
        json.dump(t, f, indent=1, sort_keys=True)
        f.write("\n")


def main(argv):
    out_dir, prefix = argv[1], argv[2]
    os.makedirs(out_dir, exist_ok=True)
    g = os.path.join(ROOT, "gpurun_out")
    for item in argv[3:]:
        cfg, alg = item.split("=")
        alg = int(alg)
        st_src = os.path.join(g, "%s_%s" % (prefix, cfg), "run_kernel_stats.csv")
        f_src = os.path.join(g, "%sf_%s" % (prefix, cfg), "run_counter_collection.csv")
        w_src = os.path.join(g, "%sw_%s" % (prefix, cfg), "run_counter_collection.csv")
        shutil.copyfile(st_src, os.path.join(out_dir, cfg + "_kernel_stats.csv"))
        shutil.copyfile(f_src, os.path.join(out_dir, cfg + "_pmc_fetch.csv"))
        shutil.copyfile(w_src, os.path.join(out_dir, cfg + "_pmc_write.csv"))
        fold = [r for r in csv.DictReader(open(st_src)) if "k_fold" in r["Name"]][0]
        fetch = [float(r["Counter_Value"]) for r in csv.DictReader(open(f_src))
                 if "k_fold" in r["Kernel_Name"]]
        write = [float(r["Counter_Value"]) for r in csv.DictReader(open(w_src))
                 if "k_fold" in r["Kernel_Name"]]
        rd = 2 * 1024 * sum(fetch) / len(fetch)
        wr = 1024 * sum(write) / len(write)
        avg_us = float(fold["AverageNs"]) / 1e3
        s = {"config": cfg, "kernel": "k_fold", "calls": int(fold["Calls"]),
             "avg_duration_us": avg_us,
             "commands": ["rocprofv3 --kernel-trace --stats -- python3 bench.py --config %s" % cfg,
                          "rocprofv3 --pmc FETCH_SIZE --kernel-trace -- python3 bench.py ...",
                          "rocprofv3 --pmc WRITE_SIZE --kernel-trace -- python3 bench.py ..."],
             "FETCH_SIZE_KB": sum(fetch) / len(fetch), "WRITE_SIZE_KB": sum(write) / len(write),
             "hbm_read_bytes": rd, "hbm_write_bytes": wr,
             "correction": "read = 2 x FETCH_SIZE x 1024 (gfx950), write = WRITE_SIZE x 1024",
             "traffic_bytes_per_launch": rd + wr, "alg_bytes_per_launch": alg,
             "traffic_over_alg": (rd + wr) / alg,
             "achieved_alg_GBps": alg / avg_us / 1e3}
        with open(os.path.join(out_dir, cfg + "_summary.json"), "w") as f:
            json.dump(s, f, indent=1)
        record_traffic(cfg, s, os.path.join(out_dir, cfg + "_summary.json"))
        print(cfg, "avg %.1f us" % avg_us, "traffic/alg %.4f" % s["traffic_over_alg"],
              "alg %.0f GB/s" % s["achieved_alg_GBps"])


if __name__ == "__main__":
    main(sys.argv)
