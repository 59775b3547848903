#!/usr/bin/env python3
"""Print value / step / roofline / parity from bench.py logs (last JSON line)."""
import json
import sys

for path in sys.argv[1:]:
    try:
        lines = [l for l in open(path) if l.startswith("{")]
        d = json.loads(lines[-1])
        r = d.get("roofline") or {}
        print("%-40s %9.2f %s  step %.4f ms  frac %s  k_fold %s us  parity %s" % (
            path, d["value"], d["unit"], d["ms_per_step"], r.get("frac"),
            r.get("kernel_avg_us"), d.get("parity")))
    except Exception as e:  # noqa: BLE001
        print("%-40s unreadable (%s)" % (path, e))
