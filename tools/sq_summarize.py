#!/usr/bin/env python3
"""Summarise tools/sq_small.sh output: per shape and pass, the k_fold
counters averaged over dispatches, LDS-array busy and bank-conflict shares,
per-group instruction counts (pass A) and each counter's share of wave
cycles (pass B).  Writes <dir>/sq_summary.jsonl and copies the per-dispatch
CSVs next to it (rocprofv3 output names).

usage: sq_summarize.py <gpurun_out dir> <profiles dest dir> [kernel substring]
"""
import csv
import glob
import json
import os
import shutil
import sys

XCDS, CUS = 8, 256


def main(src, dst, kname="k_fold"):
    os.makedirs(dst, exist_ok=True)
    lines = []
    for d in sorted(glob.glob(os.path.join(src, "[AB]_*_*"))):
        if not os.path.isdir(d):
            continue
        p, msgs, nbytes = os.path.basename(d).split("_")
        f = os.path.join(d, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        rows = [r for r in csv.DictReader(open(f)) if kname in r["Kernel_Name"]]
        per = {}
        for r in rows:
            per.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
            per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
        avg = {k: sum(v.values()) / len(v) for k, v in per.items()}
        nd = len(next(iter(per.values()))) if per else 0
        groups = int(msgs) / 64
        line = {"pass": p, "msgs": int(msgs), "msg_bytes": int(nbytes), "dispatches": nd,
                "avg": {k: round(v) for k, v in sorted(avg.items())}}
        if "GRBM_GUI_ACTIVE" in avg:
            line["kernel_cycles_per_xcd"] = round(avg["GRBM_GUI_ACTIVE"] / XCDS)
        if p == "A":
            kc = avg["GRBM_GUI_ACTIVE"] / XCDS
            line["lds_busy_frac_per_cu"] = round(avg["SQ_LDS_IDX_ACTIVE"] / CUS / kc, 3)
            line["bank_conflict_share_of_lds_cycles"] = round(
                avg["SQ_LDS_BANK_CONFLICT"] / avg["SQ_LDS_IDX_ACTIVE"], 3)
            line["per_group"] = {"valu": round(avg["SQ_INSTS_VALU"] / groups),
                                 "lds_insts": round(avg["SQ_INSTS_LDS"] / groups, 1),
                                 "lds_cycles": round(avg["SQ_LDS_IDX_ACTIVE"] / groups),
                                 "conflict_cycles": round(avg["SQ_LDS_BANK_CONFLICT"] / groups)}
            line["waves_per_simd"] = round(avg["SQ_WAVES"] / (CUS * 4), 2)
        else:
            wc = avg["SQ_WAVE_CYCLES"]
            line["share_of_wave_cycles"] = {k: round(avg[k] / wc, 3) for k in sorted(avg)
                                            if k.startswith("SQ_") and k not in
                                            ("SQ_WAVE_CYCLES", "SQ_INSTS_SALU")}
            line["salu_per_group"] = round(avg.get("SQ_INSTS_SALU", 0) / groups)
        lines.append(line)
        shutil.copyfile(f, os.path.join(dst, "%s_%s_%s_%s.csv" % (p, msgs, nbytes, kname)))
    with open(os.path.join(dst, "sq_summary.jsonl"), "w") as fo:
        for l in lines:
            fo.write(json.dumps(l) + "\n")
            print(json.dumps(l))


if __name__ == "__main__":
    main(*sys.argv[1:])
