#!/usr/bin/env python3
"""Attribute Zipf 4M's k_fold traffic above its algorithmic bytes (CPU model).

The batch (bench.py configs[3]) lays 4M messages of 64*r bytes back to back,
so every message boundary at 64 mod 128 cuts a 128-byte line that two
messages share.  k_fold folds the batch in size-class order, so the two
neighbours of a cut line are read by different groups, usually far apart in
time: under a 128-byte fetch granularity the line is fetched from HBM twice.
This model counts, for the whole batch and for each strong-scaling shard:
  * alg          = sum(len) + 4 N (the roofline's bytes)
  * lines_128    = sum over messages of the 128-byte lines each touches x 128
                   (every message fetching its own lines, nothing shared)
  * shared_lines = lines cut by a message boundary (fetched twice above)
  * meta         = descriptors (12 B/msg), seginfo (4 B/segment) + group
                   descriptors, out (4 B/msg read-modify... counted once)
  * desc_by_class = the 128-byte lines of `offsets` (8 B/msg) and `lengths`
                   (4 B/msg) each size class touches, summed over the classes:
                   k_fold reads descriptors in the sorted map's class order, a
                   class's messages are sparse in message order, and no cache
                   keeps a descriptor line from one class to the next (round 6)
and compares alg + meta + duplicated lines with the measured FETCH/WRITE
traffic of profiles/rNN/<...>/zipf_4M_summary.json.  With 128-byte aligned
messages (bench.py --align 128) the same model predicts the aligned run.

usage: python3 tools/zipf_overfetch.py [summary.json] [out.json]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def size_class(nl):
    """crc32c_kernels.hip size_class(): 16 buckets, lanes within 1.5x."""
    nl = nl | 1
    b = np.floor(np.log2(nl)).astype(np.int64)
    c = np.where(b > 0, 2 * b + ((nl >> np.maximum(b - 1, 0)) & 1), 0)
    return np.minimum(c, 15)


def desc_by_class(lens, seg=2048, align=0):
    """Descriptor bytes k_fold fetches when the map is read class by class:
    per class, the distinct 128-byte lines of offsets and lengths."""
    lens = lens.astype(np.int64)
    size = lens if not align else (lens + align - 1) // align * align
    off = np.zeros(lens.size, dtype=np.int64)
    np.cumsum(size[:-1], out=off[1:])
    nseg = (lens + seg - 1) // seg
    msg = np.repeat(np.arange(lens.size), nseg)
    k = np.arange(int(nseg.sum())) - np.repeat(np.cumsum(nseg) - nseg, nseg)
    mo, me = off[msg], off[msg] + lens[msg]
    S = np.where(k == 0, mo, (mo + k * seg) & ~127)
    E = np.where(k + 1 == nseg[msg], me, (mo + (k + 1) * seg) & ~127)
    cls = size_class(((E + 127) >> 7) - (S >> 7))
    total = 0
    for c in range(16):
        m = np.unique(msg[cls == c])
        total += 128 * (np.unique(m >> 4).size + np.unique(m >> 5).size)
    return int(total)


def model(lens, seg=2048):
    n = lens.size
    off = np.zeros(n, dtype=np.int64)
    np.cumsum(lens[:-1], dtype=np.int64, out=off[1:])
    end = off + lens
    first = off >> 7
    last = (end - 1) >> 7
    lines = int((last - first + 1).sum())
    # a line is shared when a boundary (end of i == start of i+1) is not
    # 128-aligned
    shared = int(np.count_nonzero(end[:-1] & 127))
    nseg = int(((lens.astype(np.int64) + seg - 1) // seg).sum())
    alg = int(lens.sum(dtype=np.int64)) + 4 * n
    meta = 12 * n + 4 * n + 4 * nseg + 12 * (nseg // 64)
    return {"msgs": n, "alg_bytes": alg, "payload": int(lens.sum(dtype=np.int64)),
            "lines_128_bytes": 128 * lines, "shared_lines": shared,
            "shared_line_bytes": 128 * shared, "segments_2KiB": nseg, "meta_bytes": meta,
            "model_128_total": 128 * lines + meta, "model_64_total": alg - 4 * n + meta,
            "model_128_over_alg": round((128 * lines + meta) / alg, 4),
            "model_64_over_alg": round((alg - 4 * n + meta) / alg, 4)}


def main():
    import bench
    lens, _ = bench._zipf(0, 1)
    res = {"whole": model(lens)}
    for k in range(8):
        sl, _ = bench._zipf(k, 8)
        res["shard_%d_of_8" % k] = model(sl)
    summ = sys.argv[1] if len(sys.argv) > 1 else None
    if summ and os.path.exists(summ):
        s = json.load(open(summ))
        res["measured"] = {"source": os.path.relpath(summ, ROOT),
                           "traffic_bytes_per_launch": s["traffic_bytes_per_launch"],
                           "traffic_over_alg": round(s["traffic_over_alg"], 4),
                           "excess_over_alg": s["traffic_bytes_per_launch"] - s["alg_bytes_per_launch"]}
        w = res["whole"]
        dbc = desc_by_class(lens)
        res["attribution"] = {
            "metadata": w["meta_bytes"] - 4 * w["msgs"],
            "shared_lines_refetched": w["lines_128_bytes"] - w["payload"],
            "descriptor_rereads_by_class": dbc - 12 * w["msgs"],
            "unexplained": s["traffic_bytes_per_launch"] - w["model_128_total"]
            - (dbc - 12 * w["msgs"])}
        # the same batch with every message 128-byte aligned: no shared lines
        la = lens.astype(np.int64)
        res["aligned_128_model"] = int(((la + 127) // 128 * 128).sum()) + w["meta_bytes"] \
            + desc_by_class(lens, align=128) - 12 * w["msgs"]
    print(json.dumps(res, indent=1))
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
