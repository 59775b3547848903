"""bench_traffic.json (the PMC traffic figure the bench line quotes as
roofline.traffic) is consistent with the committed rocprofv3
summaries it names and with bench.py's algorithmic bytes (SURVEY.md 8(d):
sum of lengths + 4 bytes of CRC per message)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_every_config_has_a_sourced_traffic_figure():
    sys.path.insert(0, ROOT)
    import bench
    with open(os.path.join(ROOT, "bench_traffic.json")) as f:
        t = json.load(f)
    assert set(t) == set(bench.CONFIGS)
    for cfg, e in t.items():
        src = os.path.join(ROOT, e["source"])
        assert os.path.exists(src), (cfg, e["source"])
        with open(src) as f:
            s = json.load(f)
        # the summary's corrected bytes: 2 x FETCH_SIZE KB x 1024 + WRITE_SIZE KB x 1024
        rd = 2 * 1024 * s["FETCH_SIZE_KB"]
        wr = 1024 * s["WRITE_SIZE_KB"]
        assert abs(rd + wr - e["traffic_bytes_per_launch"]) < 1e-6 * e["traffic_bytes_per_launch"] + 2
        # algorithmic bytes: what bench.py's roofline divides by
        lens, _ = bench.CONFIGS[cfg][1](0, 1)
        alg = int(np.asarray(lens, np.uint64).sum()) + 4 * len(lens)
        assert e["alg_bytes_per_launch"] == alg == s["alg_bytes_per_launch"], cfg
        # never below the payload, at most the descriptors' overhead of the
        # smallest messages (1k x 4 KiB: 16 % over)
        assert 1.0 <= e["traffic_over_alg"] < 1.2, (cfg, e["traffic_over_alg"])


def test_pmc_traffic_reads_the_file():
    sys.path.insert(0, ROOT)
    import bench
    with open(os.path.join(ROOT, "bench_traffic.json")) as f:
        t = json.load(f)
    for cfg in t:
        v, src = bench.pmc_traffic(cfg)
        assert v == t[cfg]["traffic_bytes_per_launch"] and src == t[cfg]["source"]
