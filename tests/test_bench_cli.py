"""bench.py's CPU-only surfaces stay runnable: argument parsing of the
experiment options and the --cpu-table mode (the reference-equivalent CPU
baseline, oracle/), which needs no GPU."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_parse_experiment_options():
    sys.path.insert(0, ROOT)
    import bench
    argv = sys.argv
    try:
        sys.argv = ["bench.py", "--config", "1M_x_256B", "--msg-bytes", "64", "--shard", "1/4"]
        a = bench.parse()
    finally:
        sys.argv = argv
    assert a.config == "1M_x_256B" and a.config_given and a.msg_bytes == 64 and a.shard == "1/4"
    sys.argv = ["bench.py"]
    try:
        a = bench.parse()
    finally:
        sys.argv = argv
    assert a.config == "64k_x_64KiB" and not a.config_given and a.gpus == 1


def test_cpu_table_runs_without_gpu():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu-table",
                        "--config", "1k_x_4KiB", "--cpu-seconds", "0.2"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert {d["variant"] for d in lines} == {"hw", "hw_serial", "sw"}
    assert all(d["config"] == "1k_x_4KiB" and d["GiBps"] > 0 for d in lines)
