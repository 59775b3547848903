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


def test_gpus_n_spawns_its_own_ranks():
    """`bench.py --gpus 2` without torchrun starts two ranks itself (a child
    torch.distributed.run, no exec) that rendezvous over gloo; rank 0 sees a
    world of 2.  --launch-check stops before any GPU call."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--launch-check"], capture_output=True, text=True, timeout=300,
                       cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    assert lines[0]["n_gpus"] == 2 and lines[0]["max_rank"] == 1 and lines[0]["gpus_arg"] == 2


def test_gpus_must_match_world_size():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4",
                        "--launch-check"], capture_output=True, text=True, timeout=120,
                       cwd=ROOT, env=env)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


def test_cpu_baseline_states_its_thread_counts():
    """The bench line's cpu_baseline: measured on this GPU's thread share and
    on one thread, with the host's thread count and the counts it did not
    measure stated."""
    sys.path.insert(0, ROOT)
    import numpy as np

    import bench
    cb = bench.cpu_baseline(np.full(2048, 4096, np.uint32), 2, 0.05)
    assert cb["kind"] == "port" and cb["value"] > 0 and cb["single_thread_value"] > 0
    assert cb["cores"] == bench.host_threads() and cb["host_threads"] == os.cpu_count()
    assert "nproc/8" in cb["not_measured"]
    # the value is the cache-resident median of seven windows, the streamed
    # leg reported beside it
    assert len(cb["windows_GiBps"]) == 7 and len(cb["streamed_windows_GiBps"]) == 7
    assert cb["value"] == sorted(cb["windows_GiBps"])[3]
    assert cb["streamed_value"] == sorted(cb["streamed_windows_GiBps"])[3]
    assert "cache-resident" in cb["sample"]
