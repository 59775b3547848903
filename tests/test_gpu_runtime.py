"""Runtime properties of the batch path on the GPU: hipGraph capture after
bmqcrc_reserve (the launch path allocates and synchronizes nothing), and
concurrent batches on different streams from different host threads
(per-(device, stream) workspaces, bmqp_crc32c.h:40-42 thread safety)."""
import json
import os
import subprocess
import sys
import threading
import time

import numpy as np
import pytest

import oracle
from blazingmq_amd import Crc32c, reserve

pytestmark = pytest.mark.gpu


def _batch(rng, n, max_len, arena_size):
    lens = rng.integers(0, max_len, size=n).astype(np.uint32)
    offs = np.array([rng.integers(0, arena_size - l + 1) for l in lens], np.int64)
    seeds = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    return offs, lens, seeds


@pytest.mark.parametrize("whole", [False, True])
def test_graph_capture_and_replay(cuda, whole):
    import torch
    rng = np.random.default_rng(31 + whole)
    size = 8 << 20
    arena_np = rng.integers(0, 256, size=size, dtype=np.uint8)
    offs, lens, seeds = _batch(rng, 3000, 40000, size)
    arena = torch.from_numpy(arena_np).to(cuda)
    o = torch.from_numpy(offs).to(cuda)
    ln = torch.from_numpy(lens.view(np.int32)).to(cuda)
    sd = torch.from_numpy(seeds.view(np.int32)).to(cuda)
    out = torch.zeros(lens.size, dtype=torch.int32, device=cuda)
    side = torch.cuda.Stream(cuda)
    reserve(cuda.index or 0, side, lens.size, size)
    # warm the workspace on the capture stream, then capture one batch
    with torch.cuda.stream(side):
        Crc32c.calculate_batch(arena, o, ln, sd, out, stream=side, sync=False,
                               whole_messages=whole)
    side.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        Crc32c.calculate_batch(arena, o, ln, sd, out, stream=side, sync=False,
                               whole_messages=whole)
    for it in range(3):  # replays read the arena as it is at replay time
        new = rng.integers(0, 256, size=size, dtype=np.uint8)
        arena.copy_(torch.from_numpy(new).to(cuda))
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint32)
        assert np.array_equal(got, oracle.batch(new, offs, lens, seeds, nthreads=8)), it


def test_graph_replays_of_a_ragged_batch_with_new_lengths(cuda):
    # A planned ragged batch captured into a graph, replayed with new lengths,
    # offsets and payload each time (the device arrays rewritten in place).
    # The single-pass planner tags the words its blocks exchange with the
    # launch's epoch; captured, that tag lives on the device and advances on
    # every replay (k_epoch_advance), so no replay reads the previous one's
    # histogram or group descriptors as current.
    import torch
    from blazingmq_amd import last_launch
    rng = np.random.default_rng(35)
    size, n = 48 << 20, 200_000
    side = torch.cuda.Stream(cuda)
    arena = torch.zeros(size, dtype=torch.uint8, device=cuda)
    o = torch.zeros(n, dtype=torch.int64, device=cuda)
    ln = torch.zeros(n, dtype=torch.int32, device=cuda)
    out = torch.zeros(n, dtype=torch.int32, device=cuda)
    reserve(cuda.index or 0, side, n, size, 2048)

    def new_batch():
        lens = np.concatenate([rng.integers(0, 300, size=n - 400),
                               rng.integers(0, 60000, size=400)]).astype(np.uint32)
        rng.shuffle(lens)
        offs = (rng.random(n) * (size - lens + 1)).astype(np.int64)
        data = rng.integers(0, 256, size=size, dtype=np.uint8)
        arena.copy_(torch.from_numpy(data).to(cuda))
        o.copy_(torch.from_numpy(offs).to(cuda))
        ln.copy_(torch.from_numpy(lens.view(np.int32)).to(cuda))
        torch.cuda.synchronize()
        return oracle.batch(data, offs, lens, None, nthreads=8)

    exp = new_batch()
    with torch.cuda.stream(side):  # warm: the workspace learns the batch is ragged
        Crc32c.calculate_batch(arena, o, ln, None, out, stream=side, sync=False, seg_bytes=2048)
    side.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), exp)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        Crc32c.calculate_batch(arena, o, ln, None, out, stream=side, sync=False, seg_bytes=2048)
    assert last_launch(cuda.index or 0, side)["kernels"] == 2  # k_plan_map + k_fold captured
    for it in range(4):
        exp = new_batch()
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        bad = np.nonzero(out.cpu().numpy().view(np.uint32) != exp)[0]
        assert bad.size == 0, (it, bad[:8])


def test_graph_capture_on_a_fresh_stream_keeps_the_map(cuda):
    # With no shape history a planned batch gets the light k_plan, whose fold
    # searches seg_first, and the stream's NEXT batch gets the map -- which
    # never happens inside a graph.  A capture therefore plans with the map
    # whatever the history, and the replays stay exact.
    import torch
    from blazingmq_amd import last_launch
    rng = np.random.default_rng(36)
    size, n = 16 << 20, 60_000
    side = torch.cuda.Stream(cuda)
    lens = np.concatenate([rng.integers(0, 300, size=n - 100),
                           rng.integers(0, 40000, size=100)]).astype(np.uint32)
    rng.shuffle(lens)
    offs = (rng.random(n) * (size - lens + 1)).astype(np.int64)
    data = rng.integers(0, 256, size=size, dtype=np.uint8)
    arena = torch.from_numpy(data).to(cuda)
    o = torch.from_numpy(offs).to(cuda)
    ln = torch.from_numpy(lens.view(np.int32)).to(cuda)
    out = torch.zeros(n, dtype=torch.int32, device=cuda)
    reserve(cuda.index or 0, side, n, size, 2048)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        Crc32c.calculate_batch(arena, o, ln, None, out, stream=side, sync=False, seg_bytes=2048)
    launch = last_launch(cuda.index or 0, side)
    assert launch["spec"] == 0 and launch["map"] == 1, launch
    exp = oracle.batch(data, offs, lens, None, nthreads=8)
    for it in range(3):
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        bad = np.nonzero(out.cpu().numpy().view(np.uint32) != exp)[0]
        assert bad.size == 0, (it, bad[:8])


def test_graph_capture_while_the_pair_plans(cuda):
    # A given-up map switches the workspace to the pair planner (k_plan +
    # k_plan_sort) for its next ragged batches.  A batch captured then carries
    # device-side tags (plan_epoch 0) as in the single-pass case: k_fold's
    # group-descriptor lookup must not match words left at tag 0 (never
    # written) or by an earlier launch, so every replay must stay exact.
    import torch
    from blazingmq_amd import last_launch, plan_wait
    rng = np.random.default_rng(37)
    size, n = 16 << 20, 1_400_100
    side = torch.cuda.Stream(cuda)
    arena = torch.zeros(size, dtype=torch.uint8, device=cuda)
    o = torch.zeros(n, dtype=torch.int64, device=cuda)
    ln = torch.zeros(n, dtype=torch.int32, device=cuda)
    out = torch.zeros(n, dtype=torch.int32, device=cuda)
    reserve(cuda.index or 0, side, n, size, 2048)

    def new_batch():
        lens = np.concatenate([rng.integers(0, 300, size=n - 100),
                               rng.integers(0, 100000, size=100)]).astype(np.uint32)
        rng.shuffle(lens)
        offs = (rng.random(n) * (size - lens + 1)).astype(np.int64)
        data = rng.integers(0, 256, size=size, dtype=np.uint8)
        arena.copy_(torch.from_numpy(data).to(cuda))
        o.copy_(torch.from_numpy(offs).to(cuda))
        ln.copy_(torch.from_numpy(lens.view(np.int32)).to(cuda))
        torch.cuda.synchronize()
        return oracle.batch(data, offs, lens, None, nthreads=8)

    def run():
        with torch.cuda.stream(side):
            Crc32c.calculate_batch(arena, o, ln, None, out, stream=side, sync=False,
                                   seg_bytes=2048)
        side.synchronize()

    exp = new_batch()
    run()  # warm: ragged, mapped by the single pass
    plan_wait(cuda.index or 0, side, 0)
    run()  # the zero limit gives the map up (recorded on the workspace)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), exp)
    plan_wait(cuda.index or 0, side, 1000)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        Crc32c.calculate_batch(arena, o, ln, None, out, stream=side, sync=False, seg_bytes=2048)
    assert last_launch(cuda.index or 0, side)["kernels"] == 3  # k_plan + k_plan_sort + k_fold
    for it in range(4):
        exp = new_batch()
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        bad = np.nonzero(out.cpu().numpy().view(np.uint32) != exp)[0]
        assert bad.size == 0, (it, bad[:8])


def test_concurrent_streams_and_threads(cuda):
    import torch
    rng = np.random.default_rng(41)
    size = 16 << 20
    jobs = []
    for t in range(4):
        arena_np = rng.integers(0, 256, size=size, dtype=np.uint8)
        offs, lens, seeds = _batch(rng, 20000 if t % 2 else 400, 1 << 16 if t % 2 else 200000,
                                   size)
        jobs.append((arena_np, offs, lens, seeds))
    results = [None] * len(jobs)
    errors = []

    def work(i):
        try:
            arena_np, offs, lens, seeds = jobs[i]
            s = torch.cuda.Stream(cuda)
            with torch.cuda.stream(s):
                arena = torch.from_numpy(arena_np).to(cuda, non_blocking=False)
                o = torch.from_numpy(offs).to(cuda)
                ln = torch.from_numpy(lens.view(np.int32)).to(cuda)
                sd = torch.from_numpy(seeds.view(np.int32)).to(cuda)
                outs = [Crc32c.calculate_batch(arena, o, ln, sd, stream=s, sync=False)
                        for _ in range(5)]
            s.synchronize()
            results[i] = [x.cpu().numpy().view(np.uint32) for x in outs]
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    threads = [threading.Thread(target=work, args=(i,)) for i in range(len(jobs))]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    assert not errors, errors
    for (arena_np, offs, lens, seeds), res in zip(jobs, results):
        exp = oracle.batch(arena_np, offs, lens, seeds, nthreads=8)
        for r in res:
            assert np.array_equal(r, exp)


def test_zero_copy_host_arena(cuda):
    # bmqcrc_host_register: the kernels read ordinary (registered) host memory
    # in place over PCIe -- the zero-copy end-to-end variant of SURVEY.md 8(d)
    import torch
    from blazingmq_amd import HostRegistration, calculate_batch_ptr
    rng = np.random.default_rng(51)
    arena_np = rng.integers(0, 256, size=(2 << 20) + 77, dtype=np.uint8)
    offs, lens, seeds = _batch(rng, 3000, 5000, arena_np.size)
    with HostRegistration(arena_np, device=cuda.index or 0) as reg:
        got = calculate_batch_ptr(reg.dev_ptr, reg.nbytes, torch.from_numpy(offs).to(cuda),
                                  torch.from_numpy(lens.view(np.int32)).to(cuda),
                                  torch.from_numpy(seeds.view(np.int32)).to(cuda))
        got = got.cpu().numpy().view(np.uint32)
    assert np.array_equal(got, oracle.batch(arena_np, offs, lens, seeds, nthreads=8))


def test_default_stream_ordering(cuda):
    # opts.stream == NULL is the device's default (null) stream, so an ASYNC
    # batch enqueued on torch's default stream is ordered with the torch ops
    # that follow it there (here a non-blocking D2H copy, then a wait on that
    # stream only) -- no device-wide synchronisation needed
    import torch
    from blazingmq_amd import fill_synthetic
    rng = np.random.default_rng(61)
    n, size = 50000, 1024
    arena = torch.empty(n * size, dtype=torch.uint8, device=cuda)
    fill_synthetic(arena, 9)
    offs = np.arange(n, dtype=np.int64) * size
    lens = np.full(n, size, np.uint32)
    lens[rng.integers(0, n, 100)] = 0
    with torch.cuda.stream(torch.cuda.default_stream(cuda)):
        out = Crc32c.calculate_batch(arena, torch.from_numpy(offs).to(cuda),
                                     torch.from_numpy(lens.view(np.int32)).to(cuda), sync=False)
        host = torch.empty(n, dtype=torch.int32, pin_memory=True)
        host.copy_(out, non_blocking=True)
        torch.cuda.default_stream(cuda).synchronize()
    exp = oracle.batch(arena.cpu().numpy(), offs, lens, nthreads=8)
    assert np.array_equal(host.numpy().view(np.uint32), exp)


def test_concurrent_gather_and_multi_device_walks(cuda):
    """Host-buffer calls from several threads at once: Blob gathers (the
    default stream's workspace and its pinned ring) and recovery walks spread
    over 2 and 3 listings of the device (library-owned streams shared between
    the calls) -- no deadlock, every result equal to a serial call."""
    from blazingmq_amd import Blob, storage
    rng = np.random.default_rng(42)
    apps = [rng.integers(0, 256, size=int(k), dtype=np.uint8).tobytes()
            for k in rng.integers(0, 40000, size=1500)]
    j, d = storage.write_partition(apps)
    for i in rng.integers(0, d.size, size=9):
        d[int(i)] ^= 0x08
    serial = storage.verify_partition(j, d)
    blobs = [Blob([rng.integers(0, 256, size=int(k), dtype=np.uint8).tobytes()
                   for k in rng.integers(0, 9000, size=int(rng.integers(0, 9)))])
             for _ in range(300)]
    blob_exp = Crc32c.calculate_blobs(blobs).tolist()
    errors = []

    def walks(devs):
        try:
            for _ in range(6):
                r = storage.verify_partition(j, d, devices=devs)
                assert r["n_bad"] == serial["n_bad"]
                assert r["bad_record_offsets"].tolist() == serial["bad_record_offsets"].tolist()
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    def gathers():
        try:
            for _ in range(6):
                assert Crc32c.calculate_blobs(blobs).tolist() == blob_exp
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    threads = [threading.Thread(target=walks, args=([0, 0],)),
               threading.Thread(target=walks, args=([0, 0, 0],)),
               threading.Thread(target=gathers), threading.Thread(target=gathers)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=150)
    assert not any(th.is_alive() for th in threads), "a host-buffer call did not return"
    assert not errors, errors


@pytest.mark.perf
def test_processes_share_the_planner_on_one_gpu(cuda, record_property, perf_bound,
                                                tmp_path):
    """Three processes CRC ragged batches of 1.4M+ messages on the same GPU at
    once, with the default planner wait limit (tests/mp_planner_worker.py).
    The single-pass planner's blocks meet grid-wide, so with other processes'
    kernels resident a planner may give its map up (then the fold searches
    the segment offsets, and the stream plans with the meeting-free pair for
    a while): every CRC of every step must still match the oracle, and each
    process's median step must stay within 1.3x of its share of the GPU
    (3x one process's step alone; + 0.5 ms for the host's part of a step).
    The given-up maps are recorded (test property plan_voided)."""
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "mp_planner_worker.py")

    def launch(nproc, steps, tag):
        sync = tmp_path / tag
        sync.mkdir()
        procs = [subprocess.Popen([sys.executable, worker, str(w), str(steps), str(sync)],
                                  stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
                 for w in range(nproc)]
        try:
            deadline = time.time() + 180
            while sum((sync / ("ready_%d" % w)).exists() for w in range(nproc)) < nproc:
                assert all(p.poll() is None for p in procs), [p.stderr.read()[-2000:]
                                                              for p in procs if p.poll()]
                assert time.time() < deadline, "workers not ready"
                time.sleep(0.05)
            (sync / "go").touch()
            res = []
            for p in procs:
                out, err = p.communicate(timeout=180)
                assert p.returncode == 0, err[-3000:]
                res.append(json.loads(out.strip().splitlines()[-1]))
            return res
        finally:
            for p in procs:
                if p.poll() is None:
                    p.kill()
                    p.wait()

    alone = launch(1, 8, "alone")[0]
    shared = launch(3, 8, "shared")
    assert alone["mismatches"] == 0 and all(r["mismatches"] == 0 for r in shared), shared
    share = 3 * alone["median_ms"]
    worst = max(r["median_ms"] for r in shared)
    record_property("alone_ms", round(alone["median_ms"], 3))
    record_property("shared_ms", [round(r["median_ms"], 3) for r in shared])
    record_property("plan_voided", [r["plan_voided"] for r in shared])
    print("alone %.3f ms, three processes %s ms, given-up maps %s"
          % (alone["median_ms"], [round(r["median_ms"], 3) for r in shared],
             [r["plan_voided"] for r in shared]))
    perf_bound("shared_within_1.3x_of_share", worst <= 1.3 * share + 0.5,
               {"alone_ms": alone["median_ms"], "worst_shared_ms": worst})
