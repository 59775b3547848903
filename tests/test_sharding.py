"""Multi-GPU sharding logic, exercised on CPU with torch.distributed (gloo,
world_size 2): each rank CRCs its byte-balanced slice (here with the CPU
oracle -- the GPU path is covered by -m gpu) and the gathered results must
equal the single-process answer.  No data-path collective is used by the
product; all_gather here only collects results for the assertion."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from blazingmq_amd.shard import byte_balanced_cuts, rank_slice


def _zipf_lengths(n, seed):
    rng = np.random.default_rng(seed)
    r = np.arange(1, 16385, dtype=np.float64)
    p = r ** -1.5
    p /= p.sum()
    return (64 * rng.choice(r, size=n, p=p)).astype(np.uint32)


def test_cuts_partition_and_balance():
    for parts in (1, 2, 4, 8):
        ln = _zipf_lengths(20000, parts)
        c = byte_balanced_cuts(ln, parts)
        assert c[0] == 0 and c[-1] == ln.size and all(a <= b for a, b in zip(c, c[1:]))
        tot = int(ln.sum())
        for r in range(parts):
            share = int(ln[c[r]:c[r + 1]].sum())
            assert abs(share - tot / parts) <= int(ln.max()) + 1


def test_cuts_match_cpp_rule():
    # C++: for d in 1..N-1: advance i while acc < total*d/N (acc += len[i++])
    ln = _zipf_lengths(5000, 9)
    for parts in (2, 3, 8):
        total, acc, i, cpp = int(ln.sum()), 0, 0, [0]
        for d in range(1, parts):
            t = total * d // parts
            while i < ln.size and acc < t:
                acc += int(ln[i])
                i += 1
            cpp.append(i)
        cpp.append(ln.size)
        assert byte_balanced_cuts(ln, parts) == cpp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ln = _zipf_lengths(3000, 123)
    offs = np.concatenate([[0], np.cumsum(ln, dtype=np.uint64)[:-1]]).astype(np.uint64)
    arena = oracle.fill_payload(0, int(ln.sum()) + 8, 4)
    lo, hi = rank_slice(ln, rank, world)
    mine = oracle.batch(arena, offs[lo:hi], ln[lo:hi]).tolist()
    gathered = [None] * world
    dist.all_gather_object(gathered, (lo, hi, mine))
    if rank == 0:
        full = oracle.batch(arena, offs, ln).tolist()
        stitched = []
        for lo_r, hi_r, res in sorted(gathered):
            stitched += res
        q.put(stitched == full and sorted(g[0] for g in gathered)[0] == 0)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_sharded_batch(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    ok = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
    assert ok
    assert all(p.exitcode == 0 for p in procs)
