"""Randomized parity (the reference's fuzz harness, s_bmqfuzz_bmqp_crc32c.fuzz.cpp,
generalised to batches): random arenas, message counts, lengths from several
distributions (empty, < 4 bytes, line-edge sizes, multi-segment), random
offsets (unaligned, overlapping), random seeds and segment sizes, the
whole-messages flag and declared length bounds (exact, broken, loose) -- every
CRC compared with the oracle.  BMQCRC_FUZZ_ROUNDS
scales the number of batches (default 24), BMQCRC_FUZZ_MAX_N and
BMQCRC_FUZZ_ARENA their size."""
import os

import numpy as np
import pytest

import oracle
from blazingmq_amd import Crc32c

pytestmark = pytest.mark.gpu

ROUNDS = int(os.environ.get("BMQCRC_FUZZ_ROUNDS", "24"))
MAX_N = int(os.environ.get("BMQCRC_FUZZ_MAX_N", "5000"))
MAX_EXTRA = int(os.environ.get("BMQCRC_FUZZ_ARENA", str(1 << 20)))


def _lengths(rng, n):
    kind = rng.integers(0, 5)
    if kind == 0:  # tiny and edge sizes
        return rng.choice([0, 1, 2, 3, 4, 5, 15, 16, 17, 63, 64, 65, 127, 128, 129, 255, 256],
                          size=n)
    if kind == 1:  # small, uniform
        return rng.integers(0, 2048, size=n)
    if kind == 2:  # Zipf-like
        r = rng.zipf(1.5, size=n)
        return np.minimum(64 * r, 1 << 20)
    if kind == 3:  # one size for all (closed-form planner paths)
        return np.full(n, int(rng.integers(1, 70000)))
    return rng.integers(0, 200000, size=n)  # multi-segment mix


@pytest.mark.parametrize("round_", range(ROUNDS))
def test_fuzz_batch(cuda, round_):
    import torch
    rng = np.random.default_rng(1000 + round_)
    n = int(rng.integers(1, MAX_N))
    lens = _lengths(rng, n).astype(np.uint32)
    arena_size = int(lens.max(initial=0)) + int(rng.integers(64, MAX_EXTRA))
    arena = rng.integers(0, 256, size=arena_size, dtype=np.uint8)
    offs = (rng.random(n) * (arena_size - lens.astype(np.int64) + 1)).astype(np.uint64)
    seeds = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32) \
        if rng.integers(0, 2) else None
    seg = int(rng.choice([0, 0, 256, 384, 1024, 4096, 16384, 65536]))
    whole = bool(rng.integers(0, 4) == 0)
    # declared length bound (bmqcrc_opts.max_len): none, exact, broken, loose
    mk = int(rng.integers(0, 4))
    top = int(lens.max(initial=0))
    max_len = [0, top, int(np.median(lens)) if n else 0, top + 4096][mk]
    exp = oracle.batch(arena, offs, lens, seeds, nthreads=8)
    a = torch.from_numpy(arena).to(cuda)
    o = torch.from_numpy(offs.astype(np.int64)).to(cuda)
    ln = torch.from_numpy(lens.view(np.int32)).to(cuda)
    sd = None if seeds is None else torch.from_numpy(seeds.view(np.int32)).to(cuda)
    got = Crc32c.calculate_batch(a, o, ln, sd, seg_bytes=seg, whole_messages=whole,
                                 max_len=max_len)
    got = got.cpu().numpy().view(np.uint32)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, (round_, n, seg, whole, max_len, bad[:5], lens[bad[:5]], offs[bad[:5]])


@pytest.mark.parametrize("round_", range(max(2, ROUNDS // 8)))
def test_fuzz_single_pass_planner(cuda, round_):
    # Batches of more than four planner tiles per block (> 1.3M messages) are
    # planned by k_plan_map (round 3): random length mixes, overlapping
    # unaligned offsets, random seeds and segment sizes, a random wait limit
    # (0 gives the size-class map up), twice in a row on one stream.
    import torch
    from blazingmq_amd import last_launch, plan_wait
    rng = np.random.default_rng(5000 + round_)
    n = int(rng.integers(1_350_000, 1_800_000))
    parts = [rng.integers(0, 300, size=n - n // 64)]
    parts.append(np.minimum(_lengths(rng, n // 64), 65536))
    lens = np.concatenate(parts).astype(np.uint32)
    rng.shuffle(lens)
    arena_size = int(lens.max(initial=0)) + (48 << 20)
    arena = rng.integers(0, 256, size=arena_size, dtype=np.uint8)
    offs = (rng.random(n) * (arena_size - lens.astype(np.int64) + 1)).astype(np.uint64)
    seeds = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32) \
        if rng.integers(0, 2) else None
    seg = int(rng.choice([0, 0, 256, 1024, 2048, 16384]))
    exp = oracle.batch(arena, offs, lens, seeds, nthreads=8)
    a = torch.from_numpy(arena).to(cuda)
    o = torch.from_numpy(offs.astype(np.int64)).to(cuda)
    ln = torch.from_numpy(lens.view(np.int32)).to(cuda)
    sd = None if seeds is None else torch.from_numpy(seeds.view(np.int32)).to(cuda)
    s = torch.cuda.Stream(cuda)
    s.wait_stream(torch.cuda.current_stream(cuda))
    plan_wait(cuda.index, s, int(rng.choice([0, 1000])))
    for _ in range(2):
        got = Crc32c.calculate_batch(a, o, ln, sd, seg_bytes=seg, stream=s)
        got = got.cpu().numpy().view(np.uint32)
        bad = np.nonzero(got != exp)[0]
        assert bad.size == 0, (round_, n, seg, bad[:5], lens[bad[:5]], offs[bad[:5]])
        # planner + k_fold: the light k_plan on the fresh stream (no shape
        # history), k_plan_map once the stream has seen the batch is ragged
        assert last_launch(cuda.index, s)["kernels"] == 2
    plan_wait(cuda.index, s, 1000)


@pytest.mark.parametrize("round_", range(max(4, ROUNDS // 4)))
def test_fuzz_gather(cuda, round_):
    """bmqcrc_crc32c_gather on random Blob-shaped batches: buffer sizes from
    the same distributions (including empty buffers and empty messages),
    random message partitions, seeds -- against the oracle's Blob chain."""
    import ctypes

    from blazingmq_amd import _native as N
    rng = np.random.default_rng(5000 + round_)
    nbuf = int(rng.integers(0, 3000))
    sizes = _lengths(rng, nbuf).astype(np.uint32) if nbuf else np.zeros(0, np.uint32)
    bufs = [rng.integers(0, 256, size=int(k), dtype=np.uint8) for k in sizes]
    n = int(rng.integers(1, 400))
    first = np.sort(rng.integers(0, nbuf + 1, size=n + 1)).astype(np.uint64)
    seeds = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    ptrs = (ctypes.c_void_p * max(nbuf, 1))(*[b.ctypes.data if b.size else None for b in bufs])
    lens = sizes if nbuf else np.zeros(1, np.uint32)
    out = np.zeros(n, np.uint32)
    o = N.make_opts()
    N.check(N.lib.bmqcrc_crc32c_gather(ptrs, lens.ctypes.data, nbuf, first.ctypes.data,
                                       seeds.ctypes.data, out.ctypes.data, n, ctypes.byref(o)))
    exp = [oracle.blob([bufs[k].tobytes() for k in range(int(first[m]), int(first[m + 1]))],
                       int(seeds[m])) for m in range(n)]
    assert out.tolist() == exp


@pytest.mark.parametrize("round_", range(max(3, ROUNDS // 8)))
def test_fuzz_walks_over_devices(cuda, round_):
    """Recovery verify of random partitions spread over 2-5 listings of the
    device (bmqcrc_opts.ndevices) equals the single-device call: counts,
    alarm offsets in order, bounded reports."""
    from blazingmq_amd import storage
    rng = np.random.default_rng(6000 + round_)
    n = int(rng.integers(1, 3000))
    apps = [rng.integers(0, 256, size=int(k), dtype=np.uint8).tobytes()
            for k in _lengths(rng, n)]
    j, d = storage.write_partition(apps)
    for _ in range(int(rng.integers(0, 30))):
        if d.size:
            d[int(rng.integers(0, d.size))] ^= 0x20
    one = storage.verify_partition(j, d)
    for k in (2, 3, 5):
        many = storage.verify_partition(j, d, devices=[0] * k)
        assert (many["n_messages"], many["n_bad"]) == (one["n_messages"], one["n_bad"])
        assert many["bad_record_offsets"].tolist() == one["bad_record_offsets"].tolist()
        cap = int(rng.integers(0, 8))
        assert storage.verify_partition(j, d, bad_cap=cap, devices=[0] * k)[
            "bad_record_offsets"].tolist() == one["bad_record_offsets"][:cap].tolist()
