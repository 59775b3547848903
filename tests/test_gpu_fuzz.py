"""Randomized parity (the reference's fuzz harness, s_bmqfuzz_bmqp_crc32c.fuzz.cpp,
generalised to batches): random arenas, message counts, lengths from several
distributions (empty, < 4 bytes, line-edge sizes, multi-segment), random
offsets (unaligned, overlapping), random seeds and segment sizes, and the
whole-messages flag -- every CRC compared with the oracle.  BMQCRC_FUZZ_ROUNDS
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
    exp = oracle.batch(arena, offs, lens, seeds, nthreads=8)
    a = torch.from_numpy(arena).to(cuda)
    o = torch.from_numpy(offs.astype(np.int64)).to(cuda)
    ln = torch.from_numpy(lens.view(np.int32)).to(cuda)
    sd = None if seeds is None else torch.from_numpy(seeds.view(np.int32)).to(cuda)
    got = Crc32c.calculate_batch(a, o, ln, sd, seg_bytes=seg, whole_messages=whole)
    got = got.cpu().numpy().view(np.uint32)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, (round_, n, seg, whole, bad[:5], lens[bad[:5]], offs[bad[:5]])
