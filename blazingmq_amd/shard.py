"""Byte-balanced sharding of a message batch across GPUs (no collective).

Messages are independent, so a batch shards embarrassingly: rank r takes the
contiguous message range [cuts[r], cuts[r+1]) whose payload bytes are ~1/N of
the total, CRCs it on its own GPU, and owns those 4-byte results.  This is the
same cut rule as bmqcrc_crc32c_batch_multi (csrc/bmqcrc_host.cpp).
"""
import numpy as np


def byte_balanced_cuts(lengths, parts):
    """Cut points c[0]=0 <= ... <= c[parts]=n: slice r = [c[r], c[r+1]).

    c[d] is the first index at which the running byte total reaches
    total * d / parts (integer division), exactly as the C++ splitter.
    """
    ln = np.asarray(lengths, dtype=np.uint64)
    n = ln.size
    if parts < 1:
        raise ValueError("parts must be >= 1")
    total = int(ln.sum())
    csum = np.cumsum(ln, dtype=np.uint64)  # bytes through index i (inclusive)
    cuts = [0]
    for d in range(1, parts):
        target = total * d // parts
        # smallest i such that sum(ln[:i]) >= target  (i >= previous cut)
        i = int(np.searchsorted(csum, target, side="left")) + 1 if target > 0 else 0
        i = min(max(i, cuts[-1]), n)
        cuts.append(i)
    cuts.append(n)
    return cuts


def rank_slice(lengths, rank, world):
    c = byte_balanced_cuts(lengths, world)
    return c[rank], c[rank + 1]
