#!/usr/bin/env python3
"""Lane efficiency of k_fold's size-class groups on the Zipf 4M batch (CPU
only, numpy): the batch of bench.py's configs[3] cut into 2 KiB segments with
k_fold's segment geometry (seg_geom), segments ordered by size class, groups
of 64; efficiency = lines folded / (64 x rounds).  Compares the kernel's
classes (two per octave of the line count, size_class in crc32c_kernels.hip)
with one class per line count.  DESIGN.md section 6 quotes its output."""
import numpy as np

SEG = 2048


def zipf_lengths(n=4 * 1024 * 1024):
    rng = np.random.default_rng(3)  # bench.py _zipf
    r = np.arange(1, 16385, dtype=np.float64)
    p = r ** -1.5
    p /= p.sum()
    return (64 * rng.choice(16384, size=n, p=p) + 64).astype(np.int64)


def segment_lines(lens):
    off = np.concatenate([[0], np.cumsum(lens)[:-1]])
    nseg = (lens - 1) // SEG + 1
    msg = np.repeat(np.arange(len(lens)), nseg)
    k = np.arange(nseg.sum()) - np.repeat(np.cumsum(nseg) - nseg, nseg)
    ms, ns = off[msg], nseg[msg]
    me = ms + lens[msg]
    s = np.where(k == 0, ms, (ms + k * SEG) & ~127)
    e = np.where(k + 1 == ns, me, (ms + (k + 1) * SEG) & ~127)
    return (e - (s & ~127) + 127) // 128


def class_octave(nl):
    x = nl | 1
    b = np.floor(np.log2(x)).astype(np.int64)
    c = np.where(b > 0, 2 * b + ((x >> np.maximum(b - 1, 0)) & 1), 0)
    return np.minimum(c, 15)


def class_exact(nl):
    return np.minimum(nl - 1, 15)


def main():
    nl = segment_lines(zipf_lengths())
    print("segments", len(nl))
    for name, f in (("two classes per octave (k_fold)", class_octave),
                    ("one class per line count", class_exact)):
        g = nl[np.argsort(f(nl), kind="stable")]
        g = np.concatenate([g, np.zeros((-len(g)) % 64, dtype=g.dtype)]).reshape(-1, 64)
        rounds = g.max(axis=1)
        print("%s: groups %d, rounds %d, lane efficiency %.4f, one-round groups %d"
              % (name, len(rounds), rounds.sum(), nl.sum() / (64 * rounds.sum()),
                 (rounds == 1).sum()))


if __name__ == "__main__":
    main()
