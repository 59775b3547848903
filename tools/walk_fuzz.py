#!/usr/bin/env python3
"""Mutation fuzzer for the native format walks (CPU only): valid PUT events,
partitions (journal + DATA) and cluster-state ledgers from blazingmq_amd's
synthesizers, with random byte flips, overwritten words, truncations and
garbage tails, fed to the walks the broker would run on untrusted bytes
(bmqcrc_put_event_scan, bmqcrc_journal_scan / journal_bounds,
bmqcrc_csl_scan).  Any return code is fine; a crash or a sanitizer report is
not.  Meant to run against an AddressSanitizer build of the library:

  hipcc ... -fsanitize=address (host objects) -> swap in as lib/libbmqcrc.so
  ASAN_OPTIONS=detect_leaks=0 LD_PRELOAD=$(clang -print-file-name=libclang_rt.asan-x86_64.so) \\
      python tools/walk_fuzz.py 3000

(DESIGN.md section 7 records the run.)"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from blazingmq_amd import _native as N  # noqa: E402
from blazingmq_amd import csl, storage, synth  # noqa: E402


def mutate(rng, buf):
    b = bytearray(buf)
    kind = rng.integers(0, 5)
    if kind == 0 and b:  # flip a few bytes
        for i in rng.integers(0, len(b), size=int(rng.integers(1, 9))):
            b[int(i)] ^= int(rng.integers(1, 256))
    elif kind == 1 and len(b) >= 4:  # overwrite an aligned word with an extreme value
        i = int(rng.integers(0, len(b) // 4)) * 4
        b[i:i + 4] = int(rng.choice([0, 1, 0x7fffffff, 0xffffffff, 0x80000000,
                                     int(rng.integers(0, 2**32))])).to_bytes(4, "big")
    elif kind == 2 and b:  # truncate
        del b[int(rng.integers(0, len(b))):]
    elif kind == 3:  # garbage tail
        b += rng.integers(0, 256, size=int(rng.integers(1, 300)), dtype=np.uint8).tobytes()
    else:  # random block
        if b:
            i = int(rng.integers(0, len(b)))
            n = int(rng.integers(1, 64))
            b[i:i + n] = rng.integers(0, 256, size=min(n, len(b) - i), dtype=np.uint8).tobytes()
    return bytes(b)


def call(fn):
    try:
        fn()
    except (N.BmqCrcError, ValueError):
        pass  # an error code is an acceptable answer to a corrupt input


def put_scan(ev):
    """bmqcrc_put_event_scan straight on the bytes (the Python iterator
    checks the event header first, which would keep most inputs away)."""
    p = ctypes.c_void_p(ev.ctypes.data) if ev.size else None
    n = N.lib.bmqcrc_put_event_scan(p, ev.size, None, None, None, 0)
    if n > 0:
        off, ln, pos = np.zeros(n, np.uint64), np.zeros(n, np.uint32), np.zeros(n, np.uint64)
        N.lib.bmqcrc_put_event_scan(p, ev.size, ctypes.c_void_p(off.ctypes.data),
                                    ctypes.c_void_p(ln.ctypes.data),
                                    ctypes.c_void_p(pos.ctypes.data), n)


def main(iters):
    rng = np.random.default_rng(2024)
    key = b"\x01\x02\x03\x04\x05"
    counts = {"put": 0, "partition": 0, "csl": 0}
    for it in range(iters):
        which = it % 3
        if which == 0:
            ev, _, _ = synth.put_event(int(rng.integers(1, 40)), int(rng.integers(0, 3000)),
                                       seed=int(rng.integers(0, 1 << 30)))
            bad = np.frombuffer(mutate(rng, ev.tobytes()), np.uint8).copy()
            call(lambda: put_scan(bad))
            counts["put"] += 1
        elif which == 1:
            j, d, _, _ = synth.partition(int(rng.integers(1, 30)), int(rng.integers(0, 2000)),
                                         seed=int(rng.integers(0, 1 << 30)))
            if rng.integers(0, 2):
                j = np.frombuffer(mutate(rng, j.tobytes()), np.uint8).copy()
            else:
                d = np.frombuffer(mutate(rng, d.tobytes()), np.uint8).copy()
            call(lambda: storage.scan_partition(j, d))
            call(lambda: storage.journal_bounds(j))
            counts["partition"] += 1
        else:
            log = csl.file_header(key)
            for _ in range(int(rng.integers(0, 12))):
                log += csl.append_record(rng.integers(0, 256, size=int(rng.integers(0, 200)),
                                                      dtype=np.uint8).tobytes())
            bad = mutate(rng, log)
            call(lambda: csl.scan_log(bad, key))
            call(lambda: csl.scan_log(bad, None))
            counts["csl"] += 1
    print("walk_fuzz: %d inputs, no crash" % iters, counts)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 1000)
