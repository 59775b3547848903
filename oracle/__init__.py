"""CPU oracle for the CRC32C path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package, and only as the checker / reported CPU baseline; the product
(blazingmq_amd/) never imports it.  See crc32c_oracle.c for what it restates.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "liboracle_crc32c.so")

VARIANTS = {"hw": 0, "hw_serial": 1, "sw": 2, "bitwise": 3}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            import subprocess
            import sys
            subprocess.check_call([sys.executable, os.path.join(_HERE, "..", "blazingmq_amd",
                                                                "build.py")])
        L = ctypes.CDLL(LIB_PATH)
        u32, u64, vp = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p
        for f in ("oracle_crc32c_bitwise", "oracle_crc32c_sw", "oracle_crc32c_hw",
                  "oracle_crc32c_hw_serial"):
            getattr(L, f).restype = u32
            getattr(L, f).argtypes = [vp, u32, u32]
        L.oracle_crc32c_combine.restype = u32
        L.oracle_crc32c_combine.argtypes = [u32, u32, u64]
        L.oracle_crc32c_blob.restype = u32
        L.oracle_crc32c_blob.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(u32), u32, u32]
        L.oracle_crc32c_batch.restype = ctypes.c_int
        L.oracle_crc32c_batch.argtypes = [vp, vp, vp, vp, vp, ctypes.c_size_t, ctypes.c_int,
                                          ctypes.c_int]
        L.oracle_time_batch.restype = ctypes.c_double
        L.oracle_time_batch.argtypes = [vp, vp, vp, vp, vp, ctypes.c_size_t, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_int]
        L.oracle_time_batch_pinned.restype = ctypes.c_double
        L.oracle_time_batch_pinned.argtypes = [vp, vp, vp, vp, vp, ctypes.c_size_t, ctypes.c_int,
                                               ctypes.c_int, ctypes.c_int, vp]
        L.oracle_time_repeat.restype = ctypes.c_double
        L.oracle_time_repeat.argtypes = [vp, u32, ctypes.c_int, ctypes.c_int,
                                         ctypes.POINTER(u32)]
        L.oracle_fill_payload.restype = None
        L.oracle_fill_payload.argtypes = [vp, u64, u64, u64]
        L.oracle_have_sse42.restype = ctypes.c_int
        _lib = L
    return _lib


def _buf(data):
    if isinstance(data, np.ndarray):
        a = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
        return a, a.ctypes.data
    b = bytes(data)
    a = np.frombuffer(b, dtype=np.uint8) if b else np.zeros(1, np.uint8)
    return a, a.ctypes.data


def crc32c(data, crc=0, variant="bitwise"):
    a, p = _buf(data)
    n = len(data) if not isinstance(data, np.ndarray) else data.nbytes
    return getattr(lib(), "oracle_crc32c_" + variant)(p, n, crc & 0xFFFFFFFF)


def combine(a, b, len_b):
    return lib().oracle_crc32c_combine(a, b, len_b)


def blob(buffers, crc=0):
    n = len(buffers)
    keep = [_buf(b) for b in buffers]
    ptrs = (ctypes.c_void_p * max(n, 1))(*[k[1] for k in keep])
    lens = (ctypes.c_uint32 * max(n, 1))(*[len(b) for b in buffers])
    return lib().oracle_crc32c_blob(ptrs, lens, n, crc)


def batch(arena, offsets, lengths, seeds=None, nthreads=1, variant="hw"):
    a = np.ascontiguousarray(arena).view(np.uint8)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    ln = np.ascontiguousarray(lengths, dtype=np.uint32)
    sd = None if seeds is None else np.ascontiguousarray(seeds, dtype=np.uint32)
    out = np.empty(off.size, dtype=np.uint32)
    lib().oracle_crc32c_batch(a.ctypes.data, off.ctypes.data, ln.ctypes.data,
                              sd.ctypes.data if sd is not None else None, out.ctypes.data,
                              off.size, nthreads, VARIANTS[variant])
    return out


def time_batch(arena, offsets, lengths, nthreads, variant="hw", reps=1, cpus=None):
    """cpus: optional list of nthreads CPU ids, thread t pinned to cpus[t]."""
    a = np.ascontiguousarray(arena).view(np.uint8)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    ln = np.ascontiguousarray(lengths, dtype=np.uint32)
    out = np.empty(off.size, dtype=np.uint32)
    pin = None
    if cpus is not None:
        assert len(cpus) >= nthreads
        pin = np.ascontiguousarray(cpus[:nthreads], dtype=np.int32)
    t = lib().oracle_time_batch_pinned(a.ctypes.data, off.ctypes.data, ln.ctypes.data, None,
                                       out.ctypes.data, off.size, nthreads, VARIANTS[variant],
                                       reps, None if pin is None else pin.ctypes.data)
    return t, out


def time_batch_for(arena, offsets, lengths, nthreads, variant="hw", seconds=0.5, cpus=None):
    """Passes over the batch on `nthreads` threads (created once, one untimed
    warm-up pass) until about `seconds` of timed work: (seconds, passes)."""
    t, _ = time_batch(arena, offsets, lengths, nthreads, variant, 1, cpus)
    reps = 1
    while t < seconds:  # at most a few rounds: each aims 20 % past the target
        reps = max(reps + 1, int(1.2 * seconds * reps / max(t, 1e-7)))
        t, _ = time_batch(arena, offsets, lengths, nthreads, variant, reps, cpus)
    return t, reps


def _cpu_busy(sample_s=0.3):
    """Busy fraction of every CPU over a short window (/proc/stat), {} if
    unreadable."""
    import time

    def snap():
        out = {}
        with open("/proc/stat") as f:
            for line in f:
                if line.startswith("cpu") and line[3].isdigit():
                    parts = line.split()
                    v = [int(x) for x in parts[1:]]
                    idle = v[3] + (v[4] if len(v) > 4 else 0)
                    out[int(parts[0][3:])] = (sum(v), idle)
        return out
    try:
        a = snap()
        time.sleep(sample_s)
        b = snap()
    except (OSError, ValueError, IndexError):
        return {}
    busy = {}
    for c, (t1, i1) in b.items():
        t0, i0 = a.get(c, (t1, i1))
        dt = t1 - t0
        busy[c] = 1.0 - (i1 - i0) / dt if dt > 0 else 0.0
    return busy


def pick_cpus(nthreads, numa_node=None, avoid_busy=True):
    """Up to nthreads CPUs from this process's allowed set, one per physical
    core (SMT siblings skipped), preferring `numa_node`'s cores (the GPU's
    node) and, on a shared host, cores whose threads were idle over a short
    /proc/stat window (a core another job keeps busy would slow one thread,
    and with it every window).  Returns the list (shorter if the set holds
    fewer cores)."""
    allowed = sorted(os.sched_getaffinity(0))
    busy = _cpu_busy() if avoid_busy else {}

    def read(path, default):
        try:
            with open(path) as f:
                return f.read().strip()
        except OSError:
            return default

    def node_of(c):
        base = "/sys/devices/system/cpu/cpu%d" % c
        try:
            for e in os.listdir(base):
                if e.startswith("node") and e[4:].isdigit():
                    return int(e[4:])
        except OSError:
            pass
        return -1

    cores = {}  # physical core -> its allowed CPUs
    for c in allowed:
        topo = "/sys/devices/system/cpu/cpu%d/topology/" % c
        core = (read(topo + "physical_package_id", "0"), read(topo + "core_id", str(c)))
        cores.setdefault(core, []).append(c)
    ranked = []
    for core, cpus in cores.items():
        c = cpus[0]
        load = max(busy.get(x, 0.0) for x in cpus)  # a busy SMT sibling shares the core
        far = 0 if numa_node is None or node_of(c) == numa_node else 1
        ranked.append((far, load > 0.1, c, load))
    ranked.sort()
    return [r[2] for r in ranked[:nthreads]]


def time_repeat(buf, iters, variant="hw"):
    """The reference's benchmark loop (bmqp_crc32c.t.cpp:1116-1120): one
    buffer CRC'd `iters` times on one thread after an untimed call.  Returns
    seconds."""
    a, p = _buf(buf)
    c = ctypes.c_uint32()
    return lib().oracle_time_repeat(p, a.size if len(buf) else 0, iters, VARIANTS[variant],
                                    ctypes.byref(c))


def fill_payload(begin, nbytes, seed):
    """Host copy of bytes [begin, begin+nbytes) of the synthetic stream `seed`."""
    out = np.empty(nbytes, dtype=np.uint8)
    if nbytes:
        lib().oracle_fill_payload(out.ctypes.data, begin, nbytes, seed)
    return out
