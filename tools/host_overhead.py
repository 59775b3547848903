#!/usr/bin/env python3
"""Host cost of one batch call (GPU box): the time to enqueue N calls of
Crc32c.calculate_batch (sync=False) on a small device-resident batch, and
the step time with a synchronize after the N calls, for the library in
blazingmq_amd/lib/libbmqcrc.so (swap variants in from a shell).

  usage: python3 tools/host_overhead.py [n_msgs] [msg_bytes] [calls]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from blazingmq_amd import Crc32c
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    mb = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    calls = int(sys.argv[3]) if len(sys.argv) > 3 else 2000
    dev = torch.device("cuda", 0)
    arena = torch.randint(0, 256, (n * mb,), dtype=torch.uint8, device=dev)
    offs = torch.arange(n, dtype=torch.int64, device=dev) * mb
    lens = torch.full((n,), mb, dtype=torch.int32, device=dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    for _ in range(50):
        Crc32c.calculate_batch(arena, offs, lens, None, out, stream=stream, sync=False)
    torch.cuda.synchronize(dev)
    res = {"n": n, "msg_bytes": mb, "calls": calls}
    for rep in range(3):
        t0 = time.perf_counter()
        for _ in range(calls):
            Crc32c.calculate_batch(arena, offs, lens, None, out, stream=stream, sync=False)
        t1 = time.perf_counter()
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        res["enqueue_us_%d" % rep] = round(1e6 * (t1 - t0) / calls, 2)
        res["step_us_%d" % rep] = round(1e6 * (t2 - t0) / calls, 2)
    # the native call alone, from C via ctypes with prepared arguments
    from blazingmq_amd import _native as N
    import ctypes
    o = N.make_opts(device=0, stream=stream.cuda_stream, flags=0, seg_bytes=0)
    args = (ctypes.c_void_p(arena.data_ptr()), ctypes.c_uint64(arena.numel()),
            ctypes.c_void_p(offs.data_ptr()), ctypes.c_void_p(lens.data_ptr()), None,
            ctypes.c_void_p(out.data_ptr()), ctypes.c_uint64(n), ctypes.byref(o))
    f = N.lib.bmqcrc_crc32c_batch
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(calls):
        f(*args)
    t1 = time.perf_counter()
    torch.cuda.synchronize(dev)
    t2 = time.perf_counter()
    res["native_enqueue_us"] = round(1e6 * (t1 - t0) / calls, 2)
    res["native_step_us"] = round(1e6 * (t2 - t0) / calls, 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
