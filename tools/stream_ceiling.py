#!/usr/bin/env python3
"""Measure the read-only HBM streaming ceiling of this MI355X (context for the
k_fold roofline).  Prints one JSON line per variant."""
import ctypes
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    lib = ctypes.CDLL(os.path.join(HERE, "lib", "libstream_probe.so"))
    lib.probe_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                 ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    nbytes = 4 << 30
    buf = torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device=dev)
    out = torch.empty(256 * 8 * 256 * 4, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream()
    names = {0: "global_load_dwordx4", 1: "global_load_dwordx4 nt", 2: "global_load_lds_dwordx4 ring"}
    for which in (0, 1, 2):
        for grid in ((256 * 4, 256 * 8) if which < 2 else (256 * 2,)):
            for _ in range(3):
                lib.probe_launch(which, buf.data_ptr(), nbytes, out.data_ptr(), grid, st.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 10
            e0.record()
            for _ in range(reps):
                lib.probe_launch(which, buf.data_ptr(), nbytes, out.data_ptr(), grid, st.cuda_stream)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            print(json.dumps({"probe": names[which], "grid": grid, "bytes": nbytes,
                              "us": round(ms * 1e3, 1), "TBps": round(nbytes / ms / 1e9, 3)}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
