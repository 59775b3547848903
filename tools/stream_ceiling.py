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
                                 ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    nbytes = 4 << 30
    buf = torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device=dev)
    out = torch.empty(256 * 8 * 256 * 4, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream()
    names = {0: "global_load_dwordx4", 1: "global_load_dwordx4 nt",
             2: "LDS-DMA ring, contiguous 8 KiB rounds", 3: "LDS-DMA ring nt, contiguous 8 KiB rounds",
             4: "LDS-DMA ring, k_fold shape (64 segments per wave, a line of each per round)",
             5: "LDS-DMA ring nt, k_fold shape (64 segments per wave, a line of each per round)"}
    runs = [(w, g, 0) for w in (0, 1) for g in (256 * 4, 256 * 8)]
    runs += [(w, g, 0) for w in (2, 3) for g in (256, 512)]
    runs += [(w, g, seg) for w in (4, 5) for g in (256, 512) for seg in (65536, 16384)]
    if len(sys.argv) > 2 and sys.argv[1] == "--segs":  # k_fold shape, nt, given segment sizes only
        runs = [(5, g, int(seg)) for seg in sys.argv[2].split(",") for g in (256, 512)]
    for which, grid, seg in runs:
        def launch():
            rc = lib.probe_launch(which, buf.data_ptr(), nbytes, out.data_ptr(), grid, seg,
                                  st.cuda_stream)
            assert rc == 0
        for _ in range(3):
            launch()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 10
        e0.record()
        for _ in range(reps):
            launch()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        print(json.dumps({"probe": names[which], "grid": grid, "seg_bytes": seg or None,
                          "bytes": nbytes, "us": round(ms * 1e3, 1),
                          "TBps": round(nbytes / ms / 1e9, 3)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
