"""Host-side product path: scalar/blob CRC through the C ABI, the C++ drop-in
bmqp::Crc32c, the Python mirror -- all against the oracle and golden vectors.
(No GPU: these run in the CPU suite.)"""
import os
import subprocess

import numpy as np
import pytest

import oracle
from blazingmq_amd import Blob, BmqCrcError, Crc32c, device_count

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_scalar_golden(golden):
    for v in golden["calculate"] + golden["rfc3720"]:
        assert Crc32c.calculate(bytes.fromhex(v["hex"])) == v["crc"]
    assert Crc32c.calculate(None, length=0) == 0
    assert Crc32c.calculate(None, 0x1234, length=0) == 0x1234
    assert Crc32c.calculate(b"12345678", length=0) == 0


def test_scalar_chained(golden):
    for v in golden["chained"]:
        b, p = bytes.fromhex(v["hex"]), v["prefix_len"]
        c = Crc32c.calculate(b[p:], Crc32c.calculate(b[:p]))
        assert c == v["crc"]
        assert Crc32c.calculate(b, c, length=0) == c


def test_scalar_misaligned_random():
    rng = np.random.default_rng(21)
    big = rng.integers(0, 256, size=300000, dtype=np.uint8)
    # the product's method boundaries (crc32c_cpu.cpp): serial below 192 B,
    # one-accumulator fold below 256, four accumulators, 16-byte and < 16-byte
    # tails; three-way lanes (hosts without AVX-512) are checked below
    for n in list(range(0, 40)) + [63, 64, 65, 191, 192, 193, 207, 208, 255, 256, 257, 271, 319,
                                   320, 511, 512, 513, 767, 1535, 1536, 1537, 12287, 12288, 12289,
                                   100000, 262147]:
        for mis in range(0, 8):
            buf = big[mis:mis + n]
            seed = int(rng.integers(0, 2**32))
            assert Crc32c.calculate(buf, seed) == oracle.crc32c(buf.tobytes(), seed), (n, mis)


def test_blob(golden):
    for v in golden["blob"]:
        assert Crc32c.calculate_blob(Blob(bytes.fromhex(h) for h in v["buffers_hex"])) == v["crc"]
    for v in golden["blob_chained"]:
        c = v.get("seed", 0)
        for blob in v["blobs_hex"]:
            c = Crc32c.calculate_blob(Blob(bytes.fromhex(h) for h in blob), c)
        assert c == v["crc"]


def test_blob_fuzz_property():
    # s_bmqfuzz_bmqp_crc32c.fuzz.cpp: raw CRC == Blob CRC, any split in 1..256, any seed
    rng = np.random.default_rng(31)
    for _ in range(300):
        size = int(rng.integers(1, 257))
        data = rng.integers(0, 256, size=size, dtype=np.uint8).tobytes()
        seed = int(rng.integers(0, 2**32))
        cuts = sorted(set(rng.integers(1, size, size=int(rng.integers(0, 6))).tolist())) if size > 1 else []
        parts = [data[a:b] for a, b in zip([0] + cuts, cuts + [size])]
        assert Crc32c.calculate_blob(Blob(parts), seed) == Crc32c.calculate(data, seed)


def test_last_data_buffer_length():
    b = Blob([b"one", b"two", b"threeXYZ"])
    b.set_last_data_buffer_length(5)
    assert Crc32c.calculate_blob(b) == 0xA0EA6901


def test_scalar_methods_agree(tmp_path):
    # every method of crc32c_cpu.cpp the host supports (serial crc32q, the
    # three-way lanes, the VPCLMULQDQ fold, slicing-by-8) against the bitwise
    # definition on 20,000 random lengths, seeds and misalignments, plus
    # combine; built from the same source with the A/B harness
    exe = tmp_path / "scalar_ab"
    subprocess.run(["g++", "-O2", "-std=c++17", os.path.join(ROOT, "tools", "scalar_ab.cpp"),
                    "-o", str(exe)], check=True)
    r = subprocess.run([str(exe), "check"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and '"bad": 0' in r.stdout, r.stdout + r.stderr


def test_combine_long_lengths():
    # bmqcrc_combine over lengths past 32 bits (every bit of lenB a clmul
    # step) against the oracle's bit-serial combine
    rng = np.random.default_rng(43)
    for _ in range(200):
        a, b = (int(x) for x in rng.integers(0, 2**32, size=2))
        lb = int(rng.integers(0, 2**60))  # the oracle forms 8 * lenB in 64 bits
        assert Crc32c.combine(a, b, lb) == oracle.combine(a, b, lb)


def test_combine():
    rng = np.random.default_rng(41)
    for _ in range(40):
        a = rng.integers(0, 256, size=int(rng.integers(0, 5000)), dtype=np.uint8).tobytes()
        b = rng.integers(0, 256, size=int(rng.integers(0, 5000)), dtype=np.uint8).tobytes()
        assert Crc32c.combine(Crc32c.calculate(a), Crc32c.calculate(b), len(b)) == \
            Crc32c.calculate(a + b)


def test_cpp_dropin_selftest():
    exe = os.path.join(ROOT, "tests", "cpp", "bin", "bmqp_selftest")
    if not os.path.exists(exe):
        pytest.skip("selftest not built")
    env = dict(os.environ, BMQCRC_GOLDEN_DIR=os.path.join(ROOT, "tests", "golden"))
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASS" in r.stdout


def test_cpp_spellings_fall_back_without_gpu():
    """the reference's calls have no error channel, so the C++
    spellings at its call sites (bmqp::Crc32c::calculateBatch,
    PutEventCrc32c, FileStoreCrc32c, ClusterStateLedgerCrc32c) finish on the
    host, bit-exact, when no GPU is visible -- while the C-ABI batch calls
    still return BMQCRC_ENODEV (both checked inside the self-test)."""
    exe = os.path.join(ROOT, "tests", "cpp", "bin", "bmqp_selftest")
    if not os.path.exists(exe):
        pytest.skip("selftest not built")
    env = dict(os.environ, BMQCRC_GOLDEN_DIR=os.path.join(ROOT, "tests", "golden"),
               HIP_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASS" in r.stdout


@pytest.mark.skipif(device_count() > 0, reason="GPU present: batch path is exercised by -m gpu")
def test_batch_refuses_without_gpu():
    # the batch path never falls back to the CPU
    with pytest.raises(BmqCrcError) as e:
        Crc32c.calculate_batch(np.zeros(64, np.uint8), [0], [64])
    assert e.value.rc == -19


def test_batch_rejects_unknown_flags():
    import ctypes
    from blazingmq_amd import _native as N
    a = np.zeros(64, np.uint8)
    off = np.zeros(1, np.uint64)
    ln = np.full(1, 64, np.uint32)
    out = np.zeros(1, np.uint32)
    o = N.make_opts(flags=0x100)
    rc = N.lib.bmqcrc_crc32c_batch(a.ctypes.data, a.size, off.ctypes.data, ln.ctypes.data, None,
                                   out.ctypes.data, 1, ctypes.byref(o))
    assert rc == N.BMQCRC_EINVAL
    assert b"flags" in N.lib.bmqcrc_last_error()
    # the whole-messages flag is known: without a GPU it refuses with ENODEV
    o = N.make_opts(flags=N.BMQCRC_F_WHOLE_MESSAGES)
    rc = N.lib.bmqcrc_crc32c_batch(a.ctypes.data, a.size, off.ctypes.data, ln.ctypes.data, None,
                                   out.ctypes.data, 1, ctypes.byref(o))
    if N.lib.bmqcrc_device_count() == 0:
        assert rc == N.BMQCRC_ENODEV


def test_gather_refuses_without_gpu():
    """bmqcrc_crc32c_gather is a GPU-only batch entry point: ENODEV here, and
    argument errors are still reported first."""
    import ctypes
    from blazingmq_amd import _native as N
    bufs = [np.frombuffer(b"hello ", np.uint8), np.frombuffer(b"world", np.uint8)]
    ptrs = (ctypes.c_void_p * 2)(*[b.ctypes.data for b in bufs])
    lens = np.array([6, 5], np.uint32)
    first = np.array([0, 2], np.uint64)
    out = np.zeros(1, np.uint32)
    o = N.make_opts()
    assert N.lib.bmqcrc_crc32c_gather(ptrs, lens.ctypes.data, 2, first.ctypes.data, None,
                                      out.ctypes.data, 1, ctypes.byref(o)) == N.BMQCRC_ENODEV
    bad_first = np.array([1, 0], np.uint64)
    assert N.lib.bmqcrc_crc32c_gather(ptrs, lens.ctypes.data, 2, bad_first.ctypes.data, None,
                                      out.ctypes.data, 1, ctypes.byref(o)) == N.BMQCRC_EINVAL
    # the C++ Blob overload finishes on the host instead (checked in the self-test)


def test_host_register_refuses_without_gpu():
    import ctypes
    import numpy as np
    from blazingmq_amd import _native as N
    a = np.zeros(4096, np.uint8)
    p = ctypes.c_void_p()
    assert N.lib.bmqcrc_host_register(None, 16, -1, ctypes.byref(p)) == N.BMQCRC_EINVAL
    if N.lib.bmqcrc_device_count() == 0:
        assert N.lib.bmqcrc_host_register(a.ctypes.data, a.size, -1,
                                          ctypes.byref(p)) == N.BMQCRC_ENODEV
        assert N.lib.bmqcrc_host_unregister(a.ctypes.data) == N.BMQCRC_ENODEV


@pytest.mark.parametrize("bad", ["short", "dtype", "strided", "readonly", "list"])
def test_host_batch_rejects_bad_out(bad):
    """A caller-supplied `out` the C library would overrun is refused before
    the call (it writes 4 * n bytes)."""
    a = np.zeros(256, np.uint8)
    off, ln = np.arange(4, dtype=np.uint64) * 8, np.full(4, 8, np.uint32)
    out = {"short": np.zeros(3, np.uint32), "dtype": np.zeros(4, np.int64),
           "strided": np.zeros(8, np.uint32)[::2], "list": [0, 0, 0, 0]}.get(bad)
    if bad == "readonly":
        out = np.zeros(4, np.uint32)
        out.flags.writeable = False
    with pytest.raises(TypeError):
        Crc32c.calculate_batch(a, off, ln, out=out)


def test_torch_batch_rejects_bad_out_and_seeds():
    """Same for the torch form (CPU tensors stand in for device tensors: the
    checks run before any device call)."""
    import torch
    from blazingmq_amd import crc32c as C
    dev = torch.device("cpu")
    a = torch.zeros(256, dtype=torch.uint8)
    off = torch.arange(4, dtype=torch.int64) * 8
    ln = torch.full((4,), 8, dtype=torch.int32)
    for out in (torch.zeros(3, dtype=torch.int32), torch.zeros(4, dtype=torch.int64),
                torch.zeros(8, dtype=torch.int32)[::2]):
        with pytest.raises(TypeError):
            C._batch_torch(torch, a, off, ln, None, out, 0, None, True)
    with pytest.raises(TypeError):
        C._batch_torch(torch, a, off, ln, torch.zeros(8, dtype=torch.int32)[::2], None, 0, None,
                       True)
    assert dev.type == "cpu"
