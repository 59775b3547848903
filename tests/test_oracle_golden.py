"""Pin the CPU oracle to the reference's own golden vectors.

Every oracle variant must reproduce bmqp_crc32c.t.cpp's constants, RFC 3720
B.4, and the CRC stored in the bmqstoragetool DATA/journal fixture, before it
may serve as the checker for the GPU path.
"""
import os

import numpy as np
import pytest

import oracle

VARIANTS = ["bitwise", "sw", "hw_serial", "hw"]


@pytest.mark.parametrize("variant", VARIANTS)
def test_calculate_vectors(golden, variant):
    for v in golden["calculate"] + golden["rfc3720"]:
        assert oracle.crc32c(bytes.fromhex(v["hex"]), 0, variant) == v["crc"], v


@pytest.mark.parametrize("variant", VARIANTS)
def test_chained_vectors(golden, variant):
    for v in golden["chained"]:
        b, p = bytes.fromhex(v["hex"]), v["prefix_len"]
        c = oracle.crc32c(b[p:], oracle.crc32c(b[:p], 0, variant), variant)
        assert c == v["crc"]
        assert oracle.crc32c(b"", c, variant) == c  # (buf, 0, prev) -> prev


def test_blob_vectors(golden):
    for v in golden["blob"]:
        assert oracle.blob([bytes.fromhex(h) for h in v["buffers_hex"]]) == v["crc"]
    for v in golden["blob_chained"]:
        c = v.get("seed", 0)
        for blob in v["blobs_hex"]:
            c = oracle.blob([bytes.fromhex(h) for h in blob], c)
        assert c == v["crc"]


def test_data_file_fixture(golden):
    df = golden["data_file"]
    data = np.fromfile(os.path.join(os.path.dirname(__file__), "golden", df["file"]), np.uint8)
    assert data.size == 88
    for r in df["records"]:
        s = r["record_offset"] + r["header_bytes"]
        app = data[s:s + r["app_data_len"]].tobytes()
        assert app == b"hello world"
        assert oracle.crc32c(app) == r["crc"] == 3381945770


@pytest.mark.parametrize("variant", ["sw", "hw_serial", "hw"])
def test_variants_agree_random(variant):
    rng = np.random.default_rng(3)
    for n in list(range(0, 70)) + [255, 256, 257, 768, 769, 24575, 24576, 24577, 80000]:
        buf = rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()
        seed = int(rng.integers(0, 2**32))
        assert oracle.crc32c(buf, seed, variant) == oracle.crc32c(buf, seed, "bitwise")


def test_combine_property():
    rng = np.random.default_rng(4)
    for _ in range(50):
        a = rng.integers(0, 256, size=int(rng.integers(0, 3000)), dtype=np.uint8).tobytes()
        b = rng.integers(0, 256, size=int(rng.integers(0, 3000)), dtype=np.uint8).tobytes()
        assert oracle.combine(oracle.crc32c(a), oracle.crc32c(b), len(b)) == oracle.crc32c(a + b)


def test_batch_threads_match_serial():
    rng = np.random.default_rng(9)
    lens = rng.integers(0, 5000, size=500)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    arena = rng.integers(0, 256, size=int(lens.sum()) + 1, dtype=np.uint8)
    seeds = rng.integers(0, 2**32, size=500, dtype=np.uint64).astype(np.uint32)
    exp = [oracle.crc32c(arena[int(o):int(o) + int(l)].tobytes(), int(s))
           for o, l, s in zip(offs, lens, seeds)]
    for t in (1, 3, 8):
        assert oracle.batch(arena, offs, lens, seeds, nthreads=t).tolist() == exp


def test_fill_payload_is_counter_based():
    a = oracle.fill_payload(0, 4096, 17)
    assert np.array_equal(oracle.fill_payload(1000, 96, 17), a[1000:1096])
    assert not np.array_equal(oracle.fill_payload(0, 64, 18), a[:64])
