"""GPU parts of SURVEY 8(f): batched recovery verification, deferred-CRC PUT
events and the batched Blob overload -- all through the C ABI, bit-exact
against the oracle and the reference's fixtures."""
import os

import numpy as np
import pytest

import oracle
from blazingmq_amd import Blob, Crc32c, storage
from blazingmq_amd.put_event import PutEventBuilder, PutMessageIterator

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_verify_fixture_partition(cuda):
    j = np.fromfile(os.path.join(GOLD, "test.bmq_journal"), np.uint8)
    d = np.fromfile(os.path.join(GOLD, "test.bmq_data"), np.uint8)
    res = storage.verify_partition(j, d)
    assert res["n_messages"] == 2 and res["n_bad"] == 0


def test_verify_detects_exact_corruptions(cuda):
    rng = np.random.default_rng(8)
    sizes = rng.integers(0, 20000, size=20000)
    apps = [rng.integers(0, 256, size=int(n), dtype=np.uint8).tobytes() for n in sizes]
    j, d = storage.write_partition(apps)
    res = storage.verify_partition(j, d)
    assert res["n_bad"] == 0 and res["n_messages"] == len(apps)
    # flip one byte in the payload of some messages, and one stored CRC
    victims = sorted(set(int(i) for i in rng.integers(0, len(apps), size=37)
                         if sizes[int(i)] > 0))
    for i in victims:
        o = int(res["app_offset"][i]) + int(rng.integers(0, sizes[i]))
        d[o] ^= 0x01
    jcrc_victim = next(i for i in range(len(apps)) if i not in victims)
    rec = int(res["records"]["record_offset"][jcrc_victim])
    j[rec + 55] ^= 0x80
    res2 = storage.verify_partition(j, d)
    assert res2["bad_index"].tolist() == sorted(victims + [jcrc_victim])


def test_put_event_deferred_equals_immediate(cuda):
    rng = np.random.default_rng(9)
    apps = [rng.integers(0, 256, size=int(n), dtype=np.uint8).tobytes()
            for n in rng.integers(0, 70000, size=500)]
    evs = []
    for defer in (False, True):
        b = PutEventBuilder(defer_crc=defer)
        for i, a in enumerate(apps):
            b.pack_message(a, queue_id=i, guid=i.to_bytes(16, "big"))
        evs.append(b.finalize())
    assert np.array_equal(evs[0], evs[1])
    assert [m["crc32c"] for m in PutMessageIterator(evs[1])] == [oracle.crc32c(a) for a in apps]


def test_blobs_batch(cuda, golden):
    blobs = [Blob(bytes.fromhex(h) for h in v["buffers_hex"]) for v in golden["blob"]]
    assert Crc32c.calculate_blobs(blobs).tolist() == [v["crc"] for v in golden["blob"]]
    rng = np.random.default_rng(10)
    blobs, seeds, exp = [], [], []
    for _ in range(400):
        nb = int(rng.integers(0, 12))
        parts = [rng.integers(0, 256, size=int(rng.choice([0, 1, 3, 100, 4096, 9000])),
                              dtype=np.uint8).tobytes() for _ in range(nb)]
        seed = int(rng.integers(0, 2**32)) if rng.random() < 0.5 else 0
        blobs.append(Blob(parts))
        seeds.append(seed)
        exp.append(oracle.blob(parts, seed))
    got = Crc32c.calculate_blobs(blobs, seeds=np.array(seeds, np.uint32))
    assert got.tolist() == exp
