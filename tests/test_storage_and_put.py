"""SURVEY 8(f) rows 1-2 on the host side: journal/DATA parsing (FileStore
recovery layout) against the reference's on-disk fixture, the partition
writer, and the PUT event builder/iterator wire format.  GPU parts are in
test_gpu_extensions.py."""
import os

import numpy as np
import pytest

import oracle
from blazingmq_amd import storage
from blazingmq_amd.put_event import PutEventBuilder, PutMessageIterator

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _fixture():
    return (np.fromfile(os.path.join(GOLD, "test.bmq_journal"), np.uint8),
            np.fromfile(os.path.join(GOLD, "test.bmq_data"), np.uint8))


def test_fixture_recovery_selection(golden):
    """bmqstoragetool's fixture: two MESSAGE records, the first confirmed and
    deleted (DELETION at 404), so recovery CRCs only the outstanding one
    (summary_result.txt: 1 outstanding; test_journalfile.py TEST_GUID_1)."""
    j, d = _fixture()
    rec = golden["recovery"]
    py = storage.recovery_selection_py(j, d)
    assert py["recovery_rc"] == 0
    assert py["record_offset"] == rec["outstanding_record_offsets"]
    assert len(py["record_offset"]) == rec["outstanding_messages"]
    guid = bytes.fromhex(rec["outstanding_guids"][0])
    r = int(py["record_offset"][0])
    assert j[r + 36:r + 52].tobytes() == guid
    assert py["crc32c"] == golden["journal_file"]["crc"][1:]
    o, n = py["app_offset"][0], py["app_length"][0]
    assert d[o:o + n].tobytes() == b"hello world"
    assert oracle.crc32c(d[o:o + n].tobytes()) == py["crc32c"][0]
    assert storage.journal_bounds_py(j) == (rec["last_valid_syncpoint_offset"],
                                            rec["last_valid_record_offset"])


def test_writer_reproduces_data_fixture():
    _, d = _fixture()
    j2, d2 = storage.write_partition([b"hello world", b"hello world"])
    assert np.array_equal(d2, d)
    r = storage.recovery_selection_py(j2, d2)
    assert r["crc32c"] == [3381945770, 3381945770]


def test_writer_roundtrip_random():
    rng = np.random.default_rng(2)
    apps = [rng.integers(0, 256, size=int(n), dtype=np.uint8).tobytes()
            for n in rng.integers(0, 3000, size=200)]
    j, d = storage.write_partition(apps)
    r = storage.recovery_selection_py(j, d)
    got = [d[o:o + n].tobytes() for o, n in zip(r["app_offset"], r["app_length"])]
    assert got[::-1] == apps  # backward journal order
    assert r["crc32c"][::-1] == [oracle.crc32c(a) for a in apps]


def test_preallocated_journal_tail_is_ignored():
    j, d = storage.write_partition([b"a", b"bc"])
    jz = np.concatenate([j, np.zeros(600, np.uint8)])
    assert len(storage.recovery_selection_py(jz, d)["crc32c"]) == 2


@pytest.mark.parametrize("corrupt", ["magic", "type"])
def test_invalid_files_raise(corrupt):
    j, d = storage.write_partition([b"hello world"])
    if corrupt == "magic":
        j[0] ^= 0xFF
        with pytest.raises(storage.StorageFormatError):
            storage.recovery_selection_py(j, d)
    else:
        with pytest.raises(storage.StorageFormatError):
            storage.recovery_selection_py(d, d)  # a DATA file is not a journal


def test_put_event_layout_and_roundtrip():
    b = PutEventBuilder(defer_crc=False)
    apps = [b"", b"a", b"abcd", b"x" * 13, bytes(range(256))]
    for i, a in enumerate(apps):
        b.pack_message(a, queue_id=i - 2, guid=bytes([i]) * 16, flags=i & 0xF)
    ev = b.finalize()
    # EventHeader: length, PV=1 / type PUT=2, header words 2
    assert int.from_bytes(ev[0:4].tobytes(), "big") == ev.size
    assert ev[4] == (1 << 6) | 2 and ev[5] == 2
    msgs = list(PutMessageIterator(ev))
    assert [m["app_data"] for m in msgs] == apps
    assert [m["queue_id"] for m in msgs] == [-2, -1, 0, 1, 2]
    assert [m["crc32c"] for m in msgs] == [oracle.crc32c(a) for a in apps]
    # PutHeader: 9 header words, messageWords covers header + data + 1..4 pad bytes
    pos = 8
    for a in apps:
        w0 = int.from_bytes(ev[pos:pos + 4].tobytes(), "big")
        w1 = int.from_bytes(ev[pos + 4:pos + 8].tobytes(), "big")
        assert w1 & 0x1F == 9
        total = (w0 & 0x0FFFFFFF) * 4
        pad = total - 36 - len(a)
        assert 1 <= pad <= 4 and ev[pos + total - 1] == pad
        assert (ev[pos + 36 + len(a):pos + total] == pad).all()
        pos += total
