"""GPU parts of SURVEY 8(f): batched recovery verification, deferred-CRC PUT
events and their batched iterator check, the batched Blob overload, and the
cluster state ledger's validateLog -- all through the C ABI
(include/bmqcrc.h, include/bmqcrc_protocol.h), bit-exact against the oracle
and the reference's fixtures."""
import os

import numpy as np
import pytest

import oracle
from blazingmq_amd import Blob, Crc32c, csl, storage
from blazingmq_amd.put_event import PutEventBuilder, PutMessageIterator

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_verify_fixture_partition(cuda, golden):
    j = np.fromfile(os.path.join(GOLD, "test.bmq_journal"), np.uint8)
    d = np.fromfile(os.path.join(GOLD, "test.bmq_data"), np.uint8)
    res = storage.verify_partition(j, d)
    # the first message is deleted: only the outstanding one is CRC'd
    assert res["n_messages"] == golden["recovery"]["outstanding_messages"] == 1
    assert res["n_bad"] == 0 and res["recovery_rc"] == 0
    d2 = d.copy()
    d2[52 + 3] ^= 1   # the deleted message's payload: no alarm
    assert storage.verify_partition(j, d2)["n_bad"] == 0
    d2[76 + 3] ^= 1   # the outstanding one's: alarm at its record
    res = storage.verify_partition(j, d2)
    assert res["n_bad"] == 1 and res["bad_record_offsets"].tolist() == [644]


def test_verify_rich_partition_alarms_only_on_live_messages(cuda):
    """Every skip rule of recoverMessages at once (deleted GUIDs, whole-queue
    purges, records before their queue's DELETION, a new lease), with the
    payload of every skipped message corrupted and one skipped DataHeader
    malformed: the GPU verify raises no alarm for them, CRCs exactly the
    outstanding messages bit-exact, and finds planted corruptions in live
    messages at their exact record offsets."""
    from test_recovery_selection import rich_partition
    j, d, expected, apps = rich_partition(seed=1)
    res = storage.verify_partition(j, d)
    assert res["recovery_rc"] == 0
    assert res["n_messages"] == len(expected) and res["n_bad"] == 0
    scan = storage.scan_partition(j, d)
    got = Crc32c.calculate_batch(d, scan["app_offset"].astype(np.int64),
                                 scan["app_length"].astype(np.int32))
    assert [int(x) for x in np.asarray(got).view(np.uint32)] == \
        [oracle.crc32c(d[int(o):int(o) + int(n)].tobytes())
         for o, n in zip(scan["app_offset"], scan["app_length"])]
    live = [i for i, n in enumerate(scan["app_length"]) if n > 0]
    victims = live[1::3]
    d2 = d.copy()
    for i in victims:
        d2[int(scan["app_offset"][i]) + int(scan["app_length"][i]) // 2] ^= 0x10
    res = storage.verify_partition(j, d2)
    assert res["n_bad"] == len(victims)
    assert res["bad_record_offsets"].tolist() == scan["record_offset"][victims].tolist()


def test_verify_detects_exact_corruptions(cuda):
    rng = np.random.default_rng(8)
    sizes = rng.integers(0, 20000, size=20000)
    apps = [rng.integers(0, 256, size=int(n), dtype=np.uint8).tobytes() for n in sizes]
    j, d = storage.write_partition(apps)
    res = storage.verify_partition(j, d)
    assert res["n_bad"] == 0 and res["n_messages"] == len(apps)
    scan = storage.scan_partition(j, d)  # backward journal order
    # flip one byte in the payload of some messages, and one stored CRC
    victims = sorted(set(int(i) for i in rng.integers(0, len(apps), size=37)
                         if scan["app_length"][int(i)] > 0))
    for i in victims:
        o = int(scan["app_offset"][i]) + int(rng.integers(0, int(scan["app_length"][i])))
        d[o] ^= 0x01
    jcrc_victim = next(i for i in range(len(apps)) if i not in victims)
    rec = int(scan["record_offset"][jcrc_victim])
    j[rec + 55] ^= 0x80
    res2 = storage.verify_partition(j, d)
    want = scan["record_offset"][sorted(victims + [jcrc_victim])]
    assert res2["n_bad"] == len(want)
    assert res2["bad_record_offsets"].tolist() == want.tolist()
    # bounded report: the first bad_cap alarms, full count
    res3 = storage.verify_partition(j, d, bad_cap=5)
    assert res3["n_bad"] == len(want) and res3["bad_record_offsets"].tolist() == want[:5].tolist()


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
    # the iterator-side batched check (bmqp_putmessageiterator.cpp:670-679)
    it = PutMessageIterator(evs[1])
    n, n_bad, bad = it.verify_crcs()
    assert (n, n_bad, bad.size) == (len(apps), 0, 0)
    off, ln, _ = it.scan()
    victims = [i for i in (3, 77, 499) if ln[i] > 0]
    ev = evs[1].copy()
    for i in victims:
        ev[int(off[i]) + int(ln[i]) // 2] ^= 0x10
    n, n_bad, bad = PutMessageIterator(ev).verify_crcs()
    assert (n, n_bad, bad.tolist()) == (len(apps), len(victims), victims)


def _oracle_record(advisory, **kw):
    """A ledger record whose CRC comes from the oracle, not from the product's
    scalar path (csl.append_record's default)."""
    body = csl.append_record(advisory, crc=0, **kw)[:-4]
    return body + oracle.crc32c(body).to_bytes(4, "big")


def _csl_log(n, rng, key=b"\x01\x02\x03\x04\x05"):
    recs = [_oracle_record(rng.integers(0, 256, size=int(rng.integers(1, 3000)),
                                        dtype=np.uint8).tobytes(),
                           record_type=int(rng.integers(1, 5)), elector_term=3,
                           sequence_number=i + 1, timestamp=123567 + i)
            for i in range(n)]
    return csl.file_header(key) + b"".join(recs), recs


def _fixture_ledger(golden):
    with open(os.path.join(GOLD, golden["csl"]["file"]), "rb") as f:
        return f.read(), bytes.fromhex(golden["csl"]["log_id"])


def test_csl_validate_reference_ledger(cuda, golden):
    """bmqstoragetool's broker-written ledger (test.bmq_csl, LogId 87EDF15DC0):
    the batched validateLog accepts it to its last byte; a flipped advisory
    byte in the SNAPSHOT at 388 (detail_csl_result.txt) or the COMMIT at 540
    is INVALID_CHECKSUM at that record; a wrong log id is INVALID_LOG_ID."""
    log, log_id = _fixture_ledger(golden)
    assert csl.validate_log(log, log_id) == (csl.SUCCESS, len(log), None) == \
        (csl.SUCCESS, 612, None)
    for rec in golden["csl"]["records"]:
        b = bytearray(log)
        b[rec["offset"] + 4 * rec["header_words"] + 5] ^= 0x20
        assert csl.validate_log(bytes(b), log_id) == (csl.INVALID_CHECKSUM, 0, rec["offset"])
    b = bytearray(log)
    b[540 + 4 * 18 - 1] ^= 0x01  # the COMMIT's stored CRC itself
    assert csl.validate_log(bytes(b), log_id) == (csl.INVALID_CHECKSUM, 0, 540)
    assert csl.validate_log(log, b"\x87\xed\xf1\x5d\xc1")[0] == csl.INVALID_LOG_ID


def test_csl_mode_recovery_of_reference_partition(cuda, golden):
    """The journal/DATA fixture recovered with the cluster state the ledger
    names (summary_csl_result.txt: key 26DACDC974): the outstanding message at
    644 is CRC'd and verifies; a cluster state without that key fails the
    CREATION at 104 (queueop_result.txt) with INVALID_QUEUE_KEY."""
    j = np.fromfile(os.path.join(GOLD, "test.bmq_journal"), np.uint8)
    d = np.fromfile(os.path.join(GOLD, "test.bmq_data"), np.uint8)
    key = bytes.fromhex(golden["csl"]["queue_key"])
    res = storage.verify_partition(j, d, with_csl=True, queue_keys=[key])
    assert (res["recovery_rc"], res["n_messages"], res["n_bad"]) == (0, 1, 0)
    d2 = d.copy()
    d2[76 + 3] ^= 1
    res = storage.verify_partition(j, d2, with_csl=True, queue_keys=[key])
    assert res["n_bad"] == 1 and res["bad_record_offsets"].tolist() == [644]
    res = storage.verify_partition(j, d, with_csl=True, queue_keys=[b"\x01\x02\x03\x04\x05"])
    assert (res["recovery_rc"], res["error_record_offset"]) == \
        (storage.RC_INVALID_QUEUE_KEY, golden["journal_queue_ops"]["creation"]["offset"])


def test_csl_validate_log(cuda):
    rng = np.random.default_rng(12)
    key = b"\x01\x02\x03\x04\x05"
    log, recs = _csl_log(3, rng, key)
    # mqbc_clusterstateledgerutil.t.cpp test4: valid log, then a record whose
    # size runs past the end of the log
    assert csl.validate_log(log, key) == (csl.SUCCESS, len(log), None)
    bad_hdr = bytes(csl.record_header(csl.UPDATE, 400))
    rc, _, _ = csl.validate_log(log + bad_hdr, key)
    assert rc == csl.REACHED_END_OF_LOG
    # test5: a record with an incorrect CRC
    wrong = csl.append_record(b"advisory", csl.UPDATE, 3, 8, 123567, crc=111111)
    assert oracle.crc32c(wrong[:-4]) != 111111
    assert csl.validate_log(log + wrong, key) == (csl.INVALID_CHECKSUM, 0, len(log))
    # a cleanly invalid record header ends the walk with success
    zeros = bytes(64)
    assert csl.validate_log(log + zeros, key) == (csl.SUCCESS, len(log), None)
    assert csl.validate_log(log, b"\x09" * 5)[0] == csl.INVALID_LOG_ID


def test_csl_validate_large_log_first_bad(cuda):
    rng = np.random.default_rng(13)
    log, recs = _csl_log(5000, rng)
    ends = np.cumsum([csl.FILE_HEADER_SIZE] + [len(r) for r in recs])
    assert csl.validate_log(log)[:2] == (csl.SUCCESS, len(log))
    b = bytearray(log)
    for k in (4100, 1234, 2500):  # the earliest corrupt record is reported
        b[int(ends[k]) + csl.RECORD_HEADER_SIZE] ^= 0x01  # first advisory byte
    assert csl.validate_log(bytes(b)) == (csl.INVALID_CHECKSUM, 0, int(ends[1234]))


@pytest.mark.parametrize("gather", [True, False])
def test_blobs_batch(cuda, golden, gather):
    blobs = [Blob(bytes.fromhex(h) for h in v["buffers_hex"]) for v in golden["blob"]]
    assert Crc32c.calculate_blobs(blobs, gather=gather).tolist() == \
        [v["crc"] for v in golden["blob"]]
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
    got = Crc32c.calculate_blobs(blobs, seeds=np.array(seeds, np.uint32), gather=gather)
    assert got.tolist() == exp
    # a shorter last data buffer (lastDataBufferLength, bmqp_crc32c.cpp:62-64)
    b = Blob([b"abcdefgh", b"ijklmnop"])
    b.set_last_data_buffer_length(3)
    assert Crc32c.calculate_blobs([b], gather=gather).tolist() == [oracle.crc32c(b"abcdefghijk")]


def test_gather_spans_many_staging_chunks(cuda):
    """bmqcrc_crc32c_gather over ~80 MiB of separately allocated buffers: more
    chunks than the pinned ring has slots (every slot reused, several gather
    threads), buffers and messages crossing chunk boundaries, empty buffers and
    empty messages, seeds; then the same call again on the warm workspace."""
    from blazingmq_amd import _native as N
    import ctypes
    rng = np.random.default_rng(31)
    sizes = rng.choice([0, 1, 7, 4096, 65536, 1 << 20, 3_000_001], size=90,
                       p=[.1, .1, .1, .3, .2, .15, .05])
    bufs = [rng.integers(0, 256, size=int(k), dtype=np.uint8) for k in sizes]
    cuts = np.sort(rng.choice(np.arange(1, len(bufs)), size=14, replace=False))
    first = np.concatenate([[0], cuts, [len(bufs)], [len(bufs)]]).astype(np.uint64)  # + empty msg
    n = first.size - 1
    seeds = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    ptrs = (ctypes.c_void_p * len(bufs))(*[b.ctypes.data for b in bufs])
    lens = np.array([b.size for b in bufs], np.uint32)
    exp = [oracle.blob([bufs[k].tobytes() for k in range(int(first[m]), int(first[m + 1]))],
                       int(seeds[m])) for m in range(n)]
    for _ in range(2):
        out = np.zeros(n, np.uint32)
        o = N.make_opts()
        N.check(N.lib.bmqcrc_crc32c_gather(ptrs, lens.ctypes.data, len(bufs), first.ctypes.data,
                                           seeds.ctypes.data, out.ctypes.data, n, ctypes.byref(o)))
        assert out.tolist() == exp
    # host pointers only
    o = N.make_opts(flags=N.BMQCRC_F_DEVICE_PTRS)
    assert N.lib.bmqcrc_crc32c_gather(ptrs, lens.ctypes.data, len(bufs), first.ctypes.data, None,
                                      out.ctypes.data, n, ctypes.byref(o)) == N.BMQCRC_EINVAL


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_walks_spread_over_devices(cuda, devices):
    """bmqcrc_opts.ndevices (ABI 2.1): the format-walk entry points cut the
    input buffer into byte ranges, stage and verify each on its own device
    listing (here the one GPU listed several times: each listing is its own
    stream and workspace), messages straddling a cut on the first listing.
    Results equal the single-device call exactly: counts, alarm offsets and
    their order, bounded reports, filled CRCs, the ledger's first bad record."""
    rng = np.random.default_rng(40)
    sizes = rng.integers(0, 30000, size=6000)
    apps = [rng.integers(0, 256, size=int(k), dtype=np.uint8).tobytes() for k in sizes]
    j, d = storage.write_partition(apps)
    scan = storage.scan_partition(j, d)
    live = [i for i in range(len(apps)) if scan["app_length"][i] > 0]
    victims = sorted(int(v) for v in rng.choice(live, size=41, replace=False))
    for i in victims:
        d[int(scan["app_offset"][i]) + int(scan["app_length"][i]) - 1] ^= 0x04
    one = storage.verify_partition(j, d)
    many = storage.verify_partition(j, d, devices=devices)
    assert one["n_bad"] == many["n_bad"] == len(victims)
    assert many["bad_record_offsets"].tolist() == one["bad_record_offsets"].tolist() == \
        scan["record_offset"][victims].tolist()
    assert storage.verify_partition(j, d, bad_cap=7, devices=devices)[
        "bad_record_offsets"].tolist() == one["bad_record_offsets"][:7].tolist()
    from test_recovery_selection import rich_partition
    rj, rd, expected, _ = rich_partition(seed=2)
    r1, rm = storage.verify_partition(rj, rd), storage.verify_partition(rj, rd, devices=devices)
    assert (rm["n_messages"], rm["n_bad"], rm["recovery_rc"]) == \
        (r1["n_messages"], r1["n_bad"], r1["recovery_rc"]) == (len(expected), 0, 0)
    # PUT events: deferred fill over several listings == immediate CRCs
    papps = [rng.integers(0, 256, size=int(k), dtype=np.uint8).tobytes()
             for k in rng.integers(0, 9000, size=700)]
    evs = []
    for defer, devs in ((False, None), (True, devices)):
        b = PutEventBuilder(defer_crc=defer, devices=devs)
        for i, a in enumerate(papps):
            b.pack_message(a, queue_id=i, guid=i.to_bytes(16, "big"))
        evs.append(b.finalize())
    assert np.array_equal(evs[0], evs[1])
    off, ln, _ = PutMessageIterator(evs[1]).scan()
    ev = evs[1].copy()
    pv = [i for i in (5, 300, 699) if ln[i] > 0]
    for i in pv:
        ev[int(off[i])] ^= 0x01
    n, n_bad, bad = PutMessageIterator(ev).verify_crcs(devices=devices)
    assert (n, n_bad, bad.tolist()) == (len(papps), len(pv), pv)
    # ledger: the first corrupt record, as with one device
    log, recs = _csl_log(3000, rng)
    ends = np.cumsum([csl.FILE_HEADER_SIZE] + [len(r) for r in recs])
    b = bytearray(log)
    for k in (2900, 1500, 2000):
        b[int(ends[k]) + csl.RECORD_HEADER_SIZE] ^= 0x01
    assert csl.validate_log(bytes(b), devices=devices) == csl.validate_log(bytes(b)) == \
        (csl.INVALID_CHECKSUM, 0, int(ends[1500]))
    assert csl.validate_log(log, devices=devices)[:2] == (csl.SUCCESS, len(log))


def test_gather_edges(cuda):
    """bmqcrc_crc32c_gather edge cases: no buffers at all (every message the
    seed), buffers outside [msg_first_buf[0], msg_first_buf[n]) ignored, one
    buffer, a NULL pointer with length 0, and the Blob overload's seeds."""
    from blazingmq_amd import _native as N
    import ctypes

    def run(bufs, first, seeds=None):
        keep = [np.frombuffer(b, np.uint8) if b is not None else None for b in bufs]
        ptrs = (ctypes.c_void_p * max(len(keep), 1))(
            *[k.ctypes.data if k is not None and k.size else None for k in keep])
        lens = np.array([0 if k is None else k.size for k in keep] or [0], np.uint32)
        fb = np.asarray(first, np.uint64)
        n = fb.size - 1
        sd = None if seeds is None else np.asarray(seeds, np.uint32)
        out = np.zeros(max(n, 1), np.uint32)
        o = N.make_opts()
        N.check(N.lib.bmqcrc_crc32c_gather(ptrs, lens.ctypes.data, len(bufs), fb.ctypes.data,
                                           sd.ctypes.data if sd is not None else None,
                                           out.ctypes.data, n, ctypes.byref(o)))
        return out[:n].tolist()

    assert run([], [0, 0, 0], seeds=[7, 0xFFFFFFFF]) == [7, 0xFFFFFFFF]
    assert run([b"skip", b"hello world", b"skip too"], [1, 2]) == [oracle.crc32c(b"hello world")]
    assert run([b"abc", None, b"def"], [0, 3], seeds=[5]) == [oracle.crc32c(b"abcdef", 5)]
    assert run([b"x" * 5000], [0, 1, 1]) == [oracle.crc32c(b"x" * 5000), 0]
