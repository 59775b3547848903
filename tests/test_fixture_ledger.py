"""The reference's own on-disk fixtures for the ledger and the journal's queue
records, on the CPU (the GPU validate/verify over the same files is in
test_gpu_extensions.py).

* test.bmq_csl -- a broker-written cluster state ledger
  (src/applications/bmqstoragetool/integration-tests/data/), with what
  bmqstoragetool prints for it: detail_csl_result.txt / short_csl_result.txt
  (SNAPSHOT at 388, COMMIT at 540, LogId 87EDF15DC0), summary_csl_result.txt
  (queue key 26DACDC974) and test_cslfile.py's searches.
* queueop_result.txt / summary_queueop_journalop_result.txt -- the journal's
  QueueOp CREATION at 104 and its record counts.
* journalop_result.txt -- the journal's eight SYNCPOINT records (offset, PSN,
  epoch, sync point type and PSN, node, DATA offset); with them the recovery
  walk's sync point checks (mqbs_filestore.cpp:1647-1713) are pinned to the
  reference's own file: mutating one sync point's PSN gives the reference's
  rc at that record, in the native walk and in the Python restatement.
* summary_result_with_queue_info.txt -- per-queue record counts, message
  counts and the journal's last sync point.

All extracted into tests/golden/crc32c_vectors.json by make_golden.py.  The
native ledger walk (bmqcrc_csl_scan) must find these records, and every CRC
stored in the ledger must equal the ORACLE's CRC of the record's bytes
(mqbc_clusterstateledgerutil.cpp:309,411: the CRC covers header, advisory and
padding).  CSL-mode recovery of the journal fixture with the ledger's key
(mqbs_filestore.cpp:1120-1453) selects exactly the outstanding message."""
import os

import numpy as np
import pytest

import oracle
from blazingmq_amd import csl
from blazingmq_amd import storage as S

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _ledger(golden):
    with open(os.path.join(GOLD, golden["csl"]["file"]), "rb") as f:
        return f.read()


def _records(log):
    """(offset, type, elector term, sequence number, header words, advisory
    words, timestamp) of every record the native walk finds."""
    wrc, end, off, ln, crc = csl.scan_log(log)
    out = []
    for o in off.tolist():
        h = log[o:o + 32]
        out.append((o, h[0] & 0xF, int.from_bytes(h[8:16], "big"),
                    int.from_bytes(h[16:24], "big"), h[0] >> 4,
                    int.from_bytes(h[4:8], "big") & 0x0FFFFFFF, int.from_bytes(h[24:32], "big")))
    return wrc, end, off, ln, crc, out


def test_ledger_walk_finds_the_records_bmqstoragetool_prints(golden):
    log = _ledger(golden)
    g = golden["csl"]
    log_id = bytes.fromhex(g["log_id"])
    assert log[1:6] == log_id                      # ClusterStateFileHeader file key
    wrc, end, off, ln, crc, recs = _records(log)
    assert (wrc, end) == (0, len(log)) == (0, 612)
    assert csl.scan_log(log, log_id)[:2] == (0, 612)
    by_off = {r[0]: r for r in recs}
    for want in g["records"]:                       # detail_csl_result.txt
        o, t, term, seq, hw, aw, ts = by_off[want["offset"]]
        assert (t, term, seq, hw, aw, ts) == (want["type"], want["elector_term"],
                                               want["sequence_number"], want["header_words"],
                                               want["advisory_words"], want["epoch"])
    # the record after each printed one starts where its words end
    starts = [r[0] for r in recs]
    for r in recs[:-1]:
        assert starts[starts.index(r[0]) + 1] == r[0] + 4 * (r[4] + r[5])
    assert recs[-1][0] + 4 * (recs[-1][4] + recs[-1][5]) == len(log)
    # test_cslfile.py's searches
    s = g["search"]
    o, t, term, seq = by_off[s["commit_at"]["offset"]][:4]
    assert (t, term, seq) == (csl.COMMIT, s["commit_at"]["elector_term"],
                              s["commit_at"]["sequence_number"])
    assert s["not_a_record"] not in by_off
    assert sum(r[1] == csl.SNAPSHOT for r in recs) == s["snapshots_from_begin"]
    between = [r[1] for r in recs if s["between"]["gt"] < r[0] < s["between"]["lt"]]
    assert {str(t): between.count(t) for t in (1, 2, 3, 4)} == s["between"]["counts"]


def test_every_stored_ledger_crc_equals_the_oracle(golden):
    log = _ledger(golden)
    _, _, off, ln, crc, _ = _records(log)
    assert off.size == 6
    for o, n, c in zip(off.tolist(), ln.tolist(), crc.tolist()):
        assert int.from_bytes(log[o + n:o + n + 4], "big") == c
        assert oracle.crc32c(log[o:o + n]) == c
        assert oracle.crc32c(log[o:o + n], 0, "bitwise") == c


def test_ledger_scan_rejects_a_foreign_log_id(golden):
    log = _ledger(golden)
    wrc, _, _, _, _ = csl.scan_log(log, b"\x00\x01\x02\x03\x04")
    assert wrc == csl.INVALID_LOG_ID


def _journal():
    return (np.fromfile(os.path.join(GOLD, "test.bmq_journal"), np.uint8),
            np.fromfile(os.path.join(GOLD, "test.bmq_data"), np.uint8))


def test_journal_queue_records_match_bmqstoragetool(golden):
    """queueop_result.txt: the CREATION at 104 (lease 1, seq 2, QLIST offset
    words 9, the ledger's key); summary_queueop_journalop_result.txt: one
    QueueOp and eight JournalOp records in the journal."""
    j, _ = _journal()
    q = golden["journal_queue_ops"]
    c = q["creation"]
    r = j[c["offset"]:c["offset"] + S.JOURNAL_RECORD_SIZE].tobytes()
    assert r[0] >> 4 == S.REC_QUEUE_OP
    assert r[22:27] == bytes.fromhex(c["queue_key"]) == bytes.fromhex(golden["csl"]["queue_key"])
    assert r[27:32] == bytes.fromhex(c["app_key"])
    assert int.from_bytes(r[32:36], "big") == S.OP_CREATION
    assert int.from_bytes(r[8:12], "big") == c["primary_lease_id"]
    assert (int.from_bytes(r[2:4], "big") << 32 | int.from_bytes(r[4:8], "big")) == \
        c["sequence_number"]
    assert int.from_bytes(r[36:40], "big") == c["qlist_offset_words"]
    _, last = S.journal_bounds(j)
    fh = S.parse_file_header(j, S.FILE_TYPE_JOURNAL)
    start = fh + int(j[fh]) * S.WORD              # the first record, after the JournalFileHeader
    types = [int(j[p]) >> 4 for p in range(start, last + 1, S.JOURNAL_RECORD_SIZE)]
    assert types.count(S.REC_QUEUE_OP) == q["queue_op_records"] == q["creation_ops"] == 1
    assert types.count(S.REC_JOURNAL_OP) == q["journal_op_records"] == 8


def test_csl_mode_recovery_with_the_ledgers_queue_key(golden):
    """With CSL, the cluster state is the ledger's one queue (26DACDC974):
    recovery selects exactly the outstanding message (644) with rc 0; a
    cluster state without that key fails the CREATION at 104 with
    INVALID_QUEUE_KEY (mqbs_filestore.cpp:1391-1402)."""
    j, d = _journal()
    key = bytes.fromhex(golden["csl"]["queue_key"])
    for fn in (S.scan_partition, S.recovery_selection_py):
        r = fn(j, d, with_csl=True, queue_keys=[key])
        assert r["recovery_rc"] == 0
        assert list(r["record_offset"]) == golden["recovery"]["outstanding_record_offsets"] == [644]
        o, n = int(r["app_offset"][0]), int(r["app_length"][0])
        assert oracle.crc32c(d[o:o + n].tobytes()) == int(r["crc32c"][0]) == \
            golden["journal_file"]["crc"][1]
        r = fn(j, d, with_csl=True, queue_keys=[b"\x26\xda\xcd\xc9\x75"])
        assert (r["recovery_rc"], r["error_record_offset"]) == \
            (S.RC_INVALID_QUEUE_KEY, golden["journal_queue_ops"]["creation"]["offset"])


def _be(r, off, n):
    return int.from_bytes(r[off:off + n], "big")


def _record_offsets(j):
    _, last = S.journal_bounds(j)
    fh = S.parse_file_header(j, S.FILE_TYPE_JOURNAL)
    start = fh + int(j[fh]) * S.WORD
    return start, list(range(start, last + 1, S.JOURNAL_RECORD_SIZE))


def test_journal_sync_points_match_bmqstoragetool(golden):
    """journalop_result.txt, field by field from the file (JournalOpRecord,
    mqbs_filestoreprotocol.h:1953: sync point type @23, JournalOpType @24,
    SyncPt sequence @28/@32, node @36, SyncPt lease @40, DATA offset dwords
    @44), and summary_result_with_queue_info.txt's last sync point (the
    native journal bounds and the Python restatement agree with it)."""
    j, _ = _journal()
    g = golden["journal_ops"]
    start, offs = _record_offsets(j)
    jops = [o for o in offs if int(j[o]) >> 4 == S.REC_JOURNAL_OP]
    assert jops == [r["offset"] for r in g["records"]] and len(jops) == g["count"] == 8
    for want in g["records"]:
        r = j[want["offset"]:want["offset"] + S.JOURNAL_RECORD_SIZE].tobytes()
        assert (want["offset"] - start) // S.JOURNAL_RECORD_SIZE == want["index"]
        assert _be(r, 8, 4) == want["primary_lease_id"]
        assert (_be(r, 2, 2) << 32 | _be(r, 4, 4)) == want["sequence_number"]
        assert _be(r, 12, 8) == want["epoch"]
        assert r[23] == want["sync_point_type"] and _be(r, 24, 4) == S.JOURNAL_OP_SYNCPOINT
        assert (_be(r, 28, 4) << 32 | _be(r, 32, 4)) == want["sync_pt_sequence_number"]
        assert _be(r, 36, 4) == want["primary_node_id"]
        assert _be(r, 40, 4) == want["sync_pt_primary_lease_id"]
        assert _be(r, 44, 4) == want["data_file_offset_dwords"]
    ls = golden["queue_summary"]["last_sync_point"]
    assert S.journal_bounds(j) == S.journal_bounds_py(j) == (ls["offset"],
                                                           ls["last_valid_record_offset"])
    r = j[ls["offset"]:ls["offset"] + S.JOURNAL_RECORD_SIZE].tobytes()
    assert (_be(r, 28, 4) << 32 | _be(r, 32, 4)) == ls["sequence_number"]
    assert (_be(r, 40, 4), _be(r, 36, 4), _be(r, 12, 8)) == (ls["primary_lease_id"],
                                                            ls["primary_node_id"], ls["epoch"])
    assert (_be(r, 44, 4), _be(r, 48, 4)) == (ls["data_file_offset_dwords"],
                                              ls["qlist_file_offset_words"])


def _mutate(j, off, field_off, value, n=4):
    m = j.copy()
    m[off + field_off:off + field_off + n] = np.frombuffer(value.to_bytes(n, "big"), np.uint8)
    return m


@pytest.mark.parametrize("at", [764, 704, 584, 524, 164])
def test_sync_point_mutations_give_the_references_codes(golden, at):
    """The recovery walk's sync point checks in the reference's order
    (mqbs_filestore.cpp:1647-1713) on the reference's journal: a sync point
    whose SyncPt sequence number disagrees with the PSN chain fails with
    rc_INVALID_SEQ_NUMBER at that record, one whose SyncPt lease id is ahead
    of its record's (or zero) with rc_INVALID_PRIMARY_LEASE_ID, a zero SyncPt
    sequence with rc_INVALID_SEQ_NUMBER, a DATA offset past the DATA file with
    rc_INVALID_DATA_OFFSET (:1589-1606).  Native walk and Python restatement
    alike; the unmodified journal recovers with rc 0."""
    j, d = _journal()
    want = {r["offset"]: r for r in golden["journal_ops"]["records"]}[at]
    sp_seq, sp_lease = want["sync_pt_sequence_number"], want["sync_pt_primary_lease_id"]
    cases = [
        (_mutate(j, at, 32, (sp_seq + 1) & 0xFFFFFFFF), S.RC_INVALID_SEQ_NUMBER),
        (_mutate(_mutate(j, at, 28, 0), at, 32, 0), S.RC_INVALID_SEQ_NUMBER),
        (_mutate(j, at, 40, sp_lease + 1), S.RC_INVALID_PRIMARY_LEASE_ID),
        (_mutate(j, at, 40, 0), S.RC_INVALID_PRIMARY_LEASE_ID),
        (_mutate(j, at, 44, d.size // S.DWORD + 1), S.RC_INVALID_DATA_OFFSET),
    ]
    for fn in (S.scan_partition, S.recovery_selection_py):
        assert fn(j, d)["recovery_rc"] == 0
        for m, rc in cases:
            r = fn(m, d)
            assert (r["recovery_rc"], r["error_record_offset"]) == (rc, at), (fn, rc)


def test_queue_record_counts_match_bmqstoragetool(golden):
    """summary_result_with_queue_info.txt: queue 26DACDC974 has 4 records --
    2 MESSAGE, 1 CONFIRM, 1 DELETION (bmqstoragetool's summary leaves the
    queue's QueueOp CREATION out unless asked; summary_queueop_journalop
    counts it) -- of 2 messages 1 is confirmed and 1 outstanding, and that
    one is what recovery CRCs."""
    j, d = _journal()
    q = golden["queue_summary"]
    queue = q["queues"][0]
    key = bytes.fromhex(queue["queue_key"])
    assert queue["queue_key"] == golden["csl"]["queue_key"]
    _, offs = _record_offsets(j)
    key_at = {S.REC_MESSAGE: 22, S.REC_CONFIRM: 22, S.REC_DELETION: 23, S.REC_QUEUE_OP: 22}
    counts = {t: 0 for t in key_at}
    for o in offs:
        t = int(j[o]) >> 4
        if t in key_at and j[o + key_at[t]:o + key_at[t] + 5].tobytes() == key:
            counts[t] += 1
    assert counts[S.REC_MESSAGE] == queue["message_records"] == q["total_messages"] == 2
    assert counts[S.REC_CONFIRM] == queue["confirm_records"] == 1
    assert counts[S.REC_DELETION] == queue["delete_records"] == 1
    assert counts[S.REC_MESSAGE] + counts[S.REC_CONFIRM] + counts[S.REC_DELETION] == \
        queue["total_records"] == q["total_records"] == 4
    assert counts[S.REC_QUEUE_OP] == golden["journal_queue_ops"]["creation_ops"] == 1
    assert queue["queue_op_records"] == 0
    for fn in (S.scan_partition, S.recovery_selection_py):
        r = fn(j, d)
        assert len(r["record_offset"]) == q["outstanding"] == 1
        assert q["total_messages"] - q["outstanding"] == q["confirmed"] == 1
