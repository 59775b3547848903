#!/usr/bin/env python3
"""Extract the reference's CRC32C golden vectors into tests/golden/crc32c_vectors.json.

Run in the build container (where /root/reference exists); the JSON it writes
is the committed fixture -- the GPU box never reads /root/reference.

Sources (all in /root/reference, read as text):
  * src/groups/bmq/bmqp/bmqp_crc32c.t.cpp
      test1 breathing "12345678" -> 0x6087809A              (:311-319)
      test2 table {line, buffer, crc}                        (:416-434)
      test4 table {line, buffer, prefixLen, crc}             (:604-622)
      test7/8 blob "one"+"two"+"three" -> 0xA0EA6901         (:845, :970)
      test7/8 277-byte sentence + 550 '#' -> 0xD86F726E      (:854-881, :980-1022)
  * src/applications/bmqstoragetool/integration-tests/data/test.bmq_data
      and test.bmq_journal (copied verbatim) with the journal CRC printed by
      bmqstoragetool in detail_result.txt:15,53 (3381945770) for the two
      MESSAGE records at DATA offsets 40 and 64 (payload_dump.txt).
  * src/applications/bmqstoragetool/integration-tests/data/test.bmq_csl (copied
      verbatim): a broker-written cluster state ledger, with what
      bmqstoragetool prints for it -- detail_csl_result.txt (SNAPSHOT@388,
      COMMIT@540, LogId 87EDF15DC0, sequence numbers, header and advisory
      words), short_csl_result.txt, summary_csl_result.txt (the one queue and
      its key 26DACDC974) and test_cslfile.py's searches (a COMMIT at offset
      316 with seqnum 1-4, none at 317; two SNAPSHOTs from the beginning; one
      UPDATE and one COMMIT strictly between offsets 88 and 388).
  * queueop_result.txt / summary_queueop_journalop_result.txt: the journal's
      QueueOp CREATION at offset 104 for that key, and its record counts.
  * journalop_result.txt: every JOURNAL_OP sync point of the journal (index,
      offset, PSN, epoch, sync point type, SyncPt PSN, node, DATA offset).
  * summary_result_with_queue_info.txt: per-queue record counts (queue
      26DACDC974: 2 message, 1 confirm, 1 delete, 4 records), message counts
      and the journal's last sync point (offset 764, PSN 2/4, DATA 11 dwords,
      QLIST 32 words).
  * RFC 3720 section B.4 (iSCSI CRC32C test patterns) as external known answers.
"""
import json
import os
import re
import shutil
import sys

REF = "/root/reference"
T_CPP = os.path.join(REF, "src/groups/bmq/bmqp/bmqp_crc32c.t.cpp")
DATA_DIR = os.path.join(REF, "src/applications/bmqstoragetool/integration-tests/data")
HERE = os.path.dirname(os.path.abspath(__file__))


def c_unescape(s):
    return s.encode("latin-1").decode("unicode_escape").encode("latin-1")


def table_rows(src, start_marker):
    i = src.index(start_marker)
    j = src.index("};", i)
    return src[i:j]


def main():
    src = open(T_CPP, encoding="latin-1").read()
    out = {"source": "bmqp_crc32c.t.cpp + bmqstoragetool fixture + RFC3720 B.4"}

    # test2 (first k_DATA table after test2_calculateOnBuffer)
    t2 = table_rows(src[src.index("static void test2_calculateOnBuffer"):], "k_DATA[] =")
    vec2 = [(c_unescape(b), int(c, 0))
            for b, c in re.findall(r'\{L_,\s*"((?:[^"\\]|\\.)*)",\s*(0x[0-9A-Fa-f]+|0)\}', t2)]
    assert len(vec2) == 19, len(vec2)
    out["calculate"] = [{"hex": b.hex(), "text": b.decode("latin-1"), "crc": c} for b, c in vec2]
    out["calculate"].insert(0, {"hex": b"12345678".hex(), "text": "12345678", "crc": 0x6087809A})

    # test4 chained table
    t4 = table_rows(src[src.index("static void test4_calculateOnBufferWithPreviousCrc"):],
                    "k_DATA[] =")
    vec4 = [(c_unescape(b), int(p), int(c, 0)) for b, p, c in re.findall(
        r'\{L_,\s*"((?:[^"\\]|\\.)*)",\s*(\d+),\s*(0x[0-9A-Fa-f]+|0)\}', t4)]
    assert len(vec4) == 19, len(vec4)
    out["chained"] = [{"hex": b.hex(), "prefix_len": p, "crc": c} for b, p, c in vec4]

    # test7 blobs
    t7 = src[src.index("static void test7_calculateOnBlob"):
             src.index("static void test8_calculateOnBlobWithPreviousCrc")]
    assert "0xA0EA6901" in t7 and "0xD86F726E" in t7
    m = re.search(r'char buf\[\] = ((?:\s*"(?:[^"\\]|\\.)*")+);', t7)
    sentence = b"".join(c_unescape(x) for x in re.findall(r'"((?:[^"\\]|\\.)*)"', m.group(1)))
    out["blob"] = [
        {"buffers_hex": [b"one".hex(), b"two".hex(), b"three".hex()], "crc": 0xA0EA6901},
        {"buffers_hex": [sentence.hex()], "crc": 0xD86F726E},
        {"buffers_hex": [], "crc": 0},
    ]
    # test8: same content split over two blobs, chained through the CRC
    t8 = src[src.index("static void test8_calculateOnBlobWithPreviousCrc"):]
    m1 = re.search(r'char one\[\] = ((?:\s*"(?:[^"\\]|\\.)*")+);', t8)
    m2 = re.search(r'char two\[\] = ((?:\s*"(?:[^"\\]|\\.)*")+);', t8)
    one = b"".join(c_unescape(x) for x in re.findall(r'"((?:[^"\\]|\\.)*)"', m1.group(1)))
    two = b"".join(c_unescape(x) for x in re.findall(r'"((?:[^"\\]|\\.)*)"', m2.group(1)))
    assert one + two == sentence, (len(one), len(two), len(sentence))
    out["blob_chained"] = [
        {"blobs_hex": [[b"one".hex()], [b"two".hex(), b"three".hex()]], "crc": 0xA0EA6901},
        {"blobs_hex": [[one.hex()], [two.hex()]], "crc": 0xD86F726E},
        {"blobs_hex": [[]], "seed": 0xA0EA6901, "crc": 0xA0EA6901},
    ]

    # RFC 3720 B.4
    out["rfc3720"] = [
        {"hex": (b"\x00" * 32).hex(), "crc": 0x8A9136AA},
        {"hex": (b"\xff" * 32).hex(), "crc": 0x62A8AB43},
        {"hex": bytes(range(32)).hex(), "crc": 0x46DD794E},
        {"hex": bytes(range(31, -1, -1)).hex(), "crc": 0x113FDB5C},
    ]

    # on-disk DATA fixture
    detail = open(os.path.join(DATA_DIR, "detail_result.txt")).read()
    crcs = [int(x) for x in re.findall(r"Crc32c\s*:\s*(\d+)", detail)]
    assert crcs == [3381945770, 3381945770], crcs
    shutil.copyfile(os.path.join(DATA_DIR, "test.bmq_data"), os.path.join(HERE, "test.bmq_data"))
    shutil.copyfile(os.path.join(DATA_DIR, "test.bmq_journal"),
                    os.path.join(HERE, "test.bmq_journal"))
    # journal offsets of the two MESSAGE records as printed by bmqstoragetool
    blocks = detail.split("RecordType      : ")
    msg_offsets = [int(re.search(r"Offset\s*:\s*(\d+)", b).group(1)) for b in blocks
                   if b.startswith("MESSAGE")]
    assert msg_offsets == [224, 644], msg_offsets
    out["journal_file"] = {"file": "test.bmq_journal", "message_record_offsets": msg_offsets,
                           "crc": crcs}
    # Which MESSAGE records recovery keeps (FileStore::recoverMessages CRCs
    # exactly these): bmqstoragetool's summary counts 1 outstanding message
    # (summary_result.txt) and names it (test_journalfile.py
    # test_confirmed_outstanding_result: TEST_GUID_1 outstanding, TEST_GUID_2
    # confirmed and deleted); the summary also prints the journal bounds.
    summary = open(os.path.join(DATA_DIR, "summary_result.txt")).read()
    tests_py = open(os.path.join(DATA_DIR, "..", "test_journalfile.py")).read()
    guids = dict(re.findall(r'(TEST_GUID_\d)\s*=\s*b"([0-9A-F]{32})"', tests_py))
    outstanding = int(re.search(r"Number of outstanding messages:\s*(\d+)", summary).group(1))
    guid_at = {}
    for b in blocks:
        if b.startswith("MESSAGE"):
            guid_at[re.search(r"GUID\s*:\s*([0-9A-F]{32})", b).group(1)] = \
                int(re.search(r"Offset\s*:\s*(\d+)", b).group(1))
    out["recovery"] = {
        "outstanding_messages": outstanding,
        "outstanding_guids": [guids["TEST_GUID_1"]],
        "deleted_guids": [guids["TEST_GUID_2"]],
        "outstanding_record_offsets": [guid_at[guids["TEST_GUID_1"]]],
        "last_valid_record_offset": int(re.search(r"Last Valid Record Offset\s*:\s*(\d+)",
                                                  summary).group(1)),
        "last_valid_syncpoint_offset": int(re.search(r"Last Valid SyncPoint Offset\s*:\s*(\d+)",
                                                     summary).group(1)),
    }
    assert outstanding == 1 and out["recovery"]["outstanding_record_offsets"] == [644], out["recovery"]
    out["data_file"] = {
        "file": "test.bmq_data",
        "records": [{"record_offset": 40, "header_bytes": 12, "app_data_len": 11, "crc": crcs[0]},
                    {"record_offset": 64, "header_bytes": 12, "app_data_len": 11, "crc": crcs[1]}],
    }
    out["csl"] = csl_fixture()
    out["journal_queue_ops"] = queue_op_fixture()
    out["journal_ops"] = journal_op_fixture()
    out["queue_summary"] = queue_summary_fixture()
    assert out["csl"]["queue_key"] == out["journal_queue_ops"]["creation"]["queue_key"]
    with open(os.path.join(HERE, "crc32c_vectors.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote crc32c_vectors.json:", {k: len(v) if isinstance(v, list) else 1
                                         for k, v in out.items()})


CSL_TYPES = {"SNAPSHOT": 1, "UPDATE": 2, "COMMIT": 3, "ACK": 4}


def csl_fixture():
    """The ledger and bmqstoragetool's view of it (ClusterStateRecordType,
    mqbc_clusterstateledgerprotocol.h:154)."""
    shutil.copyfile(os.path.join(DATA_DIR, "test.bmq_csl"), os.path.join(HERE, "test.bmq_csl"))
    detail = open(os.path.join(DATA_DIR, "detail_csl_result.txt")).read()
    recs = []
    for blk in detail.split("RecordType           : ")[1:]:
        def field(name):
            return re.search(name + r"\s*:\s*(\S+)", blk).group(1)
        recs.append({"offset": int(field("Offset")), "type": CSL_TYPES[blk.split()[0]],
                     "log_id": field("LogId"), "elector_term": int(field("ElectorTerm")),
                     "sequence_number": int(field("SequenceNumber")),
                     "header_words": int(field("HeaderWords")),
                     "advisory_words": int(field("LeaderAdvisoryWords")),
                     "epoch": int(field("Epoch"))})
    assert [(r["offset"], r["type"]) for r in recs] == [(388, 1), (540, 3)], recs
    short = open(os.path.join(DATA_DIR, "short_csl_result.txt")).read()
    short_offs = [int(x) for x in re.findall(r"offset = (\d+)", short)]
    assert short_offs == [r["offset"] for r in recs], short_offs
    assert set(re.findall(r"logId = (\w+)", short)) == {recs[0]["log_id"]}
    summary = open(os.path.join(DATA_DIR, "summary_csl_result.txt")).read()
    keys = re.findall(r"key = \[ (\w+) \]", summary)
    assert len(keys) == 1, keys
    tests_py = open(os.path.join(DATA_DIR, "..", "test_cslfile.py")).read()

    def const(name):
        return re.search(name + r'\s*=\s*"?([^"\n]+)"?', tests_py).group(1)
    seq1 = [int(x) for x in const("TEST_SEARCH_SEQNUM_1").split("-")]
    # test_search_offset: --offset=316 finds 1 commit record, --offset=317 none;
    # test_search_seqnum: --seqnum=1-4 finds 1 commit record;
    # test_short_result --csl-from-begin: "2 snapshot record";
    # test_search_range: offsets in (88, 388) hold 1 update and 1 commit, no snapshot
    assert 'b"1 commit record"' in tests_py and 'b"2 snapshot record"' in tests_py
    return {
        "file": "test.bmq_csl", "log_id": recs[0]["log_id"], "records": recs,
        "queue_key": keys[0],
        "search": {
            "commit_at": {"offset": int(const("TEST_SEARCH_OFFSET_1")),
                          "elector_term": seq1[0], "sequence_number": seq1[1]},
            "not_a_record": int(const("TEST_SEARCH_OFFSET_2")),
            "snapshots_from_begin": 2,
            "between": {"gt": int(const("TEST_OFFSET_LOWER")),
                        "lt": int(const("TEST_OFFSET_UPPER")),
                        "counts": {"1": 0, "2": 1, "3": 1, "4": 0}},
        },
    }


def queue_op_fixture():
    """The journal's QueueOp and JournalOp records as bmqstoragetool lists them."""
    qop = open(os.path.join(DATA_DIR, "queueop_result.txt")).read()

    def field(name):
        return re.search(name + r"\s*:\s*(\S+)", qop).group(1)
    summ = open(os.path.join(DATA_DIR, "summary_queueop_journalop_result.txt")).read()

    def count(label):
        return int(re.search(label + r"\s*:?\s*(\d+)", summ).group(1))
    out = {
        "creation": {"offset": int(field("Offset")), "queue_key": field("QueueKey"),
                     "app_key": field("AppKey"), "op": field("QueueOpType"),
                     "primary_lease_id": int(field("PrimaryLeaseId")),
                     "sequence_number": int(field("SequenceNumber")),
                     "qlist_offset_words": int(field("QLIST OffsetWords"))},
        "queue_op_records": count("Total number of queueOp records"),
        "creation_ops": count("Number of 'creation' operations"),
        "journal_op_records": count("Number of journalOp records"),
    }
    assert out["creation"]["offset"] == 104 and out["creation"]["op"] == "CREATION", out
    return out


SYNC_POINT_TYPES = {"REGULAR": 1, "ROLLOVER": 2}  # SyncPointType (mqbs_filestoreprotocol.h:1901)


def journal_op_fixture():
    """journalop_result.txt: the JOURNAL_OP records bmqstoragetool lists."""
    txt = open(os.path.join(DATA_DIR, "journalop_result.txt")).read()
    recs = []
    for blk in txt.split("RecordType      : ")[1:]:
        def field(name):
            return re.search(r"\b" + name + r"\s*:\s*(\S+)", blk).group(1)
        assert blk.startswith("JOURNAL_OP") and field("JournalOpType") == "SYNCPOINT", blk
        recs.append({"index": int(field("Index")), "offset": int(field("Offset")),
                     "primary_lease_id": int(field("PrimaryLeaseId")),
                     "sequence_number": int(field("SequenceNumber")),
                     "epoch": int(field("Epoch")),
                     "sync_point_type": SYNC_POINT_TYPES[field("SyncPointType")],
                     "sync_pt_primary_lease_id": int(field("SyncPtPrimaryLeaseId")),
                     "sync_pt_sequence_number": int(field("SyncPtSequenceNumber")),
                     "primary_node_id": int(field("PrimaryNodeId")),
                     "data_file_offset_dwords": int(field("DataFileOffsetDwords"))})
    n = int(re.search(r"(\d+) journalOp record\(s\) found", txt).group(1))
    assert n == len(recs) == 8 and recs[0]["offset"] == 44 and recs[-1]["offset"] == 764, recs
    return {"records": recs, "count": n}


def queue_summary_fixture():
    """summary_result_with_queue_info.txt: message and per-queue record counts
    and the journal's last sync point."""
    txt = open(os.path.join(DATA_DIR, "summary_result_with_queue_info.txt")).read()

    def num(label):
        return int(re.search(label + r"\s*:\s*(\d+)", txt).group(1))
    q = txt[txt.index("Number of records per Queue:"):txt.index("Details of journal file:")]
    queues = []
    for blk in q.split("Queue Key             : ")[1:]:
        def qf(label):
            return int(re.search(label + r"\s*:\s*(\d+)", blk).group(1))
        queues.append({"queue_key": blk.split()[0],
                       "uri": re.search(r"Queue URI\s*:\s*(\S+)", blk).group(1),
                       "total_records": qf("Total Records"),
                       "queue_op_records": qf("Num Queue Op Records"),
                       "message_records": qf("Num Message Records"),
                       "confirm_records": qf("Num Confirm Records"),
                       "delete_records": qf("Num Delete Records")})
    sp = txt[txt.index("Journal SyncPoint"):]
    out = {
        "total_messages": num("Total number of messages"),
        "partially_confirmed": num("Number of partially confirmed messages"),
        "confirmed": num("Number of confirmed messages"),
        "outstanding": num("Number of outstanding messages"),
        "total_records": num("Total number of records"),
        "queues": queues,
        "last_sync_point": {
            "last_valid_record_offset": int(re.search(r"Last Valid Record Offset\s*:\s*(\d+)",
                                                      sp).group(1)),
            "offset": int(re.search(r"Last Valid SyncPoint Offset\s*:\s*(\d+)", sp).group(1)),
            "epoch": int(re.search(r"SyncPoint Epoch\s*:\s*(\d+)", sp).group(1)),
            "sequence_number": int(re.search(r"SyncPoint SeqNum\s*:\s*(\d+)", sp).group(1)),
            "primary_node_id": int(re.search(r"SyncPoint Primary NodeId\s*:\s*(\d+)",
                                             sp).group(1)),
            "primary_lease_id": int(re.search(r"SyncPoint Primary LeaseId\s*:\s*(\d+)",
                                              sp).group(1)),
            "data_file_offset_dwords": int(re.search(
                r"SyncPoint DataFileOffset \(DWORDS\)\s*:\s*(\d+)", sp).group(1)),
            "qlist_file_offset_words": int(re.search(
                r"SyncPoint QlistFileOffset \(WORDS\)\s*:\s*(\d+)", sp).group(1)),
        },
    }
    assert len(queues) == 1 and queues[0]["total_records"] == 4, queues
    return out


if __name__ == "__main__":
    sys.exit(main())
