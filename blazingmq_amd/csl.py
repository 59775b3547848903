"""Cluster state ledger (CSL) record CRCs.

Host-side mirror of the CRC parts of ``mqbc::ClusterStateLedgerUtil``
(/root/reference/src/groups/mqb/mqbc/mqbc_clusterstateledgerutil.cpp):

* ``append_record`` -- ``appendRecord`` (:360-417): ClusterStateRecordHeader,
  the (opaque here) BER-encoded advisory, word padding, then the big-endian
  CRC32C of everything before it.  One record at a time on the cluster
  thread, so it uses the scalar ``Crc32c.calculate`` like the reference.
* ``validate_log`` -- ``validateLog`` (:248-336): walks every record of a log
  and checks its CRC.  The walk is native (``bmqcrc_csl_validate``,
  include/bmqcrc_protocol.h) and every record CRC is checked in ONE batched
  GPU call; the result code is the reference's (``ClusterStateLedgerUtilRc``).

Layouts (mqbc_clusterstateledgerprotocol.h): ClusterStateFileHeader (:76,
8 bytes) u8 PV(2)|HeaderWords(6), FileKey[5], reserved[2];
ClusterStateRecordHeader (:272, 32 bytes) u8 HW(4)|RecordType(4), reserved[3],
BE u32 reserved(4)|LeaderAdvisoryWords(28), BE elector term hi/lo, sequence
number hi/lo, timestamp hi/lo.
"""
import ctypes

import numpy as np

from . import _native as N
from .crc32c import Crc32c

# mqbc::ClusterStateLedgerUtilRc (mqbc_clusterstateledgerutil.h:65-124)
SUCCESS = 0
INVALID_PROTOCOL_VERSION = -5
INVALID_LOG_ID = -6
INVALID_HEADER_WORDS = -7
INVALID_CHECKSUM = -10
RECORD_ALIAS_FAILURE = -13
# mqbsi::LogOpResult::e_REACHED_END_OF_LOG (mqbsi_log.h:138), returned raw by
# validateLog when a record runs past the end of the log (:293-298)
REACHED_END_OF_LOG = -15

# ClusterStateRecordType (mqbc_clusterstateledgerprotocol.h:154)
SNAPSHOT, UPDATE, COMMIT, ACK = 1, 2, 3, 4

PROTOCOL_VERSION = 1
FILE_HEADER_SIZE = 8
RECORD_HEADER_SIZE = 32
WORD = 4


def file_header(log_id):
    """ClusterStateFileHeader for the 5-byte file key `log_id`
    (ClusterStateLedgerUtil::writeFileHeader, :338-358)."""
    log_id = bytes(log_id)
    if len(log_id) != 5:
        raise ValueError("log id is 5 bytes")
    return bytes([(PROTOCOL_VERSION << 6) | (FILE_HEADER_SIZE // WORD)]) + log_id + bytes(2)


def record_header(record_type, advisory_words, elector_term=0, sequence_number=0, timestamp=0):
    h = bytearray(RECORD_HEADER_SIZE)
    h[0] = ((RECORD_HEADER_SIZE // WORD) << 4) | (record_type & 0xF)
    h[4:8] = (advisory_words & 0x0FFFFFFF).to_bytes(4, "big")
    h[8:16] = int(elector_term).to_bytes(8, "big")
    h[16:24] = int(sequence_number).to_bytes(8, "big")
    h[24:32] = int(timestamp).to_bytes(8, "big")
    return h


def append_record(advisory, record_type=UPDATE, elector_term=0, sequence_number=0,
                  timestamp=0, crc=None):
    """One ledger record: header + `advisory` bytes + word padding + CRC.
    `crc` overrides the computed CRC (corruption tests)."""
    advisory = bytes(advisory)
    length = RECORD_HEADER_SIZE + len(advisory)
    num_words = (length + WORD) // WORD          # calcNumWordsAndPadding
    pad = num_words * WORD - length              # 1..4 bytes, each = pad
    law = num_words + 1 - RECORD_HEADER_SIZE // WORD
    body = bytes(record_header(record_type, law, elector_term, sequence_number, timestamp)) + \
        advisory + bytes([pad]) * pad
    value = Crc32c.calculate(body) if crc is None else int(crc)
    return body + value.to_bytes(4, "big")


def validate_log(log, expected_log_id=None, device=-1, devices=None):
    """``ClusterStateLedgerUtil::validateLog`` over a whole log buffer.

    Returns (rc, offset, bad_record_offset): rc is the reference's result
    code; offset is the end of the valid records when rc == 0; for
    INVALID_CHECKSUM bad_record_offset is the first corrupt record."""
    a = np.ascontiguousarray(np.frombuffer(bytes(log), np.uint8) if not isinstance(
        log, np.ndarray) else log.view(np.uint8).reshape(-1))
    key = None
    if expected_log_id is not None:
        key = ctypes.create_string_buffer(bytes(expected_log_id), 5)
    rc, off, bad = ctypes.c_int(0), ctypes.c_uint64(0), ctypes.c_uint64(0)
    opts = N.make_opts(device=device, devices=devices)
    N.check(N.lib.bmqcrc_csl_validate(
        ctypes.c_void_p(a.ctypes.data) if a.size else None, a.size, key, ctypes.byref(rc),
        ctypes.byref(off), ctypes.byref(bad), ctypes.byref(opts)))
    return rc.value, int(off.value), (int(bad.value) if rc.value == INVALID_CHECKSUM else None)


def scan_log(log, expected_log_id=None):
    """Native walk without the CRC check (``bmqcrc_csl_scan``, CPU only).
    Returns (walk_rc, end_offset, record_offsets, crc'd lengths, stored CRCs)."""
    a = np.ascontiguousarray(np.frombuffer(bytes(log), np.uint8) if not isinstance(
        log, np.ndarray) else log.view(np.uint8).reshape(-1))
    p = ctypes.c_void_p(a.ctypes.data) if a.size else None
    key = ctypes.create_string_buffer(bytes(expected_log_id), 5) if expected_log_id else None
    wrc, end = ctypes.c_int(0), ctypes.c_uint64(0)
    n = N.check_count(N.lib.bmqcrc_csl_scan(p, a.size, key, None, None, None, 0,
                                            ctypes.byref(wrc), ctypes.byref(end)))
    off, ln, crc = np.zeros(n, np.uint64), np.zeros(n, np.uint32), np.zeros(n, np.uint32)
    if n:
        N.check_count(N.lib.bmqcrc_csl_scan(
            p, a.size, key, ctypes.c_void_p(off.ctypes.data), ctypes.c_void_p(ln.ctypes.data),
            ctypes.c_void_p(crc.ctypes.data), n, ctypes.byref(wrc), ctypes.byref(end)))
    return wrc.value, int(end.value), off, ln, crc
