"""Batched recovery-time CRC32C verification over BlazingMQ partition files.

Host-side mirror of the CRC part of ``mqbs::FileStore::recoverMessages``
(/root/reference/src/groups/mqb/mqbs/mqbs_filestore.cpp:1045, record walk
:1490, DATA checks :2495-2575, CRC check :2603-2624).  The reference walks the
journal and CRCs one message at a time; here every MESSAGE record is
collected first, then all payloads are verified with ONE batched GPU call.

The product path is native: ``scan_partition`` / ``verify_partition`` call
``bmqcrc_journal_scan`` / ``bmqcrc_recover_verify`` (include/bmqcrc_protocol.h,
csrc/bmqcrc_protocol.cpp).  ``journal_message_records`` / ``data_app_ranges``
restate the same walk in numpy; the CPU tests hold the two against each other
and against the bmqstoragetool fixture.

On-disk layouts (mqbs_filestoreprotocol.h):
  FileHeader (:306)        magic1 "!bmq", magic2 "BMQ!", PV(2b)|HW(6b), B(1b)|FileType(7b),
                           ..., partitionId (BE, byte 20)
  JournalFileHeader (:483) headerWords, recordWords (15 = 60-byte records), ...
  DataFileHeader (:426)    headerWords, reserved, fileKey[5], reserved
  RecordHeader (:1014)     BE u16 type(4b)|flags(12b), seqNum hi/lo, leaseId, timestamp
  MessageRecord (:1125)    header(20) refCountHi(1) CAT(1) queueKey(5) fileKey(5)
                           messageOffsetDwords(BE u32 @32) GUID(16 @36) CRC32C(BE @52)
                           magic 0x2A724563 "*rEc" (@56)
  DataHeader (:703)        BE u32 HW(3b)|messageWords(29b), BE u32 optionsWords(24b)|flags(8b)
  A DATA record is DataHeader + options + application data + 1..8 padding
  bytes, each equal to the padding count (bmqp_protocolutil.cpp:44, dword
  padding); MessageOffsetDwords counts 8-byte units.
"""
import ctypes

import numpy as np

from . import _native as N
from .crc32c import Crc32c

MAGIC1 = 0x21626D71  # !bmq
MAGIC2 = 0x424D5121  # BMQ!
RECORD_MAGIC = 0x2A724563  # *rEc
JOURNAL_RECORD_SIZE = 60
FILE_TYPE_DATA, FILE_TYPE_JOURNAL, FILE_TYPE_QLIST = 1, 2, 3
REC_MESSAGE, REC_CONFIRM, REC_DELETION, REC_QUEUE_OP, REC_JOURNAL_OP = 1, 2, 3, 4, 5
WORD, DWORD = 4, 8


class StorageFormatError(ValueError):
    """Invalid journal/DATA content (the reference returns rc_INVALID_* codes)."""


def _be32(a, off):
    return (a[off].astype(np.uint32) << 24) | (a[off + 1].astype(np.uint32) << 16) | \
           (a[off + 2].astype(np.uint32) << 8) | a[off + 3].astype(np.uint32)


def _as_u8(buf):
    if isinstance(buf, np.ndarray):
        return buf.view(np.uint8).reshape(-1)
    return np.frombuffer(bytes(buf), dtype=np.uint8)


def parse_file_header(buf, expect_type):
    """Return the byte size of the BlazingMQ FileHeader (FileHeader::headerWords)."""
    a = _as_u8(buf)
    if a.size < 32 or int(_be32(a, 0)) != MAGIC1 or int(_be32(a, 4)) != MAGIC2:
        raise StorageFormatError("bad BlazingMQ file magic")
    hw = int(a[8]) & 0x3F
    ftype = int(a[9]) & 0x7F
    if ftype != expect_type:
        raise StorageFormatError("file type %d, expected %d" % (ftype, expect_type))
    return hw * WORD


def journal_message_records(journal):
    """All MESSAGE records of a journal: dict of numpy arrays
    (record_offset, data_offset, crc32c, guid)."""
    a = _as_u8(journal)
    fh = parse_file_header(a, FILE_TYPE_JOURNAL)
    jh_words = int(a[fh])
    rec_words = int(a[fh + 1])
    if rec_words * WORD != JOURNAL_RECORD_SIZE:
        raise StorageFormatError("journal recordWords %d != 15" % rec_words)
    start = fh + jh_words * WORD
    nrec = (a.size - start) // JOURNAL_RECORD_SIZE
    recs = a[start:start + nrec * JOURNAL_RECORD_SIZE].reshape(nrec, JOURNAL_RECORD_SIZE)
    magic = _be32(recs.T, 56)
    valid = magic == RECORD_MAGIC
    # a pre-allocated journal is zero past the last record: stop at the first hole
    if not valid.all():
        first_bad = int(np.argmin(valid))
        if recs[first_bad:].any():
            raise StorageFormatError("journal record %d has a bad magic" % first_bad)
        recs = recs[:first_bad]
        nrec = first_bad
    rtype = recs[:, 0] >> 4
    msg = np.nonzero(rtype == REC_MESSAGE)[0]
    m = recs[msg]
    return {
        "record_offset": (start + msg * JOURNAL_RECORD_SIZE).astype(np.uint64),
        "data_offset": _be32(m.T, 32).astype(np.uint64) * DWORD,
        "crc32c": _be32(m.T, 52).astype(np.uint32),
        "guid": m[:, 36:52].copy(),
    }


def data_app_ranges(data, data_offsets):
    """Application-data (offset, length) of DATA records, validated like
    mqbs_filestore.cpp:2495-2575 (header/options/total sizes, padding 1..8)."""
    a = _as_u8(data)
    off = np.asarray(data_offsets, dtype=np.uint64)
    if off.size == 0:
        return off, np.zeros(0, np.uint32)
    if int(off.max()) + 8 > a.size:
        raise StorageFormatError("DATA record offset beyond the DATA file")
    o = off.astype(np.int64)
    w0 = _be32(a, o)
    w1 = _be32(a, o + 4)
    header_size = (w0 >> 29).astype(np.int64) * WORD
    total_len = (w0 & 0x1FFFFFFF).astype(np.int64) * WORD
    options_size = (w1 >> 8).astype(np.int64) * WORD
    if (header_size == 0).any() or (total_len == 0).any():
        raise StorageFormatError("DATA record with zero headerWords/messageWords")
    if ((header_size + options_size) >= total_len).any():
        raise StorageFormatError("DATA record header/options exceed messageWords")
    if int((o + total_len).max()) > a.size:
        raise StorageFormatError("DATA record extends beyond the DATA file")
    last_byte = a[o + total_len - 1].astype(np.int64)
    if ((last_byte < 1) | (last_byte > DWORD)).any():
        raise StorageFormatError("DATA record with invalid padding")
    if (total_len < header_size + options_size + last_byte).any():
        raise StorageFormatError("DATA record sizes inconsistent with padding")
    app_off = (o + header_size + options_size).astype(np.uint64)
    app_len = (total_len - header_size - options_size - last_byte).astype(np.uint32)
    return app_off, app_len


def _native_call(fn, *args):
    try:
        return fn(*args)
    except N.BmqCrcError as e:
        if e.rc == N.BMQCRC_EINVAL:
            raise StorageFormatError(str(e)) from e
        raise


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a.size else None


def scan_partition(journal, data):
    """Native walk (``bmqcrc_journal_scan``, CPU only): every MESSAGE record
    as numpy arrays (record_offset, app_offset, app_length, crc32c)."""
    j, d = np.ascontiguousarray(_as_u8(journal)), np.ascontiguousarray(_as_u8(data))

    def scan(cap, *arrs):
        n = N.lib.bmqcrc_journal_scan(_ptr(j), j.size, _ptr(d), d.size,
                                      *[_ptr(a) if a is not None else None for a in arrs], cap)
        return N.check_count(n)

    n = _native_call(scan, 0, None, None, None, None)
    out = {"record_offset": np.zeros(n, np.uint64), "app_offset": np.zeros(n, np.uint64),
           "app_length": np.zeros(n, np.uint32), "crc32c": np.zeros(n, np.uint32)}
    _native_call(scan, n, out["record_offset"], out["app_offset"], out["app_length"],
                 out["crc32c"])
    return out


def verify_partition(journal, data, bad_cap=1 << 20, device=-1):
    """Recovery CRC check of a whole partition: one native walk, one batched
    GPU verify (``bmqcrc_recover_verify``).

    Returns dict(n_messages, n_bad, bad_record_offsets).  A mismatch is what
    the reference reports with BMQTSK_ALARMLOG_ALARM("RECOVERY")
    (mqbs_filestore.cpp:2613-2624); like the reference, recovery continues.
    """
    j, d = np.ascontiguousarray(_as_u8(journal)), np.ascontiguousarray(_as_u8(data))
    n_msgs, n_bad = ctypes.c_uint64(0), ctypes.c_uint64(0)
    bad = np.zeros(max(int(bad_cap), 1), np.uint64)
    opts = N.make_opts(device=device)

    def run():
        return N.check(N.lib.bmqcrc_recover_verify(
            _ptr(j), j.size, _ptr(d), d.size, ctypes.byref(n_msgs), ctypes.byref(n_bad),
            _ptr(bad), int(bad_cap), ctypes.byref(opts)))

    _native_call(run)
    k = min(int(n_bad.value), int(bad_cap))
    return {"n_messages": int(n_msgs.value), "n_bad": int(n_bad.value),
            "bad_record_offsets": bad[:k].copy()}


# ----------------------------------------------------------------------------
# Writer (tests and synthetic partitions): the layout FileStore produces.
# ----------------------------------------------------------------------------
def file_header(file_type, partition_id=0):
    h = np.zeros(32, np.uint8)
    h[0:4] = np.frombuffer(MAGIC1.to_bytes(4, "big"), np.uint8)
    h[4:8] = np.frombuffer(MAGIC2.to_bytes(4, "big"), np.uint8)
    h[8] = (1 << 6) | 8          # protocol version 1, 8 header words
    h[9] = 0x80 | file_type      # bitness 64, file type
    h[20:24] = np.frombuffer(int(partition_id).to_bytes(4, "big"), np.uint8)
    return h


def write_partition(app_datas, crcs=None, seq_start=1, lease_id=1, timestamp=0x6720EAB4,
                    queue_key=b"\x26\xda\xcd\xc9\x74"):
    """Build (journal, data) byte arrays holding one MESSAGE record per entry
    of `app_datas` (bytes).  `crcs` (optional) overrides the CRC stored in the
    journal (default: the true CRC32C of the app data)."""
    data = [file_header(FILE_TYPE_DATA).tobytes(), bytes([2, 0, 0, 0, 0, 0, 0, 0])]
    pos = 40
    recs = []
    for i, app in enumerate(app_datas):
        app = bytes(app)
        pad = DWORD - ((12 + len(app)) % DWORD) if (12 + len(app)) % DWORD else DWORD
        total = 12 + len(app) + pad
        hdr = ((3 << 29) | (total // WORD)).to_bytes(4, "big") + bytes(8)
        data.append(hdr + app + bytes([pad]) * pad)
        crc = Crc32c.calculate(app) if crcs is None else int(crcs[i])
        r = bytearray(JOURNAL_RECORD_SIZE)
        seq = seq_start + i
        r[0:2] = ((REC_MESSAGE << 12) | 1).to_bytes(2, "big")  # type, refcount low bits = 1
        r[2:4] = (seq >> 32).to_bytes(2, "big")
        r[4:8] = (seq & 0xFFFFFFFF).to_bytes(4, "big")
        r[8:12] = lease_id.to_bytes(4, "big")
        r[12:20] = timestamp.to_bytes(8, "big")
        r[22:27] = queue_key
        r[32:36] = (pos // DWORD).to_bytes(4, "big")
        r[36:52] = (0x40000000000000000000000000000000 | (seq + 1)).to_bytes(16, "big")
        r[52:56] = crc.to_bytes(4, "big")
        r[56:60] = RECORD_MAGIC.to_bytes(4, "big")
        recs.append(bytes(r))
        pos += total
    journal = file_header(FILE_TYPE_JOURNAL).tobytes() + bytes([3, 15]) + bytes(10) + b"".join(recs)
    return np.frombuffer(journal, np.uint8).copy(), np.frombuffer(b"".join(data), np.uint8).copy()
