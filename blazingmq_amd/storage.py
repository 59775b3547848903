"""Batched recovery-time CRC32C verification over BlazingMQ partition files.

Host-side mirror of the CRC part of ``mqbs::FileStore::recoverMessages``
(/root/reference/src/groups/mqb/mqbs/mqbs_filestore.cpp:1045, two backward
passes :1120-1453 and :1490-2646, DATA checks :2494-2575, CRC check
:2603-2624).  The reference CRCs the outstanding messages one at a time as it
walks; here the same records are selected first (deleted GUIDs, purged
queues and records before their queue's DELETION are skipped, their DATA
never read), then all payloads are verified with ONE batched GPU call.

The product path is native: ``scan_partition`` / ``verify_partition`` call
``bmqcrc_journal_scan`` / ``bmqcrc_recover_verify`` (include/bmqcrc_protocol.h,
csrc/bmqcrc_protocol.cpp).  ``recovery_selection_py`` restates the selection
in Python; the CPU tests hold the two against each other, against
bmqstoragetool's fixture and its outstanding-message outputs, and against
partitions built by ``PartitionWriter`` with every record type.

On-disk layouts (mqbs_filestoreprotocol.h):
  FileHeader (:306)        magic1 "!bmq", magic2 "BMQ!", PV(2b)|HW(6b), B(1b)|FileType(7b),
                           ..., partitionId (BE, byte 20)
  JournalFileHeader (:483) headerWords, recordWords (15 = 60-byte records), ...
  DataFileHeader (:426)    headerWords, reserved, fileKey[5], reserved
  RecordHeader (:1014)     BE u16 type(4b)|flags(12b), seqNum hi/lo, leaseId, timestamp
  MessageRecord (:1125)    header(20) refCountHi(1) CAT(1) queueKey(5) fileKey(5)
                           messageOffsetDwords(BE u32 @32) GUID(16 @36) CRC32C(BE @52)
                           magic 0x2A724563 "*rEc" (@56)
  ConfirmRecord (:1339)    queueKey @22, appKey @27, GUID @32
  DeletionRecord (:1518)   queueKey @23, GUID @28
  QueueOpRecord (:1694)    queueKey @22, appKey @27, BE i32 QueueOpType @32, uri offset @36
  JournalOpRecord (:1953)  syncPointType @23, BE i32 JournalOpType @24, seq @28/@32,
                           leaseId @40, dataFileOffsetDwords @44, qlistFileOffsetWords @48
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


# FileStore::recoverMessages result codes (mqbs_filestore.cpp:1073-1091)
RC_SUCCESS = 0
RC_INVALID_PRIMARY_LEASE_ID = -2
RC_INVALID_SEQ_NUMBER = -3
RC_INVALID_QUEUE_OP_RECORD = -4
RC_NULL_QUEUE_KEY = -5
RC_DUPLICATE_QUEUE_KEY = -7
RC_INVALID_QUEUE_KEY = -8
RC_INVALID_DATA_OFFSET = -11
RC_INVALID_SYNC_PT_SUB_TYPE = -12
RC_INVALID_DELETION_RECORD = -14
RC_INVALID_CONFIRM_RECORD = -15
RC_INVALID_MESSAGE_RECORD = -16
RC_INVALID_DATA_RECORD = -17

# QueueOpType (mqbs_filestoreprotocol.h:1630), JournalOpType (:1841)
OP_PURGE, OP_CREATION, OP_DELETION, OP_ADDITION = 1, 2, 3, 4
JOURNAL_OP_SYNCPOINT = 2
NULL_KEY = bytes(5)


class RecoveryConfig(ctypes.Structure):
    """include/bmqcrc_protocol.h bmqcrc_recovery_cfg: the queues recovery
    knows.  with_csl=False: the journal's own QueueOp CREATION records;
    with_csl=True: the cluster state's queue keys (5 bytes each)."""
    _fields_ = [("struct_size", ctypes.c_uint32), ("with_csl", ctypes.c_int32),
                ("queue_keys", ctypes.c_void_p), ("n_queue_keys", ctypes.c_uint64)]


def _cfg(with_csl, queue_keys):
    if not with_csl:
        return None, None
    keys = np.frombuffer(b"".join(bytes(k) for k in queue_keys), np.uint8).copy()
    if keys.size != 5 * len(queue_keys):
        raise ValueError("queue keys are 5 bytes each")
    c = RecoveryConfig(ctypes.sizeof(RecoveryConfig), 1,
                       keys.ctypes.data if keys.size else None, len(queue_keys))
    return c, keys  # keep the key buffer alive with the struct


def _int(b, off, n):
    return int.from_bytes(bytes(b[off:off + n]), "big")


def journal_bounds_py(journal):
    """FileStoreProtocolUtil::lastJournalSyncPoint / lastJournalRecord
    (mqbs_filestoreprotocolutil.cpp:165-289), restated: (last sync point
    offset, last record offset), 0 meaning none."""
    a = _as_u8(journal)
    fh = parse_file_header(a, FILE_TYPE_JOURNAL)
    start = fh + int(a[fh]) * WORD
    n = (a.size - start) // JOURNAL_RECORD_SIZE if a.size > start else 0
    lsp = 0
    for i in range(n - 1, -1, -1):
        r = a[start + i * JOURNAL_RECORD_SIZE:start + (i + 1) * JOURNAL_RECORD_SIZE]
        seq = (_int(r, 2, 2) << 32) | _int(r, 4, 4)
        if (r[0] >> 4) == REC_JOURNAL_OP and _int(r, 24, 4) == JOURNAL_OP_SYNCPOINT and \
                _int(r, 8, 4) and seq and _int(r, 56, 4) == RECORD_MAGIC:
            lsp = start + i * JOURNAL_RECORD_SIZE
            break
    if a.size <= start:
        return 0, 0
    cur, prev = (lsp + JOURNAL_RECORD_SIZE, lsp) if lsp else (start, 0)
    while cur + JOURNAL_RECORD_SIZE <= a.size:
        if (a[cur] >> 4) == 0 or _int(a, cur + 56, 4) != RECORD_MAGIC:
            break
        prev, cur = cur, cur + JOURNAL_RECORD_SIZE
    return lsp, prev


def recovery_selection_py(journal, data, with_csl=False, queue_keys=()):
    """Pure-Python restatement of the MESSAGE records mqbs::FileStore::
    recoverMessages CRCs (mqbs_filestore.cpp:1045-2646), used by the tests to
    hold the native walk (``scan_partition``) to the reference's decisions.

    Two backward passes from the journal's last record, each stopping at the
    first record with an undefined type, a zero lease id / sequence number or
    a bad magic.  First pass (:1120-1453): queue DELETION offsets, queues
    alive (CREATION records, or the cluster state with CSL), the first sync
    point.  Second pass (:1490-2646): PSN checks against the write head (the
    last record), sync point checks, whole-queue PURGEs, DELETION GUIDs, and
    every MESSAGE that survives them -- DATA record checks, then its CRC.
    Returns dict(recovery_rc, error_record_offset, record_offset, app_offset,
    app_length, crc32c) in the backward order."""
    j, d = _as_u8(journal), _as_u8(data)
    fh = parse_file_header(j, FILE_TYPE_JOURNAL)
    parse_file_header(d, FILE_TYPE_DATA)
    start = fh + int(j[fh]) * WORD
    out = {"recovery_rc": 0, "error_record_offset": 0, "record_offset": [], "app_offset": [],
           "app_length": [], "crc32c": []}
    _, last = journal_bounds_py(j)
    if last == 0:
        return out

    def hdr(pos):
        r = j[pos:pos + JOURNAL_RECORD_SIZE]
        return int(r[0]) >> 4, (_int(r, 2, 2) << 32) | _int(r, 4, 4), _int(r, 8, 4), r

    positions = []
    for pos in range(last, start - 1, -JOURNAL_RECORD_SIZE):
        t, seq, lease, r = hdr(pos)
        if t == 0 or seq == 0 or lease == 0 or _int(r, 56, 4) != RECORD_MAGIC:
            break
        positions.append(pos)

    def fail(rc, pos):
        out["recovery_rc"], out["error_record_offset"] = rc, pos
        return out

    live = set(bytes(k) for k in queue_keys) if with_csl else set()
    deleted_queue, deleted_app, first_sync = {}, {}, 0
    for pos in positions:
        t, _, _, r = hdr(pos)
        if t == REC_JOURNAL_OP:
            first_sync = pos
            continue
        if t != REC_QUEUE_OP:
            continue
        op, qkey, akey = _int(r, 32, 4), bytes(r[22:27]), bytes(r[27:32])
        if op == 0:
            return fail(RC_INVALID_QUEUE_OP_RECORD, pos)
        if qkey == NULL_KEY:
            return fail(RC_NULL_QUEUE_KEY, pos)
        if op == OP_DELETION:
            if with_csl and akey == NULL_KEY and qkey in live:
                return fail(RC_INVALID_DELETION_RECORD, pos)
            if akey == NULL_KEY:
                deleted_queue.setdefault(qkey, pos)
            else:
                deleted_app.setdefault(akey, pos)
        elif op in (OP_CREATION, OP_ADDITION):
            if qkey in deleted_queue:
                continue
            if with_csl:
                if qkey not in live:
                    return fail(RC_INVALID_QUEUE_KEY, pos)
            elif qkey in live:
                return fail(RC_DUPLICATE_QUEUE_KEY, pos)
            elif op == OP_CREATION:
                live.add(qkey)

    deleted_guids, purged = set(), set()
    lease, seq = hdr(last)[2], hdr(last)[1] + 1

    def before_deletion(qkey, pos):
        return qkey in deleted_queue and pos < deleted_queue[qkey]

    for pos in positions:
        t, s, ls, r = hdr(pos)
        if ls > lease:
            return fail(RC_INVALID_PRIMARY_LEASE_ID, pos)
        if ls == lease and (s != seq - 1 if pos >= first_sync else s > seq - 1):
            return fail(RC_INVALID_SEQ_NUMBER, pos)
        lease, seq = ls, s
        if t == REC_JOURNAL_OP:
            sp_seq, sp_lease, doff = (_int(r, 28, 4) << 32) | _int(r, 32, 4), _int(r, 40, 4), \
                _int(r, 44, 4) * DWORD
            if r[23] == 0:
                return fail(RC_INVALID_SYNC_PT_SUB_TYPE, pos)
            if doff == 0 or d.size < doff:
                return fail(RC_INVALID_DATA_OFFSET, pos)
            # the reference's order (:1647-1713): lease 0, seq 0, lease ahead, seq mismatch
            if sp_lease == 0:
                return fail(RC_INVALID_PRIMARY_LEASE_ID, pos)
            if sp_seq == 0:
                return fail(RC_INVALID_SEQ_NUMBER, pos)
            if sp_lease > lease:
                return fail(RC_INVALID_PRIMARY_LEASE_ID, pos)
            if sp_lease == lease and sp_seq != seq:
                return fail(RC_INVALID_SEQ_NUMBER, pos)
        elif t == REC_QUEUE_OP:
            qkey, akey, op = bytes(r[22:27]), bytes(r[27:32]), _int(r, 32, 4)
            if before_deletion(qkey, pos):
                continue
            if op == OP_ADDITION and not with_csl and qkey not in live:
                # an ADDITION whose CREATION the first pass did not see (:2018-2030)
                return fail(RC_INVALID_QUEUE_KEY, pos)
            if op == OP_PURGE and qkey in live and akey == NULL_KEY:
                purged.add(qkey)
        elif t == REC_DELETION:
            qkey, guid = bytes(r[23:28]), bytes(r[28:44])
            if guid == bytes(16) or qkey == NULL_KEY:
                return fail(RC_INVALID_DELETION_RECORD, pos)
            if not before_deletion(qkey, pos) and qkey not in purged:
                deleted_guids.add(guid)
        elif t == REC_CONFIRM:
            if bytes(r[32:48]) == bytes(16) or bytes(r[22:27]) == NULL_KEY:
                return fail(RC_INVALID_CONFIRM_RECORD, pos)
        elif t == REC_MESSAGE:
            qkey, guid = bytes(r[22:27]), bytes(r[36:52])
            if guid == bytes(16) or qkey == NULL_KEY:
                return fail(RC_INVALID_MESSAGE_RECORD, pos)
            o = _int(r, 32, 4) * DWORD
            if o == 0 or o > d.size:
                return fail(RC_INVALID_DATA_OFFSET, pos)
            if before_deletion(qkey, pos) or qkey in purged:
                continue
            if guid in deleted_guids:
                deleted_guids.discard(guid)
                continue
            if o + 8 > d.size:
                return fail(RC_INVALID_DATA_RECORD, pos)
            w0, w1 = _int(d, o, 4), _int(d, o + 4, 4)
            hs, total, opt = (w0 >> 29) * WORD, (w0 & 0x1FFFFFFF) * WORD, (w1 >> 8) * WORD
            if hs == 0 or total == 0 or hs + opt >= total or o + total > d.size:
                return fail(RC_INVALID_DATA_RECORD, pos)
            pad = int(d[o + total - 1])
            if pad < 1 or pad > DWORD or total < hs + opt + pad:
                return fail(RC_INVALID_DATA_RECORD, pos)
            if qkey not in live:
                return fail(RC_INVALID_QUEUE_KEY, pos)
            out["record_offset"].append(pos)
            out["app_offset"].append(o + hs + opt)
            out["app_length"].append(total - hs - opt - pad)
            out["crc32c"].append(_int(r, 52, 4))
    return out


def _native_call(fn, *args):
    try:
        return fn(*args)
    except N.BmqCrcError as e:
        if e.rc == N.BMQCRC_EINVAL:
            raise StorageFormatError(str(e)) from e
        raise


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a.size else None


def journal_bounds(journal):
    """Native ``bmqcrc_journal_bounds``: (last sync point offset, last record
    offset) as JournalFileIterator bounds the journal (0 = none)."""
    j = np.ascontiguousarray(_as_u8(journal))
    lsp, last = ctypes.c_uint64(0), ctypes.c_uint64(0)
    _native_call(lambda: N.check(N.lib.bmqcrc_journal_bounds(
        _ptr(j), j.size, ctypes.byref(lsp), ctypes.byref(last))))
    return int(lsp.value), int(last.value)


def scan_partition(journal, data, with_csl=False, queue_keys=()):
    """Native walk (``bmqcrc_journal_scan``, CPU only): the MESSAGE records
    FileStore::recoverMessages would CRC, in its (backward) order, as numpy
    arrays (record_offset, app_offset, app_length, crc32c), plus the
    reference's recovery_rc and the offending record's error_record_offset."""
    j, d = np.ascontiguousarray(_as_u8(journal)), np.ascontiguousarray(_as_u8(data))
    cfg, _keys = _cfg(with_csl, queue_keys)
    rrc, err = ctypes.c_int(0), ctypes.c_uint64(0)

    def scan(cap, *arrs):
        n = N.lib.bmqcrc_journal_scan(_ptr(j), j.size, _ptr(d), d.size,
                                      ctypes.byref(cfg) if cfg is not None else None,
                                      ctypes.byref(rrc), ctypes.byref(err),
                                      *[_ptr(a) if a is not None else None for a in arrs], cap)
        return N.check_count(n)

    n = _native_call(scan, 0, None, None, None, None)
    out = {"record_offset": np.zeros(n, np.uint64), "app_offset": np.zeros(n, np.uint64),
           "app_length": np.zeros(n, np.uint32), "crc32c": np.zeros(n, np.uint32)}
    _native_call(scan, n, out["record_offset"], out["app_offset"], out["app_length"],
                 out["crc32c"])
    out["recovery_rc"] = int(rrc.value)
    out["error_record_offset"] = int(err.value)
    return out


def verify_partition(journal, data, bad_cap=1 << 20, device=-1, with_csl=False, queue_keys=(),
                     devices=None):
    """Recovery CRC check of a whole partition: one native walk selecting the
    records FileStore::recoverMessages CRCs, one batched GPU verify
    (``bmqcrc_recover_verify``).

    Returns dict(n_messages, n_bad, bad_record_offsets, recovery_rc,
    error_record_offset).  A mismatch is what the reference reports with
    BMQTSK_ALARMLOG_ALARM("RECOVERY") (mqbs_filestore.cpp:2613-2624) and
    keeps going; offsets come in the order it raises them (backward).
    ``devices`` (several ordinals, repeats allowed) spreads the DATA file's
    staging and verify over those devices (bmqcrc_opts.ndevices).
    """
    j, d = np.ascontiguousarray(_as_u8(journal)), np.ascontiguousarray(_as_u8(data))
    cfg, _keys = _cfg(with_csl, queue_keys)
    n_msgs, n_bad = ctypes.c_uint64(0), ctypes.c_uint64(0)
    rrc, err = ctypes.c_int(0), ctypes.c_uint64(0)
    bad = np.zeros(max(int(bad_cap), 1), np.uint64)
    opts = N.make_opts(device=device, devices=devices)

    def run():
        return N.check(N.lib.bmqcrc_recover_verify(
            _ptr(j), j.size, _ptr(d), d.size, ctypes.byref(cfg) if cfg is not None else None,
            ctypes.byref(rrc), ctypes.byref(err), ctypes.byref(n_msgs), ctypes.byref(n_bad),
            _ptr(bad), int(bad_cap), ctypes.byref(opts)))

    _native_call(run)
    k = min(int(n_bad.value), int(bad_cap))
    return {"n_messages": int(n_msgs.value), "n_bad": int(n_bad.value),
            "bad_record_offsets": bad[:k].copy(), "recovery_rc": int(rrc.value),
            "error_record_offset": int(err.value)}


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


class PartitionWriter:
    """Builds a (journal, DATA) file pair record by record, in the layout
    FileStore writes (mqbs_filestoreprotocol.h: RecordHeader :1014,
    MessageRecord :1125, ConfirmRecord :1339, DeletionRecord :1518,
    QueueOpRecord :1694, JournalOpRecord :1953, DataHeader :703).  Every
    record takes the next sequence number of the current primary lease;
    ``new_lease`` starts a new primary (sequence numbers restart at 1).  Each
    method returns the record's journal offset (``message`` also its GUID)."""

    JOURNAL_HEADER = 32 + 12  # FileHeader + JournalFileHeader (3 words)

    def __init__(self, lease_id=1, timestamp=0x6720EAB4, partition_id=0):
        self.lease, self.seq, self.ts = lease_id, 0, timestamp
        self.recs = []
        self.data = [file_header(FILE_TYPE_DATA, partition_id).tobytes(),
                     bytes([2, 0, 0, 0, 0, 0, 0, 0])]
        self.dpos = 40
        self.partition_id = partition_id
        self._guid = 0

    def _record(self, rtype, body, flags=0):
        self.seq += 1
        r = bytearray(JOURNAL_RECORD_SIZE)
        r[0:2] = ((rtype << 12) | (flags & 0xFFF)).to_bytes(2, "big")
        r[2:4] = (self.seq >> 32).to_bytes(2, "big")
        r[4:8] = (self.seq & 0xFFFFFFFF).to_bytes(4, "big")
        r[8:12] = self.lease.to_bytes(4, "big")
        r[12:20] = self.ts.to_bytes(8, "big")
        for off, b in body:
            r[off:off + len(b)] = b
        r[56:60] = RECORD_MAGIC.to_bytes(4, "big")
        self.recs.append(bytes(r))
        return self.JOURNAL_HEADER + (len(self.recs) - 1) * JOURNAL_RECORD_SIZE

    def new_lease(self, lease_id):
        self.lease, self.seq = lease_id, 0

    def sync_point(self, sync_type=1):
        """JournalOpRecord SYNCPOINT for the current PSN (its own sequence
        number, :1953), pointing at the current end of the DATA file."""
        seq = self.seq + 1
        return self._record(REC_JOURNAL_OP, [
            (23, bytes([sync_type])), (24, JOURNAL_OP_SYNCPOINT.to_bytes(4, "big")),
            (28, (seq >> 32).to_bytes(4, "big")), (32, (seq & 0xFFFFFFFF).to_bytes(4, "big")),
            (40, self.lease.to_bytes(4, "big")), (44, (self.dpos // DWORD).to_bytes(4, "big")),
            (48, (9).to_bytes(4, "big"))])

    def queue_op(self, op, queue_key, app_key=NULL_KEY):
        return self._record(REC_QUEUE_OP, [
            (22, bytes(queue_key)), (27, bytes(app_key)), (32, int(op).to_bytes(4, "big")),
            (36, (9 if op in (OP_CREATION, OP_ADDITION) else 0).to_bytes(4, "big"))])

    def message(self, app, queue_key, crc=None, guid=None, data_header=None):
        """MESSAGE record + its DATA record (12-byte DataHeader, no options,
        1..8 padding bytes).  `crc` overrides the stored CRC (default: the
        CRC32C of `app`); `data_header` overrides the DataHeader bytes."""
        app = bytes(app)
        rem = (12 + len(app)) % DWORD
        pad = DWORD - rem if rem else DWORD
        total = 12 + len(app) + pad
        hdr = data_header if data_header is not None else \
            ((3 << 29) | (total // WORD)).to_bytes(4, "big") + bytes(8)
        self.data.append(bytes(hdr) + app + bytes([pad]) * pad)
        if guid is None:
            self._guid += 1
            guid = (0x40000000000000000000000000000000 | self._guid).to_bytes(16, "big")
        crc = Crc32c.calculate(app) if crc is None else int(crc)
        off = self._record(REC_MESSAGE, [
            (22, bytes(queue_key)), (32, (self.dpos // DWORD).to_bytes(4, "big")),
            (36, bytes(guid)), (52, crc.to_bytes(4, "big"))], flags=1)
        self.dpos += total
        return off, bytes(guid)

    def confirm(self, guid, queue_key, app_key=NULL_KEY):
        return self._record(REC_CONFIRM, [(22, bytes(queue_key)), (27, bytes(app_key)),
                                          (32, bytes(guid))])

    def deletion(self, guid, queue_key):
        return self._record(REC_DELETION, [(23, bytes(queue_key)), (28, bytes(guid))])

    def files(self):
        journal = file_header(FILE_TYPE_JOURNAL, self.partition_id).tobytes() + \
            bytes([3, 15]) + bytes(10) + b"".join(self.recs)
        return (np.frombuffer(journal, np.uint8).copy(),
                np.frombuffer(b"".join(self.data), np.uint8).copy())


DEFAULT_QUEUE_KEY = b"\x26\xda\xcd\xc9\x74"


def write_partition(app_datas, crcs=None, lease_id=1, timestamp=0x6720EAB4,
                    queue_key=DEFAULT_QUEUE_KEY):
    """(journal, data) byte arrays of one queue: a QueueOp CREATION record,
    then one MESSAGE record per entry of `app_datas` (bytes), all of them
    outstanding.  `crcs` (optional) overrides the CRC stored in the journal
    (default: the true CRC32C of the app data)."""
    w = PartitionWriter(lease_id=lease_id, timestamp=timestamp)
    w.queue_op(OP_CREATION, queue_key)
    for i, app in enumerate(app_datas):
        w.message(app, queue_key, crc=None if crcs is None else crcs[i])
    return w.files()
