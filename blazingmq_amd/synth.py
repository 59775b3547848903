"""Vectorized synthetic inputs in the reference's wire/disk formats, for the
measurements of the batch callers (``bench.py --protocol``):
a partition (journal + DATA file) of fixed-size messages and a PUT event of
fixed-size messages.  Byte-for-byte the layouts ``storage.write_partition``
and ``put_event.PutEventBuilder`` produce (checked in
``tests/test_synth.py``), built with numpy instead of a Python loop so that
GiB-sized inputs take seconds.

CRCs are computed with the library's scalar CPU path (``bmqcrc_crc32c``, the
drop-in for ``bmqp::Crc32c::calculate``), never with the test oracle.
"""
import ctypes

import numpy as np

from . import _native as N
from . import put_event as P
from . import storage as S


def _be(x, dtype):
    a = np.ascontiguousarray(np.asarray(x).astype(dtype))
    return a.reshape(-1).view(np.uint8).reshape(a.shape + (np.dtype(dtype).itemsize,))


def host_crcs(buf, offsets, lengths):
    """CRC32C of every [off, off+len) of a host buffer, scalar CPU path."""
    base = buf.ctypes.data
    f = N.lib.bmqcrc_crc32c
    return np.array([f(ctypes.c_void_p(base + int(o)), int(n), 0)
                     for o, n in zip(offsets, lengths)], dtype=np.uint32)


def partition(n, app_len, seed=11, lease_id=1, timestamp=0x6720EAB4,
              queue_key=S.DEFAULT_QUEUE_KEY):
    """(journal, data, app_offsets, app_lengths) for one queue: a QueueOp
    CREATION record, then n MESSAGE records whose application data are
    `app_len` random bytes each, all outstanding (mqbs_filestoreprotocol.h
    QueueOpRecord :1694, DataHeader :703, MessageRecord :1125) -- the bytes
    ``storage.write_partition`` produces."""
    rng = np.random.default_rng(seed)
    rem = (12 + app_len) % S.DWORD
    pad = S.DWORD - rem if rem else S.DWORD
    total = 12 + app_len + pad
    recs = np.zeros((n, total), np.uint8)
    recs[:, 0:4] = _be((3 << 29) | (total // S.WORD), ">u4")
    recs[:, 12:12 + app_len] = rng.integers(0, 256, size=(n, app_len), dtype=np.uint8)
    recs[:, 12 + app_len:] = pad
    head = np.concatenate([S.file_header(S.FILE_TYPE_DATA),
                           np.array([2, 0, 0, 0, 0, 0, 0, 0], np.uint8)])
    data = np.concatenate([head, recs.reshape(-1)])
    pos = head.size + np.arange(n, dtype=np.uint64) * total
    app_off = pos + 12
    app_lens = np.full(n, app_len, np.uint32)
    crcs = host_crcs(data, app_off, app_lens)

    seq = 1 + np.arange(n + 1, dtype=np.uint64)  # record 0: the queue's CREATION
    j = np.zeros((n + 1, S.JOURNAL_RECORD_SIZE), np.uint8)
    j[:, 0:2] = _be((S.REC_MESSAGE << 12) | 1, ">u2")
    j[0, 0:2] = _be(S.REC_QUEUE_OP << 12, ">u2")
    j[:, 2:4] = _be(seq >> 32, ">u2")
    j[:, 4:8] = _be(seq & 0xFFFFFFFF, ">u4")
    j[:, 8:12] = _be(lease_id, ">u4")
    j[:, 12:20] = _be(timestamp, ">u8")
    j[:, 22:27] = np.frombuffer(queue_key, np.uint8)
    j[0, 32:36] = _be(S.OP_CREATION, ">u4")
    j[0, 36:40] = _be(9, ">u4")
    m = j[1:]
    m[:, 32:36] = _be(pos // S.DWORD, ">u4")
    m[:, 36] = 0x40
    m[:, 44:52] = _be(np.arange(1, n + 1, dtype=np.uint64), ">u8")
    m[:, 52:56] = _be(crcs, ">u4")
    j[:, 56:60] = _be(S.RECORD_MAGIC, ">u4")
    jhead = np.concatenate([S.file_header(S.FILE_TYPE_JOURNAL),
                            np.array([3, 15] + [0] * 10, np.uint8)])
    journal = np.concatenate([jhead, j.reshape(-1)])
    return journal, data, app_off, app_lens


def put_event(m, app_len, seed=12):
    """(event, app_offsets, app_lengths) for one PUT event of m messages whose
    application data are `app_len` random bytes, CRC fields pending (zero),
    as PutEventBuilder(defer_crc=True) packs them before finalize()
    (bmqp_protocol.h:746 EventHeader, :1374 PutHeader)."""
    rng = np.random.default_rng(seed)
    pad = P._pad_len(app_len)
    msg = P.PUT_HEADER_SIZE + app_len + pad
    recs = np.zeros((m, msg), np.uint8)
    recs[:, 0:4] = _be(msg // P.WORD, ">u4")
    recs[:, 4:8] = _be(P.PUT_HEADER_SIZE // P.WORD, ">u4")
    recs[:, P.PUT_HEADER_SIZE:P.PUT_HEADER_SIZE + app_len] = rng.integers(
        0, 256, size=(m, app_len), dtype=np.uint8)
    recs[:, P.PUT_HEADER_SIZE + app_len:] = pad
    size = P.EVENT_HEADER_SIZE + m * msg
    head = np.zeros(P.EVENT_HEADER_SIZE, np.uint8)
    head[0:4] = _be(size & 0x7FFFFFFF, ">u4")
    head[4] = (P.PROTOCOL_VERSION << 6) | P.EVENT_TYPE_PUT
    head[5] = P.EVENT_HEADER_SIZE // P.WORD
    event = np.concatenate([head, recs.reshape(-1)])
    app_off = P.EVENT_HEADER_SIZE + np.arange(m, dtype=np.uint64) * msg + P.PUT_HEADER_SIZE
    return event, app_off, np.full(m, app_len, np.uint32)
