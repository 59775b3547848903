"""PUT events with a deferred, batched CRC32C (the producer side of the path).

Host-side mirror of ``bmqp::PutEventBuilder`` / ``bmqp::PutMessageIterator``
wire format (/root/reference/src/groups/bmq/bmqp/bmqp_puteventbuilder.cpp,
bmqp_protocol.h):

  EventHeader (bmqp_protocol.h:746, 8 bytes)
      BE u32  F(1b)|Length(31b); u8 PV(2b)|Type(6b); u8 HeaderWords=2; u8 typeSpecific; u8 0
  per message: PutHeader (bmqp_protocol.h:1374, 36 bytes)
      BE u32  Flags(4b)|MessageWords(28b)
      BE u32  OptionsWords(24b)|CAT(3b)|HeaderWords(5b)=9
      BE i32  QueueId;  GUID[16];  BE u32 CRC32-C (@28);  SchemaId(2) Reserved(2)
  then options, application data (properties + payload) and 1..4 padding
  bytes each equal to the padding count (ProtocolUtil::calcNumWordsAndPadding,
  bmqp_protocolutil.h:312; k_PADDING_DATA bmqp_protocolutil.cpp:44).

The reference computes ``Crc32c::calculate(appData)`` once per message inside
``packMessage`` (bmqp_puteventbuilder.cpp:302,320,400,413) and writes it into
``PutHeader::d_crc32c`` (:146-153).  ``PutEventBuilder(defer_crc=True)`` packs
every message with the CRC field pending and ``finalize()`` fills all of them
with one batched GPU call before the event is posted
(``bmqcrc_put_event_fill_crcs``: a native walk of the event, then one batch).
``PutMessageIterator.verify_crcs()`` is the batched form of the iterator's
recompute (bmqp_putmessageiterator.cpp:670-679): ``bmqcrc_put_event_verify``.
"""
import ctypes

import numpy as np

from . import _native as N
from .crc32c import Crc32c

EVENT_HEADER_SIZE = 8
PUT_HEADER_SIZE = 36
EVENT_TYPE_PUT = 2
PROTOCOL_VERSION = 1
WORD = 4


def _pad_len(n):
    # calcNumWordsAndPadding: numWords = (len + 4) / 4, padding = 4*numWords - len (1..4)
    return ((n + WORD) // WORD) * WORD - n


class PutEventBuilder:
    """Build one PUT event.  ``pack_message`` appends a message; with
    ``defer_crc=False`` the CRC is computed immediately on the CPU (like the
    reference), with ``defer_crc=True`` ``finalize()`` computes all CRCs in one
    batch on the GPU."""

    def __init__(self, defer_crc=True, devices=None):
        self.defer_crc = defer_crc
        self.devices = devices  # several ordinals: spread the deferred fill over them
        self._chunks = [bytes(EVENT_HEADER_SIZE)]
        self._size = EVENT_HEADER_SIZE
        self._app_off = []   # offset of app data inside the event
        self._app_len = []
        self._crc_pos = []   # offset of the PutHeader CRC field
        self._finalized = False

    def pack_message(self, app_data, queue_id=0, guid=None, flags=0, options=b""):
        """Append one message: ``app_data`` = properties + payload (bytes)."""
        if self._finalized:
            raise RuntimeError("event already finalized")
        app = bytes(app_data)
        if len(options) % WORD:
            raise ValueError("options must be word aligned")
        pad = _pad_len(len(app))
        header_words = PUT_HEADER_SIZE // WORD
        options_words = len(options) // WORD
        msg_words = header_words + options_words + (len(app) + pad) // WORD
        h = bytearray(PUT_HEADER_SIZE)
        h[0:4] = (((flags & 0xF) << 28) | msg_words).to_bytes(4, "big")
        h[4:8] = ((options_words << 8) | header_words).to_bytes(4, "big")
        h[8:12] = int(queue_id).to_bytes(4, "big", signed=True)
        h[12:28] = bytes(guid) if guid is not None else bytes(16)
        crc = 0 if self.defer_crc else Crc32c.calculate(app)
        h[28:32] = crc.to_bytes(4, "big")
        self._crc_pos.append(self._size + 28)
        self._app_off.append(self._size + PUT_HEADER_SIZE + len(options))
        self._app_len.append(len(app))
        self._chunks += [bytes(h), bytes(options), app, bytes([pad]) * pad]
        self._size += PUT_HEADER_SIZE + len(options) + len(app) + pad
        return len(self._app_off) - 1

    def message_count(self):
        return len(self._app_off)

    def finalize(self):
        """Return the event bytes (EventHeader filled; pending CRCs computed
        in one GPU batch when ``defer_crc``)."""
        ev = np.frombuffer(b"".join(self._chunks), dtype=np.uint8).copy()
        ev[0:4] = np.frombuffer((self._size & 0x7FFFFFFF).to_bytes(4, "big"), np.uint8)
        ev[4] = (PROTOCOL_VERSION << 6) | EVENT_TYPE_PUT
        ev[5] = EVENT_HEADER_SIZE // WORD
        if self.defer_crc and self._app_off:
            opts = N.make_opts(devices=self.devices)
            n = N.check_count(N.lib.bmqcrc_put_event_fill_crcs(
                ctypes.c_void_p(ev.ctypes.data), ev.size, ctypes.byref(opts)))
            if n != len(self._app_off):
                raise RuntimeError("PUT event walk found %d messages, packed %d"
                                   % (n, len(self._app_off)))
        self._finalized = True
        return ev


class PutMessageIterator:
    """Iterate the messages of a PUT event: (put header fields, app data)."""

    def __init__(self, event):
        self.ev = np.frombuffer(bytes(event), dtype=np.uint8) if not isinstance(
            event, np.ndarray) else event.view(np.uint8)
        length = int.from_bytes(self.ev[0:4].tobytes(), "big") & 0x7FFFFFFF
        if length != self.ev.size or (int(self.ev[4]) & 0x3F) != EVENT_TYPE_PUT:
            raise ValueError("not a PUT event of matching length")
        self.header_size = int(self.ev[5]) * WORD

    def scan(self):
        """Native walk (``bmqcrc_put_event_scan``, CPU only): numpy arrays
        (app_offset, app_length, crc_pos) of every message."""
        ev = np.ascontiguousarray(self.ev)
        p = ctypes.c_void_p(ev.ctypes.data)
        n = N.check_count(N.lib.bmqcrc_put_event_scan(p, ev.size, None, None, None, 0))
        off, ln, pos = np.zeros(n, np.uint64), np.zeros(n, np.uint32), np.zeros(n, np.uint64)
        if n:
            N.check_count(N.lib.bmqcrc_put_event_scan(
                p, ev.size, ctypes.c_void_p(off.ctypes.data), ctypes.c_void_p(ln.ctypes.data),
                ctypes.c_void_p(pos.ctypes.data), n))
        return off, ln, pos

    def verify_crcs(self, bad_cap=1 << 16, device=-1, devices=None):
        """Check every PutHeader CRC against its application data in one GPU
        batch (``devices``: spread over several devices, bmqcrc_opts.ndevices).
        Returns (n_messages, n_bad, bad message indices)."""
        ev = np.ascontiguousarray(self.ev)
        n_msgs, n_bad = ctypes.c_uint64(0), ctypes.c_uint64(0)
        bad = np.zeros(max(int(bad_cap), 1), np.uint64)
        opts = N.make_opts(device=device, devices=devices)
        N.check(N.lib.bmqcrc_put_event_verify(
            ctypes.c_void_p(ev.ctypes.data), ev.size, ctypes.byref(n_msgs), ctypes.byref(n_bad),
            ctypes.c_void_p(bad.ctypes.data), int(bad_cap), ctypes.byref(opts)))
        k = min(int(n_bad.value), int(bad_cap))
        return int(n_msgs.value), int(n_bad.value), bad[:k].copy()

    def __iter__(self):
        pos = self.header_size
        ev = self.ev
        while pos < ev.size:
            w0 = int.from_bytes(ev[pos:pos + 4].tobytes(), "big")
            w1 = int.from_bytes(ev[pos + 4:pos + 8].tobytes(), "big")
            msg_bytes = (w0 & 0x0FFFFFFF) * WORD
            hw = (w1 & 0x1F) * WORD
            opt = (w1 >> 8) * WORD
            end = pos + msg_bytes
            pad = int(ev[end - 1])
            app = ev[pos + hw + opt:end - pad].tobytes()
            yield {
                "flags": w0 >> 28,
                "queue_id": int.from_bytes(ev[pos + 8:pos + 12].tobytes(), "big", signed=True),
                "guid": ev[pos + 12:pos + 28].tobytes(),
                "crc32c": int.from_bytes(ev[pos + 28:pos + 32].tobytes(), "big"),
                "app_data": app,
                "app_offset": pos + hw + opt,
            }
            pos = end
