"""The vectorized synthetic partition / PUT event generators used by
``bench.py --protocol`` produce exactly the bytes of the reference-layout
writers in storage.py / put_event.py, and the native walks accept them."""
import numpy as np

from blazingmq_amd import put_event as P
from blazingmq_amd import storage as S
from blazingmq_amd import synth


def test_partition_matches_writer():
    journal, data, app_off, app_len = synth.partition(7, 29, seed=3)
    apps = [data[int(o):int(o) + int(n)].tobytes() for o, n in zip(app_off, app_len)]
    jw, dw = S.write_partition(apps)
    assert np.array_equal(journal, jw)
    assert np.array_equal(data, dw)
    walk = S.scan_partition(journal, data)
    assert walk["recovery_rc"] == 0
    assert np.array_equal(walk["app_offset"][::-1], app_off)
    assert np.array_equal(walk["app_length"][::-1], app_len)


def test_put_event_matches_builder():
    event, app_off, app_len = synth.put_event(5, 13, seed=4)
    b = P.PutEventBuilder(defer_crc=True)
    for o, n in zip(app_off, app_len):
        b.pack_message(event[int(o):int(o) + int(n)].tobytes())
    built = np.frombuffer(b"".join(b._chunks), np.uint8).copy()
    built[0:4] = np.frombuffer((built.size & 0x7FFFFFFF).to_bytes(4, "big"), np.uint8)
    built[4] = (P.PROTOCOL_VERSION << 6) | P.EVENT_TYPE_PUT
    built[5] = P.EVENT_HEADER_SIZE // P.WORD
    assert np.array_equal(event, built)
    off, ln, _ = P.PutMessageIterator(event).scan()
    assert np.array_equal(off, app_off) and np.array_equal(ln, app_len)
