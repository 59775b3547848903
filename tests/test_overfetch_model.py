"""tools/zipf_overfetch.py's model of Zipf's traffic above its algorithmic
bytes: the descriptor lines each size class fetches."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _model():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import zipf_overfetch
    return zipf_overfetch


def test_descriptor_lines_per_class():
    m = _model()
    # one class: 32 messages' offsets (8 B) fill 2 lines, lengths (4 B) one
    assert m.desc_by_class(np.full(32, 64, np.uint32)) == 3 * 128
    # two classes interleaved (64 B: class 0; 4 KiB at 2 KiB segments: class
    # 8 for both segments): each class touches every line once
    assert m.desc_by_class(np.tile(np.array([64, 4096], np.uint32), 16)) == 2 * 3 * 128
    # the same messages sorted by size: each class its own lines
    assert m.desc_by_class(np.repeat(np.array([64, 4096], np.uint32), 16)) == 4 * 128


def test_shared_lines_and_alignment():
    m = _model()
    # 64-byte messages back to back: every other boundary cuts a line
    r = m.model(np.full(64, 64, np.uint32))
    assert r["shared_lines"] == 32 and r["lines_128_bytes"] == 64 * 128
    # 128-byte messages: no shared line
    assert m.model(np.full(64, 128, np.uint32))["shared_lines"] == 0
