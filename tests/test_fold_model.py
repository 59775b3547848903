"""CPU model of the device fold algorithm, checked
against the oracle: sparse-relation word recurrence over a 32-word ring,
remainder Horner by x^32, x^e move (e mod 2^31-1), seed injection, byte
masking, segment XOR-combine.  Proves the math the HIP kernel implements."""
import numpy as np
import pytest

import oracle

POLY_R = 0x82F63B78


def _consts():
    import importlib.util
    import os
    p = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools",
                     "gen_crc_consts.py")
    spec = importlib.util.spec_from_file_location("gen", p)
    g = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(g)
    taps = [k for k in g.min_poly_of_y() if k < 32]
    return g, taps


G, TAPS = _consts()


def mul_y(c):
    for _ in range(32):
        c = (c >> 1) ^ (POLY_R if c & 1 else 0)
    return c


def xpow(e):
    r, sq = 1 << 31, 1 << 30
    e %= (1 << 31) - 1
    while e:
        if e & 1:
            r = G.mulmod_r(r, sq)
        sq = G.mulmod_r(sq, sq)
        e >>= 1
    return r


def fold_stream(words):
    """raw CRC (zero init, no final xor) of a word stream, len % 32 == 0."""
    q = [0] * 32
    nr = len(words) // 32
    c = 0
    for r in range(nr):
        m = words[32 * r:32 * r + 32]
        if r + 1 < nr:
            for d in range(32):
                acc = m[d]
                for k in TAPS:
                    acc ^= q[(d + k) & 31]
                q[d] = acc
        else:
            for d in range(32):
                acc = m[d]
                for k in TAPS:
                    if d + k <= 31:
                        acc ^= q[d + k]
                c = mul_y(c ^ acc)
    return c


def geom(S, E, first, ra_lines=1):
    """k_fold's seg_geom (round 3): when that saves a line or the stream is at
    most ra_lines lines (kRightAlignLines), the stream is right-aligned at
    piece granularity -- it ends with the 16-byte piece holding its last byte
    (or the seed word's) and starts nl lines before, nl the fewest lines that
    hold pieces [S/16, that piece]; otherwise it starts at S's 128-byte line.
    Returns (L0, nl)."""
    need_end = max(E, S + 4) if first else E
    pe = (need_end + 15) & ~15
    nl_r = (pe - (S & ~15) + 127) // 128
    L0_l = S & ~127
    nl_l = (need_end - L0_l + 127) // 128
    if nl_r < nl_l or nl_r <= ra_lines:
        return pe - 128 * nl_r, nl_r
    return L0_l, nl_l


def segment_contrib(arena, S, E, mstart, mend, first, seed):
    L0, nl = geom(S, E, first)
    stream = bytearray(128 * nl)
    lo, hi = S - L0, min(E, L0 + 128 * nl) - L0
    stream[lo:hi] = arena[S:E].tobytes()
    if first:
        for b in range(4):
            stream[lo + b] ^= ((~seed & 0xFFFFFFFF) >> (8 * b)) & 0xFF
    words = list(np.frombuffer(bytes(stream), dtype="<u4").astype(np.uint64))
    c = fold_stream([int(w) for w in words])
    padE = L0 + 128 * nl - E
    contrib = G.mulmod_r(c, xpow(8 * (mend - E) - 8 * padE))
    return contrib ^ (0xFFFFFFFF if first else 0)


def model_batch(arena, offs, lens, seeds, seg):
    out = []
    for off, ln, seed in zip(offs, lens, seeds):
        if ln == 0:
            out.append(seed)
            continue
        nseg = (ln - 1) // seg + 1
        b = [off] + [((off + k * seg) & ~127) for k in range(1, nseg)] + [off + ln]
        acc = 0
        for k in range(nseg):
            acc ^= segment_contrib(arena, b[k], b[k + 1], off, off + ln, k == 0, seed)
        out.append(acc)
    return out


def test_relation_vanishes():
    acc = 0
    for k in TAPS + [32]:
        acc ^= G.ppow(2, 32 * k, G.P_NORMAL)
    assert acc == 0 and len(TAPS) == 17


@pytest.mark.parametrize("seg", [256, 384, 1024])
def test_model_matches_oracle(seg):
    rng = np.random.default_rng(seg)
    arena = rng.integers(0, 256, size=20000, dtype=np.uint8)
    lens = [0, 1, 2, 3, 4, 5, 31, 127, 128, 129, 300, 1000, 2500]
    offs = [int(rng.integers(0, arena.size - l)) for l in lens]
    offs[4] = 126  # seed word crossing a line boundary
    seeds = [int(rng.integers(0, 2**32)) for _ in lens]
    got = model_batch(arena, offs, lens, seeds, seg)
    exp = [oracle.crc32c(arena[o:o + l].tobytes(), s) for o, l, s in zip(offs, lens, seeds)]
    assert got == exp


def _segment_pieces(arena, S, E, first, seed, lead_lines):
    """The k_fold stream construction: lead_lines zero lines (right alignment
    in the wave), then the segment's lines, where every 16-byte piece outside
    [S, E) is a zero piece (the DMA reads the zero line) and only the pieces cut
    by S or E are masked byte-exactly; the seed is XORed in last."""
    L0, nl = geom(S, E, first)
    sl, el = S - L0, E - L0
    gS, gE = sl // 16, (el + 15) // 16
    line = bytearray(128 * nl)
    for p in range(gS, gE):  # pieces read from HBM
        line[16 * p:16 * p + 16] = arena[L0 + 16 * p:L0 + 16 * p + 16].tobytes()
    if sl % 16:
        line[16 * (sl // 16):sl] = bytes(sl - 16 * (sl // 16))
    if el % 16:
        line[el:16 * gE] = bytes(16 * gE - el)
    if first:
        for b in range(4):
            line[sl + b] ^= ((~seed & 0xFFFFFFFF) >> (8 * b)) & 0xFF
    return bytes(128 * lead_lines) + bytes(line), nl


@pytest.mark.parametrize("lead", [0, 1, 5])
def test_right_aligned_pieces_match_oracle(lead):
    rng = np.random.default_rng(100 + lead)
    arena = rng.integers(0, 256, size=8192, dtype=np.uint8)
    for _ in range(60):
        ln = int(rng.integers(0, 700))
        off = int(rng.integers(0, arena.size - ln - 200))
        seed = int(rng.integers(0, 2**32))
        stream, nl = _segment_pieces(arena, off, off + ln, True, seed, lead)
        words = [int(w) for w in np.frombuffer(stream, dtype="<u4")]
        c = fold_stream(words)  # leading zero lines leave a zero-init CRC unchanged
        L0 = geom(off, off + ln, True)[0]
        padE = L0 + 128 * nl - (off + ln)
        if L0 % 128:  # right-aligned: no unshift when E is 16-byte aligned
            assert 0 <= padE < 16 or ln < 4
        got = G.mulmod_r(c, xpow(-8 * padE)) ^ 0xFFFFFFFF
        assert got == oracle.crc32c(arena[off:off + ln].tobytes(), seed), (off, ln, lead)


def test_right_alignment_saves_lines():
    # a message that straddles a line boundary but fits 128 bytes is one line
    assert geom(64, 192, True)[1] == 1 and geom(64, 320, True)[1] == 2
    assert geom(0, 64, True) == (-64, 1)     # one line: right-aligned
    assert geom(0, 320, True) == (0, 3)      # saves nothing: whole cache lines
    assert geom(0, 320, True, 1 << 30) == (-64, 3)
    # never more lines than the 128-byte aligned start of round 2
    for S in range(0, 300, 7):
        for ln in range(0, 700, 13):
            need_end = max(S + ln, S + 4)
            assert geom(S, S + ln, True)[1] <= (need_end - (S & ~127) + 127) // 128


def horner_words(words, skip=0):
    """k_fold's tail_horner: raw = sum R_d y^(32-d), two words per step,
    the first `skip` steps not run."""
    c = 0
    for d in range(2 * skip, 32):
        c = mul_y(c ^ words[d])
    return c


T11 = G.remainder_tables11()


def chains11(words, skip=False):
    """k_fold's tail_chains11 (8-wave blocks): 11/11/10-bit slices, one word
    per step, chain A over words 0-15 and B over 16-31, raw = A * y^16 + B.
    The slice offsets are formed as the kernel forms them: v & 0x1ffc,
    (v >> 11) & 0x1ffc and rotr(v, 22) & 0xffc (byte offsets into the
    tables)."""
    def step(c, r):
        v = c ^ r
        rot = ((v >> 22) | (v << 10)) & 0xFFFFFFFF
        return (T11[(v & 0x1FFC) >> 2] ^ T11[2048 + (((v >> 11) & 0x1FFC) >> 2)] ^
                T11[4096 + ((rot & 0xFFC) >> 2)])
    ca = cb = 0
    for d in range(16):
        if not skip:
            ca = step(ca, words[d])
        cb = step(cb, words[16 + d])
    if skip:
        return cb
    j = 0
    for k in range(4):
        j ^= T11[5120 + 256 * k + ((ca >> (8 * k)) & 0xFF)]
    return j ^ cb


def test_chains11_match_horner():
    rng = np.random.default_rng(11)
    for _ in range(300):
        words = [int(w) for w in rng.integers(0, 2**32, size=32, dtype=np.uint64)]
        assert chains11(words) == horner_words(words)
        zero_a = [0] * 16 + words[16:]
        assert chains11(zero_a, skip=True) == chains11(zero_a) == horner_words(zero_a, 8)
    for w in (0, 1, 3, 0x80000000, 0xFFFFFFFF, 0x00FFE000, 0xFF000003):
        words = [w] * 32
        assert chains11(words) == horner_words(words)


def bytes8(words, skip16=False):
    """k_fold's tail_bytes8 (BMQCRC_BYTE_FOLD): the 32 remainder words folded
    at byte granularity with the same taps (P(z) = 0 for z = x^8) to 8 words,
    word-parallel with v_alignbyte windows and the pair stream, then 8
    one-word chain steps."""
    def alignbyte(hi, lo, s):
        return (((hi << 32) | lo) >> (8 * s)) & 0xFFFFFFFF

    Q = [0] * 24
    P2 = [0] * 25

    def lagw(W, n, j, L):
        q, s = L >> 2, L & 3
        hi, lo = j - q, j - q - 1
        h = W[hi] if 0 <= hi < n and not (skip16 and hi < 16) else 0
        if s == 0:
            return h
        lo_v = W[lo] if 0 <= lo < n and not (skip16 and lo < 16) else 0
        return alignbyte(h, lo_v, 4 - s)

    def taps(j, nq):
        t = lagw(Q, nq, j, 32) ^ lagw(Q, nq, j, 26) ^ lagw(Q, nq, j, 12)
        for L in (23, 21, 18, 13, 9, 6, 4):
            t ^= lagw(P2, nq + 1, j, L)
        return t

    for j in range(24):
        if skip16 and j < 16:
            continue
        Q[j] = words[j] ^ taps(j, j)
        P2[j] = Q[j] ^ alignbyte(Q[j], Q[j - 1] if j > 0 else 0, 3)
    P2[24] = alignbyte(0, Q[23], 3)
    c = 0
    for j in range(24, 32):
        c = mul_y(c ^ words[j] ^ taps(j, 24))
    return c


def test_bytes8_match_horner():
    # the byte-granular relation: same taps as the word ring
    assert [k for k in G.min_poly_of_y() if k < 32] == TAPS
    rng = np.random.default_rng(8)
    for _ in range(200):
        words = [int(w) for w in rng.integers(0, 2**32, size=32, dtype=np.uint64)]
        assert bytes8(words) == horner_words(words)
        zero_a = [0] * 16 + words[16:]
        assert bytes8(zero_a, skip16=True) == bytes8(zero_a) == horner_words(zero_a)
    for w in (1, 0x80000000, 0xFFFFFFFF, 0x000000FF, 0xFF000000):
        for pos in (0, 5, 15, 16, 23, 24, 31):
            words = [0] * 32
            words[pos] = w
            assert bytes8(words) == horner_words(words)


def test_one_line_horner_skip():
    # One-line groups: the remainder is the line, and words before the lowest
    # S of the wave are zero, so hskip = min(sl) // 8 steps can be skipped.
    rng = np.random.default_rng(7)
    arena = rng.integers(0, 256, size=4096, dtype=np.uint8)
    for _ in range(200):
        ln = int(rng.integers(0, 129))
        off = int(rng.integers(0, 3000))
        seed = int(rng.integers(0, 2**32))
        stream, nl = _segment_pieces(arena, off, off + ln, True, seed, 0)
        if nl != 1:
            continue
        L0, _ = geom(off, off + ln, True)
        words = [int(w) for w in np.frombuffer(stream, dtype="<u4")]
        skip = (off - L0) >> 3
        assert all(w == 0 for w in words[:2 * skip])
        c = horner_words(words, skip)
        assert c == horner_words(words) == fold_stream(words)
        padE = L0 + 128 - (off + ln)
        got = G.mulmod_r(c, xpow(-8 * padE)) ^ 0xFFFFFFFF
        assert got == oracle.crc32c(arena[off:off + ln].tobytes(), seed)


# Tap pairing used by k_fold's fold_round / tail_round: adjacent taps (k, k+1)
# are read from a second ring p[j] = Q_m ^ Q_{m+1}, updated once per word.
PAIRS = [8, 10, 13, 18, 22, 25, 27]
SINGLES = [0, 6, 20]


def fold_stream_pairs(words):
    q, p = [0] * 32, [0] * 32
    nr = len(words) // 32
    c = 0
    for r in range(nr):
        m = words[32 * r:32 * r + 32]
        if r + 1 < nr:
            for d in range(32):
                acc = m[d]
                for k in SINGLES:
                    acc ^= q[(d + k) & 31]
                for k in PAIRS:
                    acc ^= p[(d + k) & 31]
                q[d] = acc
                p[(d + 31) & 31] = q[(d + 31) & 31] ^ acc
        else:
            for d in range(32):
                acc = m[d]
                for k in SINGLES:
                    if d + k <= 31:
                        acc ^= q[d + k]
                for k in PAIRS:
                    if d + k + 1 <= 31:
                        acc ^= p[d + k]
                    elif d + k <= 31:
                        acc ^= q[d + k]
                c = mul_y(c ^ acc)
    return c


def test_tap_pairs_cover_relation():
    assert sorted(SINGLES + PAIRS + [k + 1 for k in PAIRS]) == sorted(TAPS)


@pytest.mark.parametrize("rounds", [1, 2, 3, 7])
def test_pair_ring_matches_plain_ring(rounds):
    rng = np.random.default_rng(rounds)
    for _ in range(20):
        words = [int(w) for w in rng.integers(0, 1 << 32, size=32 * rounds, dtype=np.uint64)]
        assert fold_stream_pairs(words) == fold_stream(words)


def first_round_pairs(m):
    """k_fold's first_round: zero history, taps into the previous round dropped."""
    q, p = [0] * 32, [0] * 32
    for d in range(32):
        acc = m[d]
        for k in SINGLES:
            if d + k >= 32:
                acc ^= q[d + k - 32]
        for k in PAIRS:
            if d + k >= 31:
                acc ^= p[(d + k) & 31]
        q[d] = acc
        p[(d + 31) & 31] = acc if d == 0 else q[d - 1] ^ acc
    return q, p


def test_first_round_equals_fold_from_zero():
    rng = np.random.default_rng(5)
    for _ in range(50):
        m = [int(w) for w in rng.integers(0, 1 << 32, size=32, dtype=np.uint64)]
        q, p = [0] * 32, [0] * 32
        for d in range(32):
            acc = m[d]
            for k in SINGLES:
                acc ^= q[(d + k) & 31]
            for k in PAIRS:
                acc ^= p[(d + k) & 31]
            q[d] = acc
            p[(d + 31) & 31] = q[(d + 31) & 31] ^ acc
        assert first_round_pairs(m) == (q, p)


def one_line_stop_contrib(arena, S, E, mstart, mend, first, seed):
    """k_fold's one-line fast path: a stream of one line whose zero padding
    after E is a multiple of 8 bytes stops its Horner after the last data word
    instead of un-shifting by x^(-8 padE)."""
    L0 = S & ~127
    assert E <= L0 + 128 and (not first or E - S >= 4)
    padE = L0 + 128 - E
    assert padE % 8 == 0
    stream = bytearray(128)
    stream[S - L0:E - L0] = arena[S:E].tobytes()
    if first:
        for b in range(4):
            stream[S - L0 + b] ^= ((~seed & 0xFFFFFFFF) >> (8 * b)) & 0xFF
    words = [int(w) for w in np.frombuffer(bytes(stream), dtype="<u4")]
    c = 0
    for d in range(32 - padE // 4):
        c = mul_y(c ^ words[d])
    contrib = G.mulmod_r(c, xpow(8 * (mend - E)))
    return contrib ^ (0xFFFFFFFF if first else 0)


def test_one_line_stop_matches_unshift():
    rng = np.random.default_rng(9)
    arena = rng.integers(0, 256, size=4096, dtype=np.uint8)
    checked = 0
    for _ in range(400):
        L0 = 128 * int(rng.integers(1, 30))
        S = L0 + int(rng.integers(0, 120))
        E = L0 + 128 - 8 * int(rng.integers(0, (L0 + 128 - S) // 8 + 1))
        first = bool(rng.integers(0, 2))
        if E <= S or (first and E - S < 4):
            continue
        seed = int(rng.integers(0, 1 << 32))
        mend = E + 8 * int(rng.integers(0, 50))
        assert one_line_stop_contrib(arena, S, E, S, mend, first, seed) == \
            segment_contrib(arena, S, E, S, mend, first, seed)
        checked += 1
    assert checked > 100


def _header_table(name):
    """A brace-initialised table from the generated crc32c_consts.h."""
    import os
    import re
    p = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "blazingmq_amd",
                     "csrc", "crc32c_consts.h")
    text = open(p).read()
    body = text[text.index("#define %s" % name):]
    body = body[:body.index("}\n") + 1]
    return [int(v, 16) for v in re.findall(r"0x([0-9a-f]{8})u", body)]


def test_move_byte_tables_match_xpow():
    """k_fold's move to the message end (mul_xbytes): the product of
    XBYTES[i][byte i of dist] equals x^(8 dist), for the kernel's own header."""
    flat = _header_table("BMQCRC_XBYTES")
    assert len(flat) == 4 * 256
    xb = [flat[256 * i:256 * (i + 1)] for i in range(4)]
    rng = np.random.default_rng(11)
    dists = [0, 1, 255, 256, 65535, 65536, (1 << 24) - 1, 1 << 24, (1 << 32) - 1]
    dists += [int(d) for d in rng.integers(0, 1 << 32, size=200, dtype=np.uint64)]
    for dist in dists:
        f = 1 << 31
        for i in range(4):
            f = G.mulmod_r(f, xb[i][(dist >> (8 * i)) & 0xff])
        assert f == xpow(8 * dist), dist
    # the move applied to a segment CRC: crc(A || zeros(dist)) = crc(A) * x^(8 dist)
    a = rng.integers(0, 256, size=64, dtype=np.uint8).tobytes()
    for dist in (1, 100, 4096, 70000):
        raw = oracle.crc32c(a + bytes(dist), 0) ^ 0xFFFFFFFF
        moved = G.mulmod_r(oracle.crc32c(a, 0) ^ 0xFFFFFFFF, 1 << 31)
        f = 1 << 31
        for i in range(4):
            f = G.mulmod_r(f, xb[i][(dist >> (8 * i)) & 0xff])
        # raw CRCs here include the ~0 initial value, which zeros shift too
        assert G.mulmod_r(moved, f) == raw


def _decode_groups(entries, firstk):
    """k_fold's resolve_sorted over every group of 64 entries."""
    LAST = 0x80000000
    out = []
    for g in range(0, len(entries), 64):
        grp = entries[g:g + 64]
        head = []
        for l, e in enumerate(grp):
            head.append(l == 0 or grp[l - 1] != e or bool(e & LAST))
        for l, e in enumerate(grp):
            h = max(j for j in range(l + 1) if head[j])
            if e & LAST:
                out.append((e & ~LAST, None))  # k from the message's length
            else:
                out.append((e, (firstk[g >> 6] if h == 0 else 0) + (l - h)))
    return out


def test_four_byte_seginfo_round_trip():
    """Round 3's seginfo encoding (put_full / put_last / resolve_sorted): runs of
    full segments written contiguously in k order, last segments flagged, and
    firstk written for entries at multiples of 64 -- decoding every group
    recovers (message, k) exactly, for runs of any length at any offset."""
    rng = np.random.default_rng(23)
    for trial in range(40):
        nmsg = int(rng.integers(1, 300))
        nseg = [int(x) for x in rng.choice([1, 1, 1, 2, 3, 9, 40, 200], size=nmsg)]
        full = [(m, k) for m in range(nmsg) for k in range(nseg[m] - 1)]
        last = [(m, nseg[m] - 1) for m in range(nmsg)]
        order = rng.permutation(nmsg)
        # classes: full segments in one region (runs contiguous), last ones elsewhere,
        # shuffled among themselves (LDS-atomic claim order)
        entries, firstk, want = [], {}, []
        for m in order:
            for k in range(nseg[m] - 1):
                pos = len(entries)
                entries.append(int(m))
                if pos % 64 == 0:
                    firstk[pos >> 6] = k
                want.append((int(m), k))
        for j in rng.permutation(len(last)):
            m, k = last[j]
            entries.append(int(m) | 0x80000000)
            want.append((int(m), None))
        got = _decode_groups(entries, firstk)
        assert got == want
        assert len(full) + len(last) == len(entries)


def last_class_nl(off_lo, ln, seg, ra_lines=1):
    """msg_segments' 32-bit line count of a message's last segment (the
    planner's size class input): from the message's offset in its line and
    the segment's length only."""
    nseg = (ln - 1) // seg + 1
    k = nseg - 1
    s0 = off_lo & 127
    s = 0 if k else s0
    d = (ln - k * seg + s0) if k else ln
    dn = 4 if (k == 0 and d < 4) else d
    pe = (s + dn + 15) & ~15
    nl_r = (pe - (s & ~15) + 127) >> 7
    nl_l = (s + dn + 127) >> 7
    return nl_r if (nl_r < nl_l or nl_r <= ra_lines) else nl_l


def test_last_segment_class():
    """The planner's 32-bit last-segment line count equals seg_geom's (geom)
    for the last segment, over random offsets (any 64-bit address), lengths
    and segment sizes, including lengths near 2^32."""
    rng = np.random.default_rng(11)
    cases = []
    for seg in (256, 384, 2048, 16384, 65536, 1 << 30):
        for _ in range(400):
            off = int(rng.integers(0, 1 << 40))
            ln = int(rng.choice([rng.integers(1, 8), rng.integers(1, 4 * seg + 300),
                                 rng.integers((1 << 32) - 4096, 1 << 32)]))
            cases.append((off, ln, seg))
    for off, ln, seg in cases:
        nseg = (ln - 1) // seg + 1
        k = nseg - 1
        S = off if k == 0 else ((off + k * seg) & ~127)
        E = off + ln
        _, nl = geom(S, E, k == 0)
        assert last_class_nl(off & 0xFFFFFFFF, ln, seg) == nl, (off, ln, seg)



def _find_msg_group(first, n, s0, lane_segs):
    """Python restatement of k_fold's find_msg_group (crc32c_kernels.hip):
    one search for the group's first segment s0, then the window of the next
    64 messages' first segments and a 6-step search per lane; a lane past the
    window searches on its own.  first[i] = exclusive prefix of segment
    counts (message i's first segment), len n."""
    import bisect
    m0 = bisect.bisect_right(first, s0) - 1           # last i with first[i] <= s0
    w = [first[m0 + j] if m0 + j < n else 0xFFFFFFFF for j in range(64)]
    w64 = first[m0 + 64] if m0 + 64 < n else 0xFFFFFFFF
    out = []
    for seg in lane_segs:
        j = 0
        for st in (32, 16, 8, 4, 2, 1):
            if w[j + st] <= seg:
                j += st
        msg, f = m0 + j, w[j]
        if j == 63 and w64 <= seg:
            msg = bisect.bisect_right(first, seg) - 1
            f = first[msg]
        out.append((msg, seg - f))
    return out


@pytest.mark.parametrize("seed", range(6))
def test_group_search_maps_every_segment(seed):
    """The given-up map's segment search (round 4) against a brute-force map
    over batches with empty messages (zero segments) in runs, long messages
    and groups spanning more than 64 messages."""
    rng = np.random.default_rng(seed)
    n = 3000
    kinds = rng.integers(0, 4, size=n)
    segs = np.where(kinds == 0, 0, np.where(kinds == 1, 1, rng.integers(1, 90, size=n)))
    if seed % 2:
        segs[100:400] = 0                               # a long run of empty messages
    first = np.concatenate([[0], np.cumsum(segs)[:-1]]).astype(np.int64).tolist()
    total = int(segs.sum())
    owner = np.repeat(np.arange(n), segs)
    kidx = np.concatenate([np.arange(s) for s in segs if s]) if total else np.zeros(0, int)
    for g in range((total + 63) // 64):
        lanes = [s for s in range(64 * g, min(64 * g + 64, total))]
        got = _find_msg_group(first, n, 64 * g, lanes)
        assert got == [(int(owner[s]), int(kidx[s])) for s in lanes], g


def _claim_group(k, b, nbk, wpb, snake=True):
    """k_fold's claim k of block b (crc32c_kernels.hip, gid): chunks of wpb
    adjacent groups, one per block and round, blocks reversed in odd rounds."""
    r = k // wpb
    bb = nbk - 1 - b if snake and r % 2 else b
    return (bb + nbk * r) * wpb + k % wpb


@pytest.mark.parametrize("ngroups,nbk,wpb", [(1, 256, 8), (2047, 256, 8), (2048, 256, 8),
                                             (16384, 256, 8), (777, 37, 4), (5000, 512, 4)])
def test_claims_cover_every_group_once(ngroups, nbk, wpb):
    """Every group is claimed by exactly one (block, k), and a block's claims
    grow with k, so its first claim past the batch ends its loop (the main
    loop and the speculative second pass stop there)."""
    seen = []
    for b in range(nbk):
        prev = -1
        for k in range(ngroups + 2 * wpb):
            g = _claim_group(k, b, nbk, wpb)
            assert g > prev
            prev = g
            if g >= ngroups:
                break
            seen.append(g)
    assert sorted(seen) == list(range(ngroups))


def _long_runs_flat(nf, lpos, short=16):
    """k_plan_map's flattened long-run writes (BMQCRC_LONG_FLAT,
    crc32c_kernels.hip phase 2): runs of more than `short` full segments laid
    out from lpos in (lane, v) order; head and tail entries (the partial
    groups at either end) as one item list, whole groups as another, each
    walked 64 items at a time with a mark at each run's first item and an
    inclusive max-scan.  Returns ({slot: (run, k)}, {group: (run, firstk)})."""
    runs, p = [], lpos
    for x in nf:
        n = x if x > short else 0
        gf, ge = (p + 63) >> 6, (p + n) >> 6
        whole = gf < ge
        ni = (64 * gf - p) + (p + n - 64 * ge) if whole else n
        runs.append((p, n, ni, ge - gf if whole else 0))
        p += n

    def flat(counts, body):
        starts, s = [], 0
        for c in counts:
            starts.append(s if c else None)
            s += c
        total, open_ = s, 0
        for j0 in range(0, total, 64):
            mark = [0] * 64
            for q, st in enumerate(starts):
                if st is not None and 0 <= st - j0 < 64:
                    mark[st - j0] = q + 1
            scan = np.maximum.accumulate(mark).tolist()
            for lane in range(64):
                o = max(scan[lane], open_)
                if j0 + lane < total:
                    q = o - 1
                    body(q, j0 + lane - starts[q])
            open_ = max(scan[63], open_)

    ent, grp = {}, {}

    def put_entry(q, e):
        at, n = runs[q][0], runs[q][1]
        gf, ge = (at + 63) >> 6, (at + n) >> 6
        h = 64 * gf - at if gf < ge else n
        slot = at + e if e < h else 64 * ge + (e - h)
        assert slot not in ent
        ent[slot] = (q, slot - at)

    def put_group(q, e):
        at = runs[q][0]
        g = ((at + 63) >> 6) + e
        assert g not in grp
        grp[g] = (q, 64 * g - at)

    flat([r[2] for r in runs], put_entry)
    flat([r[3] for r in runs], put_group)
    return ent, grp


@pytest.mark.parametrize("seed", range(6))
def test_long_runs_flat_cover_every_segment(seed):
    """Every full segment of every long run is written exactly once: as an
    entry (message, k) at its slot, or inside a whole group described by one
    descriptor whose firstk is the group's first k -- against a brute-force
    expansion; runs aligned to groups (no entries), runs inside one group and
    runs spanning many."""
    rng = np.random.default_rng(seed)
    nf = rng.choice([0, 3, 17, 40, 63, 64, 65, 128, 200, 1000], size=256).tolist()
    lpos = int(rng.integers(0, 64)) if seed else 0
    if seed == 1:
        nf = [64] * 256                                   # every run group-aligned
    ent, grp = _long_runs_flat(nf, lpos)
    want, p = {}, lpos
    for q, x in enumerate(nf):
        if x > 16:
            for k in range(x):
                want[p + k] = (q, k)
            p += x
    got = dict(ent)
    for g, (q, k0) in grp.items():
        for lane in range(64):
            assert 64 * g + lane not in got
            got[64 * g + lane] = (q, k0 + lane)
    assert got == want


def _long_runs_records(nf, lpos, short=16):
    """k_plan_map's long runs with run records (round 6, BMQCRC_RUN_RECORDS):
    whole groups as descriptors, a run's head (the last lanes of its first
    group) as that group's suffix record, its tail (the first lanes of its
    last group) as the prefix record with firstk, entries only for a run
    inside one group touching neither end.  Returns (entries {slot: (run,
    k)}, groups {g: (run, firstk)}, prefix {g: (run, lanes, firstk)}, suffix
    {g: (run, lanes)})."""
    ent, grp, pre, suf = {}, {}, {}, {}
    p = lpos
    for q, x in enumerate(nf):
        n = x if x > short else 0
        if n:
            gf, ge = (p + 63) >> 6, (p + n) >> 6
            for g in range(gf, ge):
                assert g not in grp
                grp[g] = (q, 64 * g - p)
            hb, tb, ho, te = p >> 6, (p + n - 1) >> 6, p & 63, (p + n) & 63
            if hb == tb and ho and te:
                for k in range(n):
                    assert p + k not in ent
                    ent[p + k] = (q, k)
            if ho and (hb < tb or te == 0):
                assert hb not in suf
                suf[hb] = (q, 64 - ho)
            if te and (hb < tb or ho == 0):
                assert tb not in pre
                pre[tb] = (q, te, 64 * tb - p)
        p += n
    return ent, grp, pre, suf


@pytest.mark.parametrize("seed", range(8))
def test_run_records_cover_every_segment(seed):
    """Every full segment of every long run resolves to its (run, k) exactly
    once the way k_fold reads the map (a group descriptor first, then the
    prefix record, then the suffix record, else the entry; k of a prefix lane
    = firstk + lane, of a suffix lane = lane - (64 - lanes)), no record
    overlaps another or a group descriptor, and every side of a group has at
    most one owner -- runs aligned to groups, inside one group (touching an
    end or not) and spanning many."""
    rng = np.random.default_rng(100 + seed)
    nf = rng.choice([0, 3, 17, 30, 40, 47, 63, 64, 65, 100, 128, 200, 1000], size=300).tolist()
    lpos = int(rng.integers(0, 64)) if seed else 0
    if seed == 1:
        nf = [64] * 100
    if seed == 2:
        nf = [17 + int(i) for i in rng.integers(0, 47, size=300)]  # many runs inside one group
    ent, grp, pre, suf = _long_runs_records(nf, lpos)
    want, p = {}, lpos
    for q, x in enumerate(nf):
        if x > 16:
            for k in range(x):
                want[p + k] = (q, k)
            p += x
    got = {}
    for slot in want:
        g, lane = slot >> 6, slot & 63
        if g in grp:
            q, k0 = grp[g]
            r = (q, k0 + lane)
        elif g in pre and lane < pre[g][1]:
            q, _, k0 = pre[g]
            r = (q, k0 + lane)
        elif g in suf and lane >= 64 - suf[g][1]:
            q, h = suf[g]
            r = (q, lane - (64 - h))
        else:
            r = ent[slot]
        got[slot] = r
    assert got == want
    for g, (q, t, _) in pre.items():
        assert g not in grp and (g not in suf or t <= 64 - suf[g][1])
    for slot in ent:
        g, lane = slot >> 6, slot & 63
        assert g not in grp
        assert not (g in pre and lane < pre[g][1]) and not (g in suf and lane >= 64 - suf[g][1])
