#!/usr/bin/env python3
"""Derive the GF(2) constants the CRC32C kernels use, with self-checks.

Writes ``blazingmq_amd/csrc/crc32c_consts.h``.  Everything here is plain
polynomial arithmetic over GF(2) for the Castagnoli polynomial
P(x) = x^32 + 0x1EDC6F41 (reflected form 0x82F63B78), the polynomial that
``bmqp::Crc32c`` (``/root/reference/src/groups/bmq/bmqp/bmqp_crc32c.h:225``)
computes through BDE's ``bdlde::Crc32c``.

Constants produced:

* ``REL_TAPS``: the exponents k < 32 of the minimal polynomial of
  y = x^32 mod P,  m(y) = y^32 + sum_{k in REL_TAPS} y^k.  Because
  m(x^32) == 0 (mod P), a stream of 32-bit words can be reduced modulo m(y)
  with XORs of whole words only (no carry-less multiply per word): the
  "table-less fold" of the device kernel.
* ``YCOL[32]``: columns of the 32x32 GF(2) matrix "multiply by y mod P" in the
  reflected register convention (bit t of a register <-> x^(31-t)).
* ``X2COL[31][32]``: columns of "multiply by x^(2^j) mod P", j = 0..30, used to
  apply x^e for any exponent e mod ord(x) = 2^31 - 1 (P = (x+1) * primitive
  degree-31 factor, checked below).
* ``XBYTES[4][256]``: x^(8 * b * 256^i) mod P, the factor that moves a CRC
  past b * 256^i zero bytes; a segment's move to its message end multiplies
  the factors of the bytes of its distance (k_fold).
* ``TY[8][256]``: byte-sliced "multiply by y" and "by y^2" tables for the
  remainder reduction of 4-wave k_fold blocks (two words per Horner step).
* ``RTAB11[6144]``: the same reduction in three 11/11/10-bit slices (one word
  per step, two 16-word chains) plus the byte tables of the join by y^16,
  for the 8-wave blocks: 3 lookups per word instead of 4.
"""
import os
import sys

P_NORMAL = (1 << 32) | 0x1EDC6F41
POLY_R = 0x82F63B78
ORD = (1 << 31) - 1


def pmod(a, m):
    dm = m.bit_length() - 1
    while a and a.bit_length() - 1 >= dm:
        a ^= m << (a.bit_length() - 1 - dm)
    return a


def pmul(a, b):
    r = 0
    while b:
        if b & 1:
            r ^= a
        a <<= 1
        b >>= 1
    return r


def ppow(a, e, m):
    r, a = 1, pmod(a, m)
    while e:
        if e & 1:
            r = pmod(pmul(r, a), m)
        a = pmod(pmul(a, a), m)
        e >>= 1
    return r


def mulmod_r(a, b):
    """a*b mod P with both operands in the reflected convention."""
    p, m = 0, 1 << 31
    while m:
        if a & m:
            p ^= b
        b = (b >> 1) ^ (POLY_R if b & 1 else 0)
        m >>= 1
    return p


def columns(const_r):
    """Columns of v -> v*const mod P (reflected): col[t] = (1<<t) * const."""
    return [mulmod_r(1 << t, const_r) for t in range(32)]


def min_poly_of_y():
    y = ppow(2, 32, P_NORMAL)
    basis = {}
    for k in range(33):
        v, combo = ppow(y, k, P_NORMAL), 1 << k
        for bit in sorted(basis, reverse=True):
            if (v >> bit) & 1:
                bv, bc = basis[bit]
                v ^= bv
                combo ^= bc
        if v == 0:
            return [j for j in range(k + 1) if (combo >> j) & 1]
        basis[v.bit_length() - 1] = (v, combo)
    raise AssertionError("no relation")


def remainder_tables11():
    """11-bit remainder tables (two 16-word chains, k_fold's 8-wave blocks):
    [0][i] = (i << 2) * y, [1][i] = (i << 13) * y (2048 entries each: word
    bits 2-12 and 13-23), [2][i] = (((i & 0xff) << 24) | (i >> 8)) * y (1024:
    bits 24-31 and 0-1), then the join y^16: [k][b] = (b << 8k) * y^16; one
    flat list of 6144 words, self-checked."""
    one_r = 1 << 31
    x32_r = one_r
    for _ in range(32):
        x32_r = mulmod_r(x32_r, 1 << 30)
    y16_r = one_r
    for _ in range(16):
        y16_r = mulmod_r(y16_r, x32_r)
    t11 = ([mulmod_r(i << 2, x32_r) for i in range(2048)] +
           [mulmod_r(i << 13, x32_r) for i in range(2048)] +
           [mulmod_r(((i & 0xff) << 24) | (i >> 8), x32_r) for i in range(1024)] +
           [mulmod_r(b << (8 * k), y16_r) for k in range(4) for b in range(256)])
    assert len(t11) == 6144
    # the three fields cover every bit of a word once: T0 ^ T1 ^ T2 = v * y
    for v in (0, 1, 0x80000000, 0xdeadbeef, 0x12345678, 0xffffffff):
        got = (t11[(v >> 2) & 0x7ff] ^ t11[2048 + ((v >> 13) & 0x7ff)] ^
               t11[4096 + (((v >> 24) & 0xff) | ((v & 3) << 8))])
        assert got == mulmod_r(v, x32_r)
        j = 0
        for k in range(4):
            j ^= t11[5120 + 256 * k + ((v >> (8 * k)) & 0xff)]
        assert j == mulmod_r(v, y16_r)
    return t11


def main(out_path):
    # P = (x+1) * Q31, Q31 primitive (2^31-1 is prime) -> ord(x) = 2^31-1.
    assert pmod(P_NORMAL, 0b11) == 0
    assert ppow(2, ORD, P_NORMAL) == 1 and ppow(2, 1, P_NORMAL) != 1
    terms = min_poly_of_y()
    assert terms[-1] == 32 and terms[0] == 0
    taps = [k for k in terms if k < 32]
    # check relation: sum y^k == 0
    acc = 0
    for k in terms:
        acc ^= ppow(2, 32 * k, P_NORMAL)
    assert acc == 0
    x1_r = 1 << 30                      # reflected x^1
    one_r = 1 << 31                     # reflected 1
    assert mulmod_r(one_r, x1_r) == x1_r
    x32_r = one_r
    for _ in range(32):
        x32_r = mulmod_r(x32_r, x1_r)
    ycol = columns(x32_r)
    x2 = [x1_r]
    for _ in range(30):
        x2.append(mulmod_r(x2[-1], x2[-1]))
    x2col = [columns(c) for c in x2]
    # x^(-8p) mod P, p = 0..135: un-shift of the zero padding after a segment end
    def xpow_r(e):
        r, sq = one_r, x1_r
        while e:
            if e & 1:
                r = mulmod_r(r, sq)
            sq = mulmod_r(sq, sq)
            e >>= 1
        return r
    xneg = [xpow_r((ORD - (8 * p) % ORD) % ORD) for p in range(136)]
    for p in range(136):
        assert mulmod_r(xneg[p], xpow_r(8 * p)) == one_r
    # byte-indexed move factors: XB[i][b] = x^(8 * b * 256^i)
    xb = [[xpow_r((8 * b * 256 ** i) % ORD) for b in range(256)] for i in range(4)]
    for dist in (0, 1, 255, 256, 4095, 65537, 1 << 20, (1 << 32) - 1, 0x12345678):
        f_ = one_r
        for i in range(4):
            f_ = mulmod_r(f_, xb[i][(dist >> (8 * i)) & 0xff])
        assert f_ == xpow_r((8 * dist) % ORD)
    # slicing tables for the remainder reduction: TY[k][b] = (b << 8(k%4)) * y^(1 + k//4)
    y2_r = mulmod_r(x32_r, x32_r)
    ty = [[mulmod_r(b << (8 * (k % 4)), x32_r if k < 4 else y2_r) for b in range(256)]
          for k in range(8)]
    t11 = remainder_tables11()
    with open(out_path, "w") as f:
        f.write("// GENERATED by tools/gen_crc_consts.py -- do not edit.\n")
        f.write("#pragma once\n#include <stdint.h>\n\n")
        f.write("// minimal polynomial of y = x^32 mod P: y^32 + sum y^k, k in REL_TAPS\n")
        f.write("#define BMQCRC_REL_NTAPS %d\n" % len(taps))
        f.write("#define BMQCRC_REL_TAPS {%s}\n\n" % ", ".join(str(k) for k in taps))
        f.write("// columns of v -> v * x^32 mod P (reflected)\n")
        f.write("#define BMQCRC_YCOL {%s}\n\n" % ", ".join("0x%08xu" % c for c in ycol))
        f.write("// columns of v -> v * x^(2^j) mod P (reflected), j = 0..30\n")
        f.write("#define BMQCRC_X2COL { \\\n")
        for j, cols in enumerate(x2col):
            f.write("  {%s}%s \\\n" % (", ".join("0x%08xu" % c for c in cols), "," if j < 30 else ""))
        f.write("}\n\n#define BMQCRC_ORD 0x7fffffffu\n\n")
        f.write("// x^(-8p) mod P (reflected), p = 0..135\n")
        f.write("#define BMQCRC_XNEG8 {%s}\n\n" % ", ".join("0x%08xu" % c for c in xneg))
        f.write("// move factors: [i][b] = x^(8 * b * 256^i) mod P (reflected)\n")
        f.write("#define BMQCRC_XBYTES { \\\n")
        for i in range(4):
            f.write("  {%s}%s \\\n" % (", ".join("0x%08xu" % c for c in xb[i]), "," if i < 3 else ""))
        f.write("}\n\n")
        f.write("// remainder-reduction tables: [k][b] = (b << 8*(k%4)) * x^(32*(1+k/4)) mod P\n")
        f.write("#define BMQCRC_TY { \\\n")
        for k in range(8):
            f.write("  {%s}%s \\\n" % (", ".join("0x%08xu" % c for c in ty[k]), "," if k < 7 else ""))
        f.write("}\n\n")
        f.write("// 11-bit remainder tables and the y^16 join (6144 words, see gen_crc_consts.py)\n")
        f.write("#define BMQCRC_RTAB11 { \\\n")
        for i in range(0, 6144, 8):
            f.write("  %s%s \\\n" % (", ".join("0x%08xu" % c for c in t11[i:i + 8]),
                                    "," if i + 8 < 6144 else ""))
        f.write("}\n")
    print("wrote", out_path, "taps", taps)


if __name__ == "__main__":
    here = os.path.dirname(os.path.abspath(__file__))
    main(sys.argv[1] if len(sys.argv) > 1 else
         os.path.join(here, "..", "blazingmq_amd", "csrc", "crc32c_consts.h"))
