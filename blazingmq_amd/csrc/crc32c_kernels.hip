// crc32c_kernels.hip -- MI355X (gfx950) batched CRC32C.
//
// Replaces, for batches, the arithmetic behind
//   bmqp::Crc32c::calculate(const void*, unsigned, unsigned)
//   (/root/reference/src/groups/bmq/bmqp/bmqp_crc32c.cpp:41-45 -> BDE
//   bdlde::Crc32c::calculate) with bit-exact CRC-32C (Castagnoli).
//
// Design (DESIGN.md sections 2-4):
//   * A message is cut into segments of <= seg_bytes; one LANE owns one
//     segment and folds it serially as a stream of 32-bit words.
//   * The fold is table-less: the minimal polynomial of y = x^32 mod P,
//     m(y) = y^32 + sum_{k in REL_TAPS} y^k, vanishes mod P, so the word
//     stream is reduced modulo m(y) by a 17-tap Fibonacci recurrence over a
//     32-word register ring -- 6 VALU per word (seven adjacent tap pairs come
//     from a second ring of pair XORs), no carry-less multiply, no lookup
//     table.
//   * Only the last 32 remainder words get a real GF(2) reduction (Horner by
//     x^32 with slicing tables in LDS), once per segment.
//   * Bytes reach the lanes through LDS: per round a wave DMAs (LDS-DMA,
//     global_load_lds_dwordx4) the next 128-byte line of each of its 64
//     segments, 8 lanes per full 128-byte line (coalesced), with the piece
//     order XOR-swizzled on the SOURCE address so that every owner lane's
//     ds_read_b128 is bank-conflict free.  Pieces outside a segment's bytes
//     are read from a zero line instead, so only the 16-byte pieces cut by a
//     segment's first or last byte need a byte mask (a few LDS
//     read-modify-writes).  Two LDS slots per wave: round r+1 is in flight
//     while round r folds.
//   * Streams are right-aligned in the wave: a lane with nl lines starts at
//     round R - nl (R = the wave's longest stream) and folds zero lines
//     before that, which leaves a zero-init CRC unchanged.  Every lane thus
//     ends in round R-1 and the remainder reduction runs once per wave, not
//     once per distinct segment length.
//   * Per-segment raw remainders are moved to the message end with x^e mod P
//     (e mod ord(x) = 2^31-1, which also un-shifts the zero padding) and
//     XOR-combined into out[msg] (plain store for single-segment messages,
//     global atomic XOR otherwise -- XOR is order independent, so results are
//     deterministic).  The seed enters as ~seed XORed into the message's
//     first 4 bytes; the final inversion is one XOR with 0xFFFFFFFF.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "bmqcrc_internal.h"
#include "crc32c_consts.h"

namespace bmqcrc {

typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const u32x4 lds_cu4;
typedef __attribute__((address_space(3))) u32x4 lds_u4;
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
// element-aligned vectors: one dwordx4 access at any dword-aligned address
typedef uint32_t u32x4e __attribute__((ext_vector_type(4), aligned(4)));
typedef uint64_t u64x2e __attribute__((ext_vector_type(2), aligned(8)));

__constant__ uint32_t c_x2col[31][32] = BMQCRC_X2COL;
__constant__ uint32_t c_xneg8[136] = BMQCRC_XNEG8;
__constant__ uint32_t c_xbytes[4][256] = BMQCRC_XBYTES;
__constant__ uint32_t c_ty[8][256] = BMQCRC_TY;
__constant__ uint32_t c_rtab11[6144] = BMQCRC_RTAB11;

// All-zero line in device memory: the LDS-DMA source of every 16-byte piece
// that lies outside a segment's bytes, and of every round outside its stream.
__device__ __attribute__((aligned(128))) uint8_t g_zero_line[128];

// ------------------------------------------------------------ GF(2) helpers
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // a ^ b ^ c
}

__device__ __forceinline__ uint32_t xand(uint32_t acc, uint32_t mask, uint32_t col)
{
    return __builtin_amdgcn_bitop3_b32(acc, mask, col, 0x78);  // acc ^ (mask & col)
}

__device__ __forceinline__ uint32_t bitmask(uint32_t v, int t)
{
    return (uint32_t)__builtin_amdgcn_sbfe((int)v, t, 1);  // 0 or ~0
}

// v * x^32 mod P (reflected), 64 VALU.
__device__ __forceinline__ uint32_t mul_y(uint32_t v)
{
    constexpr uint32_t col[32] = BMQCRC_YCOL;
    uint32_t a0 = 0, a1 = 0;
#pragma unroll
    for (int t = 0; t < 32; t += 2) {
        a0 = xand(a0, bitmask(v, t), col[t]);
        a1 = xand(a1, bitmask(v, t + 1), col[t + 1]);
    }
    return a0 ^ a1;
}

// v * x^e mod P (reflected), e in [0, 2^31-1).  Column tables are uniform
// (scalar loads); bits no lane needs are skipped wave-uniformly.
__device__ uint32_t mul_xpow(uint32_t v, uint32_t e)
{
    if (__ballot(e != 0) == 0) {
        return v;
    }
    for (int j = 0; j < 31; ++j) {
        const bool bit = (e >> j) & 1u;
        if (__ballot(bit) == 0) {
            continue;
        }
        uint32_t a0 = 0, a1 = 0;
#pragma unroll
        for (int t = 0; t < 32; t += 2) {
            a0 = xand(a0, bitmask(v, t), c_x2col[j][t]);
            a1 = xand(a1, bitmask(v, t + 1), c_x2col[j][t + 1]);
        }
        v = bit ? (a0 ^ a1) : v;
    }
    return v;
}

// v * w mod P (reflected), both variable: 32 shift-and-add steps, 160 VALU.
__device__ __forceinline__ uint32_t gmul(uint32_t v, uint32_t w)
{
    uint32_t acc = 0;
#pragma unroll
    for (int t = 31; t >= 0; --t) {  // bit t of v <-> x^(31-t); w tracks w * x^(31-t)
        acc = xand(acc, bitmask(v, t), w);
        w = xand(w >> 1, bitmask(w, 0), 0x82F63B78u);
    }
    return acc;
}

#ifndef BMQCRC_XB_FIRST
#define BMQCRC_XB_FIRST 1  // 0: the move factor's product starts with byte 0's factor (A/B)
#endif
constexpr bool kXbFirst = BMQCRC_XB_FIRST != 0;
#ifndef BMQCRC_SPREAD
#define BMQCRC_SPREAD 1  // 0: small batches fill 4-wave blocks on fewer CUs (A/B)
#endif
constexpr bool kSpread = BMQCRC_SPREAD != 0;

// v * x^(8 dist) mod P: the move of a CRC past dist zero bytes, as the
// product of the factors of dist's bytes (tables XBYTES[i][b] = x^(8 b 256^i)
// in LDS at xb): one lookup per byte position any lane needs and one 160-VALU
// multiply per factor, against one 64-VALU column pass per exponent bit.
__device__ __forceinline__ uint32_t mul_xbytes(uint32_t v, uint32_t dist, uint32_t xb)
{
    if (__ballot(dist != 0) == 0) {
        return v;
    }
    // the first byte position any lane needs starts the product (a lane whose
    // byte there is 0 looks up x^0 = 1): one 160-VALU multiply fewer than
    // starting from byte 0, whose factor is 1 in every lane when the
    // distances are multiples of 256 (uniform messages, segment moves)
    if constexpr (!kXbFirst) {  // A/B: round 4's form
        uint32_t f = *(const lds_u32*)(uintptr_t)(xb + 4u * (dist & 0xffu));
#pragma unroll
        for (int i = 1; i < 4; ++i) {
            if (__ballot((dist >> (8 * i)) != 0) != 0) {
                f = gmul(f, *(const lds_u32*)(uintptr_t)(xb + 1024u * i + 4u * ((dist >> (8 * i)) & 0xffu)));
            }
        }
        return gmul(v, f);
    }
    uint32_t f = 0;
    bool have = false;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (__ballot(((dist >> (8 * i)) & 0xffu) != 0) != 0) {
            const uint32_t t = *(const lds_u32*)(uintptr_t)(xb + 1024u * i + 4u * ((dist >> (8 * i)) & 0xffu));
            f = have ? gmul(f, t) : t;
            have = true;
        }
    }
    return gmul(v, f);
}

__device__ __forceinline__ uint32_t mersenne31(uint64_t x)
{
    // x mod (2^31 - 1)
    x = (x & 0x7fffffffull) + (x >> 31);
    x = (x & 0x7fffffffull) + (x >> 31);
    x = (x & 0x7fffffffull) + (x >> 31);
    return (x >= 0x7fffffffull) ? (uint32_t)(x - 0x7fffffffull) : (uint32_t)x;
}

// Wave-wide maximum by DPP (no LDS round trips): row_shr 1/2/4/8 leaves each
// row's maximum in its lane 15, row_bcast 15/31 carries it across rows, lane
// 63 ends with the wave's maximum.  Lanes without a source keep their own
// value (old = v), which a maximum ignores.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp_max(uint32_t v)
{
    return max(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, CTRL, ROW_MASK, 0xf,
                                                        false));
}

// (the same steps leave lane l with the maximum of lanes 0..l: an inclusive
// max-scan)
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v)
{
    v = dpp_max<0x111, 0xf>(v);  // row_shr:1
    v = dpp_max<0x112, 0xf>(v);  // row_shr:2
    v = dpp_max<0x114, 0xf>(v);  // row_shr:4
    v = dpp_max<0x118, 0xf>(v);  // row_shr:8
    v = dpp_max<0x142, 0xa>(v);  // row_bcast:15 -> rows 1, 3
    v = dpp_max<0x143, 0xc>(v);  // row_bcast:31 -> rows 2, 3
    return v;
}

__device__ __forceinline__ uint32_t wave_max(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_max(v), 63);
}

// Inclusive prefix sum over the wave's 64 lanes by DPP (all lanes active):
// row_shr 1/2/4/8 scan each row of 16, row_bcast 15/31 carry the row totals.
// Lanes without a source add old = 0.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp_add(uint32_t v)
{
    return v + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROW_MASK, 0xf, false);
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v)
{
    v = dpp_add<0x111, 0xf>(v);  // row_shr:1
    v = dpp_add<0x112, 0xf>(v);  // row_shr:2
    v = dpp_add<0x114, 0xf>(v);  // row_shr:4
    v = dpp_add<0x118, 0xf>(v);  // row_shr:8
    v = dpp_add<0x142, 0xa>(v);  // row_bcast:15 -> rows 1, 3
    v = dpp_add<0x143, 0xc>(v);  // row_bcast:31 -> rows 2, 3
    return v;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(v), 63);
}

// 64-bit wave sum of per-lane values below 2^38 (two 32-bit scans)
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v)
{
    return ((uint64_t)wave_sum((uint32_t)(v >> 16)) << 16) + wave_sum((uint32_t)v & 0xffffu);
}

template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp_min(uint32_t v)
{
    return min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, CTRL, ROW_MASK, 0xf,
                                                        false));
}

__device__ __forceinline__ uint32_t wave_min(uint32_t v)
{
    v = dpp_min<0x111, 0xf>(v);
    v = dpp_min<0x112, 0xf>(v);
    v = dpp_min<0x114, 0xf>(v);
    v = dpp_min<0x118, 0xf>(v);
    v = dpp_min<0x142, 0xa>(v);
    v = dpp_min<0x143, 0xc>(v);
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src)
{
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src);
    return ((uint64_t)hi << 32) | lo;
}

// ---------------------------------------------------- fold ring (m(y) taps)
constexpr int kTaps[BMQCRC_REL_NTAPS] = BMQCRC_REL_TAPS;
constexpr int kNTaps = BMQCRC_REL_NTAPS;

// One full round = 32 words = one turn of the ring.  Ring slot d holds the
// quotient word Q_i of the latest stream index i == d (mod 32):
//   Q_i = m_i ^ sum_{k in taps} Q_{i-32+k}
// Slot (d+k)&31 is still the previous round's word when d+k < 32 and this
// round's when d+k >= 32, exactly the recurrence.
//
// Seven tap pairs are adjacent (k, k+1); a second ring p holds
// p[j] = Q_m ^ Q_{m+1} for the latest such m == j (mod 32), updated once per
// word, so a word costs one pair update + 5 three-input XORs (m, 7 pairs,
// 3 single taps) instead of 9.
constexpr int kPairs[7] = {8, 10, 13, 18, 22, 25, 27};
constexpr int kSingles[3] = {0, 6, 20};

constexpr bool pairs_cover_taps()
{
    int n = 0;
    for (int k = 0; k < 32; ++k) {
        bool in_taps = false, covered = false;
        for (int i = 0; i < kNTaps; ++i) {
            in_taps = in_taps || kTaps[i] == k;
        }
        for (int i = 0; i < 3; ++i) {
            covered = covered || kSingles[i] == k;
        }
        for (int i = 0; i < 7; ++i) {
            covered = covered || kPairs[i] == k || kPairs[i] + 1 == k;
        }
        n += (in_taps != covered) ? 1 : 0;
    }
    return n == 0 && kNTaps == 3 + 2 * 7;
}
static_assert(pairs_cover_taps(), "tap pairs/singles must be exactly the relation's taps");

__device__ __forceinline__ void fold_round(uint32_t (&q)[32], uint32_t (&p)[32],
                                           const uint32_t (&m)[32])
{
#pragma unroll
    for (int d = 0; d < 32; ++d) {
        uint32_t acc = xor3(m[d], q[(d + kSingles[0]) & 31], q[(d + kSingles[1]) & 31]);
        acc = xor3(acc, q[(d + kSingles[2]) & 31], p[(d + kPairs[0]) & 31]);
        acc = xor3(acc, p[(d + kPairs[1]) & 31], p[(d + kPairs[2]) & 31]);
        acc = xor3(acc, p[(d + kPairs[3]) & 31], p[(d + kPairs[4]) & 31]);
        acc = xor3(acc, p[(d + kPairs[5]) & 31], p[(d + kPairs[6]) & 31]);
        q[d] = acc;
        p[(d + 31) & 31] = q[(d + 31) & 31] ^ acc;
    }
}

// First round of a stream (zero history, so the ring needs no clearing):
// taps that reach the previous round read zero and are dropped at compile
// time; p[31] pairs Q_-1 = 0 with Q_0.
__device__ __forceinline__ void first_round(uint32_t (&q)[32], uint32_t (&p)[32],
                                            const uint32_t (&m)[32])
{
#pragma unroll
    for (int d = 0; d < 32; ++d) {
        uint32_t t[11];
        int nt = 0;
        t[nt++] = m[d];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            if (d + kSingles[i] >= 32) {
                t[nt++] = q[d + kSingles[i] - 32];
            }
        }
#pragma unroll
        for (int i = 0; i < 7; ++i) {
            if (d + kPairs[i] >= 31) {  // Q_(d+k-32) ^ Q_(d+k-31), Q_-1 = 0
                t[nt++] = p[(d + kPairs[i]) & 31];
            }
        }
        uint32_t acc = t[0];
        int i = 1;
#pragma unroll
        for (; i + 1 < nt; i += 2) {
            acc = xor3(acc, t[i], t[i + 1]);
        }
        if (i < nt) {
            acc ^= t[i];
        }
        q[d] = acc;
        p[(d + 31) & 31] = d == 0 ? acc : (q[d - 1] ^ acc);
    }
}

// Final round: the last 32 words are the remainder coefficients R_d of the
// stream modulo m(y).  Taps that would reach this round's (non-existent)
// quotient words are dropped.  The remainder is reduced once per segment,
// raw = sum R_d y^(32-d), by Horner two words per step with slicing tables in
// LDS (tab[k][b], k<4: (b<<8k)*y, k>=4: (b<<8(k-4))*y^2):
//   c <- (c ^ R_d) * y^2  ^  R_{d+1} * y
__device__ __forceinline__ uint32_t tab_lookup(uint32_t tab_lds, int k, uint32_t b)
{
    return *(const lds_u32*)(uintptr_t)(tab_lds + k * 1024u + b * 4u);
}


// The last round's taps into the previous round (d + k <= 31): R_d = m_d ^
// H_d.  A pair (k, k+1) with d + k + 1 <= 31 is p[d + k].
__device__ __forceinline__ void tail_taps(const uint32_t (&q)[32], const uint32_t (&p)[32],
                                          uint32_t (&H)[32])
{
#pragma unroll
    for (int d = 0; d < 32; ++d) {
        uint32_t t[20];
        int nt = 0;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            if (d + kSingles[i] <= 31) {
                t[nt++] = q[d + kSingles[i]];
            }
        }
#pragma unroll
        for (int i = 0; i < 7; ++i) {
            if (d + kPairs[i] + 1 <= 31) {
                t[nt++] = p[d + kPairs[i]];
            } else if (d + kPairs[i] <= 31) {
                t[nt++] = q[d + kPairs[i]];
            }
        }
        uint32_t acc = nt ? t[0] : 0u;
        int i = 1;
#pragma unroll
        for (; i + 1 < nt; i += 2) {
            acc = xor3(acc, t[i], t[i + 1]);
        }
        if (i < nt) {
            acc ^= t[i];
        }
        H[d] = acc;
    }
}

// SKIP: R[0 .. 2 SKIP) is zero in every lane of the wave, so the first SKIP
// steps would leave c = 0 and are not compiled in (one-line groups, whose
// remainder is the line itself: right-aligned messages of at most 64 bytes
// leave 16 leading zero words).  A compile-time count: per-step uniform
// branches cost 2-4 % on two-line groups (profiles/r03/ab/ab2_*.jsonl).
template <int SKIP = 0>
__device__ __forceinline__ uint32_t tail_horner(const uint32_t (&R)[32], uint32_t tab_lds)
{
    uint32_t c = 0;
#pragma unroll
    for (int d = 2 * SKIP; d < 32; d += 2) {
        const uint32_t v = c ^ R[d];
        const uint32_t w = R[d + 1];
        const uint32_t hi = xor3(tab_lookup(tab_lds, 4, v & 0xffu),
                                 tab_lookup(tab_lds, 5, (v >> 8) & 0xffu),
                                 tab_lookup(tab_lds, 6, (v >> 16) & 0xffu));
        const uint32_t lo = xor3(tab_lookup(tab_lds, 0, w & 0xffu),
                                 tab_lookup(tab_lds, 1, (w >> 8) & 0xffu),
                                 tab_lookup(tab_lds, 2, (w >> 16) & 0xffu));
        c = xor3(hi, lo, tab_lookup(tab_lds, 7, v >> 24) ^ tab_lookup(tab_lds, 3, w >> 24));
    }
    return c;
}

// The same reduction with 11-bit slices (k_fold's 8-wave blocks, which have
// the LDS for them: 24 KiB, kTab11Bytes).  One word per step, c <- (c ^ R_d)
// * y, in three lookups (word bits 2-12, 13-23, and 24-31 with 0-1, each
// slice's byte offset formed by one AND, or a shift or rotate and an AND),
// against four per word with byte slices: 100 lookups per segment instead of
// 128, and no more VALU.  Two independent chains keep the dependent depth at
// 16 steps: A over words 0-15, B over 16-31, raw = A * y^16 + B, the join by
// four byte lookups.  SKIP = 8: words 0-15 are zero in every lane (chain A
// and the join drop out).
constexpr uint32_t kTab11Bytes = 6144 * 4;
constexpr uint32_t kT11Hi = 8192, kT11Top = 16384, kT11Join = 20480;  // slice offsets (bytes)

__device__ __forceinline__ uint32_t step11(uint32_t c, uint32_t r, uint32_t tab_lds)
{
    const uint32_t v = c ^ r;
    const uint32_t a0 = v & 0x1ffcu;
    const uint32_t a1 = (v >> 11) & 0x1ffcu;
    const uint32_t a2 = __builtin_amdgcn_alignbit(v, v, 22) & 0xffcu;  // rotr 22: bits 24-31, 0-1
    return xor3(*(const lds_u32*)(uintptr_t)(tab_lds + a0),
                *(const lds_u32*)(uintptr_t)(tab_lds + kT11Hi + a1),
                *(const lds_u32*)(uintptr_t)(tab_lds + kT11Top + a2));
}

template <int SKIP = 0>
__device__ __forceinline__ uint32_t tail_chains11(const uint32_t (&R)[32], uint32_t tab_lds)
{
    static_assert(SKIP == 0 || SKIP == 8, "chain A runs whole or not at all");
    uint32_t ca = 0, cb = 0;
#pragma unroll
    for (int d = 0; d < 16; ++d) {
        if (SKIP == 0) {
            ca = step11(ca, R[d], tab_lds);
        }
        cb = step11(cb, R[16 + d], tab_lds);
    }
    if (SKIP != 0) {
        return cb;
    }
    const uint32_t j = tab_lds + kT11Join;
    return xor3(cb, *(const lds_u32*)(uintptr_t)(j + 4u * (ca & 0xffu)),
                *(const lds_u32*)(uintptr_t)(j + 1024u + 4u * ((ca >> 8) & 0xffu))) ^
           xor3(*(const lds_u32*)(uintptr_t)(j + 2048u + 4u * ((ca >> 16) & 0xffu)),
                *(const lds_u32*)(uintptr_t)(j + 3072u + 4u * (ca >> 24)), 0u);
}

// The 32 remainder words reduced further at BYTE granularity before any
// lookup (BMQCRC_BYTE_FOLD, A/B).  The minimal polynomial of z = x^8 is P
// itself (as for y = x^32: x^8 and x^32 are Frobenius conjugates of x), so the
// remainder's 128 bytes b_i (raw = sum b_i z^(131-i)) reduce with the same 17
// taps at byte lags 32 - k: Q_i = b_i ^ sum_k Q_(i-32+k) for the first 96
// bytes, and the last 32 bytes (words 24-31) are what remains.  Every lag is
// at least 4 bytes, so a word's four bytes are one step: a tap is a word of
// the Q stream at that lag (one v_alignbyte when the lag is not a multiple
// of 4), and the seven adjacent tap pairs come from a pair stream P2_i =
// Q_(i-1) ^ Q_i at lag 31 - k.  About 14 VALU per word; then 8 one-word
// chain steps: 24 lookups per segment instead of 100.  SKIP16: words 0-15
// are zero in every lane (so is their part of Q).
__device__ __forceinline__ uint32_t alignbyte(uint32_t hi, uint32_t lo, int s)
{
    return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)s);
}

// One word per step with the byte-sliced "times y" tables (tab[k][b], k < 4:
// 4-wave blocks' 8 KiB tables, tail_horner's), four lookups.
__device__ __forceinline__ uint32_t step8(uint32_t c, uint32_t r, uint32_t tab_lds)
{
    const uint32_t v = c ^ r;
    return xor3(tab_lookup(tab_lds, 0, v & 0xffu), tab_lookup(tab_lds, 1, (v >> 8) & 0xffu),
                tab_lookup(tab_lds, 2, (v >> 16) & 0xffu)) ^
           tab_lookup(tab_lds, 3, v >> 24);
}

// BYTE_TABLES: the last 8 steps with the byte-sliced tables (4-wave blocks).
template <bool SKIP16, bool BYTE_TABLES = false>
__device__ __forceinline__ uint32_t tail_bytes8(const uint32_t (&R)[32], uint32_t tab_lds)
{
    uint32_t Q[24], P2[25];
    // the word of stream W (Q or P2, zero outside [0, n)) at byte lag L from word j
    auto lagw = [&](const uint32_t* W, int n, int j, int L) -> uint32_t {
        const int q = L >> 2, s = L & 3;
        const int hi = j - q, lo = j - q - 1;
        const uint32_t h = (hi >= 0 && hi < n && !(SKIP16 && hi < 16)) ? W[hi] : 0u;
        if (s == 0) {
            return h;
        }
        const uint32_t l = (lo >= 0 && lo < n && !(SKIP16 && lo < 16)) ? W[lo] : 0u;
        return alignbyte(h, l, 4 - s);
    };
    auto taps = [&](int j, int nq) -> uint32_t {
        // singles k = 0, 6, 20 (lags 32, 26, 12); pairs k = 8, 10, 13, 18, 22,
        // 25, 27 from P2 at lags 23, 21, 18, 13, 9, 6, 4
        uint32_t t = xor3(lagw(Q, nq, j, 32), lagw(Q, nq, j, 26), lagw(Q, nq, j, 12));
        t = xor3(t, lagw(P2, nq + 1, j, 23), lagw(P2, nq + 1, j, 21));
        t = xor3(t, lagw(P2, nq + 1, j, 18), lagw(P2, nq + 1, j, 13));
        t = xor3(t, lagw(P2, nq + 1, j, 9), lagw(P2, nq + 1, j, 6));
        return t ^ lagw(P2, nq + 1, j, 4);
    };
#pragma unroll
    for (int j = 0; j < 24; ++j) {
        if (SKIP16 && j < 16) {
            Q[j] = 0u;
            P2[j] = 0u;
            continue;
        }
        Q[j] = R[j] ^ taps(j, j);
        P2[j] = Q[j] ^ alignbyte(Q[j], j > 0 ? Q[j - 1] : 0u, 3);
    }
    P2[24] = alignbyte(0u, Q[23], 3);  // Q_95 (Q_96 is not a quotient byte)
    uint32_t c = 0;
#pragma unroll
    for (int j = 24; j < 32; ++j) {
        c = BYTE_TABLES ? step8(c, R[j] ^ taps(j, 24), tab_lds)
                        : step11(c, R[j] ^ taps(j, 24), tab_lds);
    }
    return c;
}

// Word w (0..31) of this lane's 128-byte line in an LDS slot (the pieces are
// XOR-swizzled; rd_off is the lane's swizzled line base, see k_fold).
__device__ __forceinline__ lds_u32* line_word(uint32_t slot, uint32_t rd_off, uint32_t w)
{
    return (lds_u32*)(uintptr_t)(slot + (rd_off ^ (16u * (w >> 2))) + 4u * (w & 3u));
}

// Byte-exact edges of a lane's line, fixed in LDS before the line is read
// into registers.  The DMA has already substituted zeros for every 16-byte
// piece outside the segment's bytes [S, E); what remains are the (at most two)
// pieces cut by S or E and the seed word:
//   lo: zero bytes [16*floor(s/16), s) of the line (s = S's offset, s % 16 != 0);
//   hi: zero bytes [e, 16*ceil(e/16))              (e = E's offset, e % 16 != 0);
//   sd: XOR ~seed into bytes [sr, sr+4) (sr in [-3, 127]: the word may begin in
//       the previous line or run into the next one), after the zeroing, so a
//       message shorter than 4 bytes gets its seed over zeros.
// A few LDS read-modify-writes per cut line replace whole-line register masks
// (~170 VALU each, once per distinct cut round of the wave).
__device__ void line_fixup(uint32_t slot, uint32_t rd_off, bool lo, uint32_t s, bool hi,
                           uint32_t e, bool sd, int sr, uint32_t c0)
{
    if (lo) {
        const uint32_t ws = s >> 2;
        for (uint32_t w = (s >> 4) << 2; w < ws; ++w) {
            *line_word(slot, rd_off, w) = 0u;
        }
        if (s & 3u) {
            lds_u32* p = line_word(slot, rd_off, ws);
            *p &= 0xffffffffu << (8u * (s & 3u));
        }
    }
    if (hi) {
        const uint32_t we = e >> 2;
        lds_u32* p = line_word(slot, rd_off, we);
        *p &= (e & 3u) ? (0xffffffffu >> (32u - 8u * (e & 3u))) : 0u;
        for (uint32_t w = we + 1u; w < (((e >> 4) + 1u) << 2); ++w) {
            *line_word(slot, rd_off, w) = 0u;
        }
    }
    if (sd) {
        const int qs = sr >> 2;  // floor
        const uint32_t sh = 8u * ((uint32_t)sr & 3u);
        if (qs >= 0) {
            lds_u32* p = line_word(slot, rd_off, (uint32_t)qs);
            *p ^= c0 << sh;
        }
        if (sh && qs + 1 < 32) {
            lds_u32* p = line_word(slot, rd_off, (uint32_t)(qs + 1));
            *p ^= c0 >> (32u - sh);
        }
    }
}

// Issue one round of LDS-DMA: 8 x global_load_lds_dwordx4 (8 x 1 KiB), each
// covering 8 segments x one full 128-byte line.  M0 = LDS destination.
#define BMQCRC_DMA_ASM(CP)                                                                    \
    "s_waitcnt lgkmcnt(0)\n\t"                                                              \
    "s_mov_b32 %0, m0\n\t"                                                                  \
    "s_mov_b32 m0, %1\n\t"                                                                  \
    "s_nop 0\n\t"                                                                           \
    "global_load_lds_dwordx4 %2, off" CP "\n\t"                                             \
    "s_add_u32 m0, m0, 0x400\n\t"                                                           \
    "s_nop 0\n\t"                                                                           \
    "global_load_lds_dwordx4 %3, off" CP "\n\t"                                             \
    "s_add_u32 m0, m0, 0x400\n\t"                                                           \
    "s_nop 0\n\t"                                                                           \
    "global_load_lds_dwordx4 %4, off" CP "\n\t"                                             \
    "s_add_u32 m0, m0, 0x400\n\t"                                                           \
    "s_nop 0\n\t"                                                                           \
    "global_load_lds_dwordx4 %5, off" CP "\n\t"                                             \
    "s_add_u32 m0, m0, 0x400\n\t"                                                           \
    "s_nop 0\n\t"                                                                           \
    "global_load_lds_dwordx4 %6, off" CP "\n\t"                                             \
    "s_add_u32 m0, m0, 0x400\n\t"                                                           \
    "s_nop 0\n\t"                                                                           \
    "global_load_lds_dwordx4 %7, off" CP "\n\t"                                             \
    "s_add_u32 m0, m0, 0x400\n\t"                                                           \
    "s_nop 0\n\t"                                                                           \
    "global_load_lds_dwordx4 %8, off" CP "\n\t"                                             \
    "s_add_u32 m0, m0, 0x400\n\t"                                                           \
    "s_nop 0\n\t"                                                                           \
    "global_load_lds_dwordx4 %9, off" CP "\n\t"                                             \
    "s_mov_b32 m0, %0\n\t"

// Instruction i carries piece pp_i of segment 8i + lane/8.  The piece's index
// in that segment's stream in round r is 8r - plo[i]; it is read from HBM when
// that index lies in [0, pcnt[i]) (the piece overlaps the segment's bytes) and
// from the zero line otherwise (before the lane's stream starts, after its
// data ends, or a piece wholly outside [S, E)).
template <bool NT>
__device__ __forceinline__ void dma_round(uint32_t lds_dst, const uint64_t (&pbase)[8],
                                          const uint32_t (&plo)[8], const uint32_t (&pcnt)[8],
                                          uint64_t zero, uint32_t r)
{
    uint64_t s[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        s[i] = (8u * r - plo[i] < pcnt[i]) ? pbase[i] + ((uint64_t)r << 7) : zero;
    }
    uint32_t keep;
    if (NT) {
        asm volatile(BMQCRC_DMA_ASM(" nt")
        : "=&s"(keep)
        : "s"(lds_dst), "v"(s[0]), "v"(s[1]), "v"(s[2]), "v"(s[3]), "v"(s[4]), "v"(s[5]),
          "v"(s[6]), "v"(s[7])
        : "memory", "scc");
        return;
    }
    asm volatile(BMQCRC_DMA_ASM("")
        : "=&s"(keep)
        : "s"(lds_dst), "v"(s[0]), "v"(s[1]), "v"(s[2]), "v"(s[3]), "v"(s[4]), "v"(s[5]),
          "v"(s[6]), "v"(s[7])
        : "memory", "scc");
}

// LDS-DMA of whole KiB from global memory (the remainder and un-shift tables
// of the one-segment kernel's prologue): instruction i copies 1 KiB, every
// lane 16 B, to lds_dst + 1024 i.  Lanes outside exec copy nothing.
template <int N>
__device__ __forceinline__ void dma_copy_kib(uint32_t lds_dst, uint64_t src)
{
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const uint64_t s = src + 1024u * (uint32_t)i + 16u * (uint32_t)__lane_id();
        uint32_t keep;
        asm volatile("s_waitcnt lgkmcnt(0)\n\t"
                     "s_mov_b32 %0, m0\n\t"
                     "s_mov_b32 m0, %1\n\t"
                     "s_nop 0\n\t"
                     "global_load_lds_dwordx4 %2, off\n\t"
                     "s_mov_b32 m0, %0\n\t"
                     : "=&s"(keep)
                     : "s"(lds_dst + 1024u * (uint32_t)i), "v"(s)
                     : "memory", "scc");
    }
}

#ifndef BMQCRC_ONE_EARLY
#define BMQCRC_ONE_EARLY 1  // the one-segment kernel issues its first group's loads before its
                            // tables (LDS-DMA'd behind them, one barrier before the first
                            // lookup); 0: tables first, through VGPRs, and a barrier (A/B)
#endif
constexpr bool kOneEarly = BMQCRC_ONE_EARLY == 1;
#ifndef BMQCRC_ROUND_WAIT
#define BMQCRC_ROUND_WAIT 0  // a round's fold first waits for every load issued before it
                             // (the next round landed too, the one after issued once the
                             // line is read); 8: for its own 8 loads only, the next round
                             // still landing while it folds (round 5; A/B)
#endif
constexpr bool kRoundWait0 = BMQCRC_ROUND_WAIT == 0;
#ifndef BMQCRC_DESC_FIRST
#define BMQCRC_DESC_FIRST 1  // the first group's descriptors before the prologue's table loads
                             // (every k_fold); 0: after them (round 5; A/B)
#endif
constexpr bool kDescFirst = BMQCRC_DESC_FIRST != 0;

#ifndef BMQCRC_GROUP_DESC
#define BMQCRC_GROUP_DESC 1  // 0: every seginfo entry written (round 3; A/B)
#endif
constexpr bool kGroupDesc = BMQCRC_GROUP_DESC != 0;
#ifndef BMQCRC_LONG_FLAT
#define BMQCRC_LONG_FLAT 1  // long runs' entries and descriptors: 1 flattened over the wave, 0 run by run
#endif
#ifndef BMQCRC_RUN_RECORDS
#define BMQCRC_RUN_RECORDS 1  // a long run's partial groups as per-group records, not entries
                              // (k_plan_map, round 6); 0: entries (round 5; A/B)
#endif
constexpr bool kRunRecords = BMQCRC_RUN_RECORDS != 0 && kGroupDesc && BMQCRC_LONG_FLAT;

// The single-pass planner's launch tag.  Normally the host's per-workspace
// count (BatchArgs::plan_epoch, below 2^31); a batch captured into a graph
// gets 0 there and takes the tag from the device word plan_sync[1], which
// k_epoch_advance moves on before every planner launch -- so every replay
// tags its words afresh (a frozen argument would let one replay read the
// previous replay's histogram as current).
__device__ __forceinline__ uint32_t launch_epoch(const BatchArgs& a)
{
    return a.plan_epoch ? a.plan_epoch : (uint32_t)a.plan_sync[1];
}

__global__ void k_epoch_advance(unsigned long long* sync)
{
    const unsigned long long e = sync[1];
    sync[1] = 0x80000000ull | ((e + 1ull) & 0x7fffffffull);  // never 0, disjoint from host tags
}

// Planner words every consumer block keeps in LDS (filled by plan_totals):
// the exclusive segment offset of each k_plan block and its common segment
// count per message (~0 when its messages differ).
struct PlanLds {
    uint32_t boff[kPlanMaxBlocks];
    uint32_t bu[kPlanMaxBlocks];
    uint32_t wsum[40];
};

// Global exclusive prefix of segment counts: the k_plan block's offset plus,
// within the block, i's rank times the common count when the block is
// uniform (k_plan then skips seg_first for single-tile blocks), else the
// block-local prefix k_plan stored.
__device__ __forceinline__ uint32_t seg_first_g(const BatchArgs& a, const PlanLds* pl, uint64_t i)
{
    const uint32_t b = (uint32_t)(i / a.per_msg);
    const uint32_t u = pl->bu[b];
    return pl->boff[b] +
           (u != 0xffffffffu ? (uint32_t)(i - (uint64_t)b * a.per_msg) * u : a.seg_first[i]);
}

// Binary search: last message i with seg_first(i) <= g.
__device__ uint32_t find_msg(const BatchArgs& a, const PlanLds* pl, uint32_t g)
{
    uint64_t lo = 0, hi = a.n;  // invariant: first(lo) <= g < first(hi) (hi == n: inf)
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (seg_first_g(a, pl, mid) <= g) {
            lo = mid;
        } else {
            hi = mid;
        }
    }
    return (uint32_t)lo;
}

// The same for a whole group (lane l holds segment s0 + l, s0 = 64 g): one
// wave-uniform search for s0's message m0, then the first segments of
// messages m0 .. m0 + 63 (one coalesced load) and a 6-step search in
// registers.  A lane past the window (the group spans more than 64
// messages: empty ones in between) searches on its own.  Returns the
// message; *first = its first segment.  All 64 lanes must be active.
__device__ __forceinline__ uint32_t find_msg_group(const BatchArgs& a, const PlanLds* pl,
                                                   uint32_t seg, bool valid, uint32_t* first)
{
    const uint32_t lane = (uint32_t)(threadIdx.x & 63);
    const uint32_t s0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(seg - lane));
    const uint32_t m0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)find_msg(a, pl, s0));
    const uint64_t mj = (uint64_t)m0 + lane;
    const uint32_t w = mj < a.n ? seg_first_g(a, pl, mj) : 0xffffffffu;
    const uint32_t wn = (lane == 63u && mj + 1u < a.n) ? seg_first_g(a, pl, mj + 1u) : 0xffffffffu;
    uint32_t j = 0;  // largest j with w_j <= seg (w_0 <= s0 <= seg)
#pragma unroll
    for (uint32_t st = 32; st; st >>= 1) {
        const uint32_t c = (uint32_t)__shfl((int)w, (int)(j + st));
        j = c <= seg ? j + st : j;
    }
    uint32_t msg = m0 + j;
    uint32_t f = (uint32_t)__shfl((int)w, (int)j);
    const uint32_t w64 = (uint32_t)__builtin_amdgcn_readlane((int)wn, 63);
    if (valid && j == 63u && w64 <= seg) {
        msg = find_msg(a, pl, seg);
        f = seg_first_g(a, pl, msg);
    }
    *first = f;
    return msg;
}

// Block-wide exclusive scan of v over blockDim.x threads (a multiple of 64,
// at most 1024); returns the block total.  wsum: 33 words of LDS.
__device__ __forceinline__ uint32_t block_scan(uint32_t v, uint32_t* excl, uint32_t* wsum)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nw = blockDim.x >> 6;
    const uint32_t x = wave_incl_scan(v);
    if (lane == 63) {
        wsum[wave] = x;
    }
    __syncthreads();
    if (threadIdx.x < 64) {  // wave 0 (DPP needs whole rows): row 0 scans the wave totals
        const uint32_t w = (int)threadIdx.x < nw ? wsum[threadIdx.x] : 0u;
        uint32_t y = dpp_add<0x111, 0xf>(w);  // row_shr:1
        y = dpp_add<0x112, 0xf>(y);           // row_shr:2
        y = dpp_add<0x114, 0xf>(y);           // row_shr:4
        y = dpp_add<0x118, 0xf>(y);           // row_shr:8
        if (threadIdx.x < 16) {
            wsum[16 + threadIdx.x] = y - w;  // exclusive wave prefix
            if (threadIdx.x == 15) {
                wsum[32] = y;
            }
        }
    }
    __syncthreads();
    *excl = x - v + wsum[16 + wave];
    const uint32_t tot = wsum[32];
    __syncthreads();
    return tot;
}

// Batch totals from k_plan's per-block words, derived by every block of a
// consumer kernel in its prologue (blockDim.x >= nblocks): the segment count,
// the identity / uniform shape, and the exclusive segment offset of every
// k_plan block (-> boff in LDS).  Reading <= 3 x 256 L2-resident words per
// block replaces a grid-wide arrival counter and a dependent last-block pass
// at the end of k_plan.
struct PlanTotals {
    uint32_t total, identity, uni, overflow;
};

// Segment indices are 32-bit.  A batch of overlapping messages can hold more
// segments than that (4,096 messages of 2^32-1 bytes at 256-byte segments is
// 6.9e10); k_plan flags a block whose count passes kSegLimit and the consumers
// then fold every message whole in one lane (BMQCRC_F_WHOLE_MESSAGES'
// schedule: correct for any lengths, just slower), never a wrapped count.
constexpr uint64_t kSegLimit = 0xFFFFFF00ull;

// The loads are split from the reduction so that k_fold can issue them
// together with its other prologue loads.
struct PlanWords {
    uint32_t v, nn, u, u0;
};

__device__ __forceinline__ PlanWords plan_load(const BatchArgs& a)
{
    const uint32_t j = threadIdx.x, nb = a.nblocks;
    PlanWords w;
    w.v = j < nb ? a.block_sum[j] : 0u;
    w.nn = j < nb ? a.block_sum[nb + j] : 0u;
    w.u0 = a.block_sum[2u * nb];
    w.u = j < nb ? a.block_sum[2u * nb + j] : w.u0;
    return w;
}

__device__ PlanTotals plan_reduce(const BatchArgs& a, PlanLds* pl, const PlanWords w)
{
    const uint32_t j = threadIdx.x, nb = a.nblocks;
    const uint32_t v = w.v, nn = w.nn, u = w.u, u0 = w.u0;
    PlanTotals t;
    t.overflow = 0u;
    // One barrier for the shape, a second for the block offsets: each wave
    // reduces its words by DPP and ballots (a chain of LDS round trips
    // before) and publishes its sum and flags; every thread then combines
    // the waves' entries.  (A block over the limit stores ~0 segments; <=
    // 256 blocks: the 64-bit sum cannot wrap.)
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const uint32_t x = wave_incl_scan(v);  // 32-bit: used only when the total fits
    const uint64_t s64 = wave_sum64(v);
    const bool w_ragged = __ballot(nn != 0u) != 0, w_mixed = __ballot(u != u0) != 0;
    if (lane == 0) {
        pl->wsum[wv] = (uint32_t)min(s64, (uint64_t)0xffffffffu);
        pl->wsum[16u + wv] = (w_ragged ? 1u : 0u) | (w_mixed ? 2u : 0u);
    }
    __syncthreads();
    uint64_t all = 0;
    uint32_t flags = 0, before = 0;
    for (uint32_t k = 0; k < nw; ++k) {
        const uint32_t sk = pl->wsum[k];
        all += sk;
        before += k < wv ? sk : 0u;
        flags |= pl->wsum[16u + k];
    }
    if (!(flags & 1u)) {  // every message exactly one segment
        t.total = (uint32_t)a.n;
        t.identity = 1u;
        t.uni = 1u;
        return t;
    }
    t.identity = 0u;
    t.uni = (!(flags & 2u) && u0 != 0xffffffffu && u0 != 0u) ? u0 : 0u;
    if (all > kSegLimit || (t.uni && (uint64_t)a.n * t.uni > kSegLimit)) {
        t.overflow = 1u;
        t.uni = 0u;
        t.total = (uint32_t)a.n;
        return t;
    }
    if (t.uni) {
        t.total = (uint32_t)a.n * t.uni;
        return t;
    }
    t.total = (uint32_t)all;
    if (j < nb) {
        pl->boff[j] = before + x - v;
        pl->bu[j] = u;
    }
    __syncthreads();
    return t;
}

__device__ __forceinline__ PlanTotals plan_totals(const BatchArgs& a, PlanLds* pl)
{
    return plan_reduce(a, pl, plan_load(a));
}

// Geometry of segment k of a message [mstart, mstart+len): byte range
// [S, E) (internal boundaries 128-byte aligned), the stream's start L0 (16-byte
// aligned, see below), lines of the folded stream (covering the seed word of
// the first segment) and of data.
struct SegGeom {
    uint64_t S, E, L0;
    uint32_t nl, nl_data;
};

__device__ __forceinline__ SegGeom seg_geom(uint64_t mstart, uint32_t len, uint32_t k,
                                            uint32_t nseg, uint32_t SEG)
{
    SegGeom g;
    const uint64_t mend = mstart + len;
    g.S = (k == 0) ? mstart : ((mstart + (uint64_t)k * SEG) & ~127ull);
    g.E = (k + 1 == nseg) ? mend : ((mstart + (uint64_t)(k + 1) * SEG) & ~127ull);
    const uint64_t need_end = (k == 0 && g.E < g.S + 4) ? g.S + 4 : g.E;
    // Right-aligned at piece granularity (round 3): the stream ends with the
    // 16-byte piece holding its last byte and starts nl lines before, nl the
    // fewest lines that hold pieces [S/16, that piece].  The stream is a run
    // of 16-byte pieces of memory, not of 128-byte lines (pieces outside
    // [S, E) come from the zero line anyway), so a message that straddles a
    // line boundary but fits 128 bytes is one round, not two, and the zero
    // padding after E -- undone by one 160-VALU multiply per lane whenever a
    // lane of the wave has any -- is under 16 bytes, none when E is 16-byte
    // aligned.  Applied when it saves a line or the stream is one line
    // (kRightAlignLines); longer streams keep whole-cache-line rounds.
    const uint64_t pe = (need_end + 15u) & ~15ull;
    const uint32_t nl_r = (uint32_t)((pe - (g.S & ~15ull) + 127u) >> 7);
    const uint64_t L0_l = g.S & ~127ull;
    const uint32_t nl_l = (uint32_t)((need_end - L0_l + 127u) >> 7);
    if (kRightAlign && (nl_r < nl_l || nl_r <= kRightAlignLines)) {
        g.nl = nl_r;
        g.L0 = pe - ((uint64_t)nl_r << 7);
    } else {
        g.nl = nl_l;
        g.L0 = L0_l;
    }
    g.nl_data = (uint32_t)((g.E - g.L0 + 127u) >> 7);
    return g;
}

// Segment -> (message, part) for the fold kernel, by planner mode.
struct SegRef {
    uint32_t msg, k;
};

struct SegDesc {
    uint64_t off;
    uint32_t msg, k, len, seed;
};

__device__ __forceinline__ SegRef map_segment(const BatchArgs& a, const PlanLds* pl,
                                              uint32_t seg, bool valid, uint32_t identity,
                                              uint32_t uni, uint32_t sorted, uint32_t ep)
{
    SegRef r = {0u, 0u};
    if (!identity && !uni && !sorted) {
        // no map (skipped, given up or past seginfo): search seg_first, one
        // search per group (wave-uniform branch: every lane takes part)
        if (__ballot(valid) != 0) {
            uint32_t f = 0;
            const uint32_t m = find_msg_group(a, pl, seg, valid, &f);
            if (valid) {
                r.msg = m;
                r.k = seg - f;
            }
        }
        return r;
    }
    if (valid) {
        if (identity) {
            r.msg = seg;
        } else if (uni) {
            r.msg = seg / uni;
            r.k = seg - r.msg * uni;
        } else {
            // sorted: the raw entry and its group's firstk (resolved in fetch_desc)
            const uint32_t gsel = (uint32_t)__builtin_amdgcn_readfirstlane((int)seg) >> 6;
            r.msg = a.seginfo[seg];
            r.k = a.firstk[gsel];
            if (kGroupDesc) {
                // a group of 64 full segments of one message: one tagged word
                // instead of its 64 entries (which are then not written)
                const unsigned long long gd = a.gdesc[gsel];
                if ((uint32_t)(gd >> 32) == ep) {
                    r.msg = (uint32_t)gd;
                } else if (kRunRecords) {
                    // a long run's tail on the group's first lanes, or its
                    // head on the last ones: tagged records (k_plan_map,
                    // round 6), the entries under them not written
                    const u32x4 pre = *(const u32x4*)&a.grec[8u * gsel];
                    const u32x4 suf = *(const u32x4*)&a.grec[8u * gsel + 4u];
                    const uint32_t l = seg & 63u;
                    if (pre.x == ep && l < pre.z) {
                        r.msg = pre.y;
                    } else if (suf.x == ep && l >= 64u - suf.z) {
                        r.msg = suf.y;
                    }
                }
            }
        }
    }
    return r;
}

// k_fold's sorted map: (message, k) from a group's raw seginfo entries (see
// put_full / put_last): k = kKFromLength for a last segment, else the lane's
// distance from its run's head, plus firstk when the run began before the
// group (its head is lane 0).
constexpr uint32_t kKFromLength = 0xffffffffu;

__device__ __forceinline__ SegRef resolve_sorted(SegRef r, bool valid)
{
    const uint32_t lane = (uint32_t)(threadIdx.x & 63);
    const uint32_t key = valid ? r.msg : 0xffffffffu;
    const uint32_t prev = (uint32_t)__shfl_up((int)key, 1);
    const bool head = lane == 0 || prev != key || (key & kSegLast);
    const uint64_t heads = __ballot(head);
    const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
    const uint32_t h = 63u - (uint32_t)__builtin_clzll(heads & upto);
    SegRef o;
    o.msg = key & ~kSegLast;
    o.k = (key & kSegLast) ? kKFromLength : (h == 0 ? r.k : 0u) + (lane - h);
    return o;
}

__device__ __forceinline__ SegDesc fetch_desc(const BatchArgs& a, SegRef r, bool valid)
{
    SegDesc d = {0ull, r.msg, r.k, 0u, 0u};
    if (valid) {
        d.off = a.offsets[r.msg];
        d.len = a.lengths[r.msg];
        d.seed = a.seeds ? a.seeds[r.msg] : 0u;
    }
    return d;
}

#ifndef BMQCRC_FOLD_DIAG
#define BMQCRC_FOLD_DIAG 0  // 1: per-wave wall-clock stamps of the last k_fold launch
                            // (timing diagnostics, tools/fold_trace_diag.py); product: 0
#endif
#if BMQCRC_FOLD_DIAG
// diagnostic build only: per wave (entry, prologue done, first loads issued,
// first group folded, last group's lines folded, loop done, end), read by
// bmqcrc_diag_fold_trace
constexpr int kFoldTraceWaves = 4096;
__device__ unsigned long long g_fold_trace[kFoldTraceWaves][8];
#define FOLD_STAMP(k)                                                              \
    if (lane == 0 && g0 < (uint32_t)kFoldTraceWaves) {                             \
        g_fold_trace[g0][k] = wall_clock64();                                      \
    }
#else
#define FOLD_STAMP(k)
#endif

#ifndef BMQCRC_ONE_DIAG
#define BMQCRC_ONE_DIAG 0  // diagnostic builds of the ONE kernel (wrong CRCs): bit 0 skips the
                           // remainder step, bit 1 the fold; product: 0
#endif

#ifndef BMQCRC_NT_LOADS
#define BMQCRC_NT_LOADS 1  // 0: every data round with the default policy (A/B)
#endif
constexpr bool kNtLoads = BMQCRC_NT_LOADS != 0;

#ifndef BMQCRC_SHORT_NT_WHOLE_LINES
#define BMQCRC_SHORT_NT_WHOLE_LINES 1  // 0: every short group with the default policy (round 4)
#endif
constexpr bool kShortNtWholeLines = BMQCRC_SHORT_NT_WHOLE_LINES != 0;

#ifndef BMQCRC_SNAKE
#define BMQCRC_SNAKE 1  // 0: every round in block order (A/B)
#endif
constexpr bool kSnakeRounds = BMQCRC_SNAKE != 0;

#ifndef BMQCRC_TWO_ENDED
#define BMQCRC_TWO_ENDED 0  // 1: claims from both ends of each block's groups (A/B)
#endif
constexpr bool kTwoEnded = BMQCRC_TWO_ENDED != 0;

#ifndef BMQCRC_BYTE_FOLD
#define BMQCRC_BYTE_FOLD 1  // remainder words folded to 8 at byte granularity first (8-wave
                            // blocks): 1 every group (product), 2 one-line groups only, 0
                            // never: the 11-bit chains over all 32 words (A/B)
#endif
constexpr int kByteFold = BMQCRC_BYTE_FOLD;
#ifndef BMQCRC_BYTE_FOLD4
#define BMQCRC_BYTE_FOLD4 1  // 0: 4-wave blocks keep the two-word Horner over all 32 words (A/B)
#endif
constexpr bool kByteFold4 = BMQCRC_BYTE_FOLD4 != 0;

#ifndef BMQCRC_NT_RESULTS
#define BMQCRC_NT_RESULTS 0  // 1: result stores with the non-temporal hint (A/B)
#endif
constexpr bool kNtResults = BMQCRC_NT_RESULTS != 0;

#ifndef BMQCRC_ONE_PRIO
#define BMQCRC_ONE_PRIO 2  // the one-segment kernel's wave behind its SIMD partner in groups
                           // takes issue priority: 2 in groups of two or more lines (product),
                           // 1 in every group, 0 never (A/B)
#endif
constexpr int kOnePrio = BMQCRC_ONE_PRIO;

#ifndef BMQCRC_ONE_CLAIMS
#define BMQCRC_ONE_CLAIMS 0  // 1: the one-segment kernel claims its groups from the block's LDS
                             // counter too (the claiming loop and block list; A/B)
#endif
constexpr bool kOneClaims = BMQCRC_ONE_CLAIMS != 0;

#ifndef BMQCRC_HORNER11
#define BMQCRC_HORNER11 1  // 0: byte-sliced remainder tables in every block shape (round 4; A/B)
#endif
constexpr bool kHorner11 = BMQCRC_HORNER11 != 0;

// Groups whose speculative first pass skipped a message (a block's list for
// the second pass; past this many the second pass scans the block's groups).
constexpr uint32_t kLongListCap = 64;

// ONE: a speculative launch predicting one segment per message (spec == 1),
// compiled apart so the first pass knows k = 0 and nseg = 1 (no planner words,
// no move to the message end, no run combine); it keeps static grid-stride
// shares (below).
// WPB: waves per block.  8 = one block of two waves per SIMD per CU (round
// 4), whose waves (ONE aside) take the block's groups from an LDS counter:
// with two 4-wave blocks per CU and a static grid-stride share each, the
// CU's second block ran its waves 9 % longer (later start, then less issue
// share) and the launch ended on it (tools/fold_trace_diag.py,
// profiles/r04/fold_trace/).  4 = one wave per SIMD (large-message batches,
// one block per CU) or small batches spread over more CUs.
template <bool NT, bool ONE, int WPB>
__global__ __launch_bounds__(WPB * 64, WPB == 4 ? 2 : 1) void k_fold(BatchArgs a)
{
    constexpr uint32_t kThreads = WPB * 64;
    constexpr int kLds = WPB * kSlots * kSlotBytes;
    // 11-bit remainder slices in the 8-wave blocks (one per CU: 159 KiB of
    // LDS with them); 4-wave blocks, two of which share a CU, keep the 8 KiB
    // byte slices
    constexpr bool H11 = kHorner11 && WPB == 8;
    constexpr int kTab = H11 ? (int)kTab11Bytes : kTabBytes;
    // remainder tables, DMA slots, move factors (not needed by ONE: no moves
    // in its first pass)
    __shared__ __attribute__((aligned(16))) uint8_t lds[kTab + kLds + (ONE ? 0 : kXbBytes)];
    // group claims (gid below): wave w starts with claim k = w, later k come
    // from this counter; long_n / long_list: the block's groups with a message
    // its speculative first pass skipped
    __shared__ uint32_t claim_ctr, long_n;
    __shared__ unsigned long long claim2;  // two-ended claims: front count | back count << 32
    __shared__ uint32_t long_list[kLongListCap];
    __shared__ uint32_t one_prog[WPB];  // BMQCRC_ONE_PRIO: groups each wave has started

    const int lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t tab_lds = (uint32_t)(uintptr_t)(lds_u8*)lds;
    const uint32_t wave_lds = tab_lds + kTab + wave * (kSlots * kSlotBytes);
    const uint32_t xb_lds = tab_lds + kTab + kLds;
    // a segment's raw CRC from its 32 remainder words (skip: words 0-15 are
    // zero in every lane; one_line: the group's streams are one line; both
    // wave-uniform, choosing between compiled copies)
    auto remainder = [&](const uint32_t (&Rm)[32], bool skip, bool one_line) -> uint32_t {
        if constexpr (H11 && kByteFold != 0) {
            if (kByteFold == 1 || one_line) {
                return skip ? tail_bytes8<true>(Rm, tab_lds) : tail_bytes8<false>(Rm, tab_lds);
            }
            return tail_chains11(Rm, tab_lds);  // (skip is set for one-line groups only)
        } else if constexpr (H11) {
            return skip ? tail_chains11<8>(Rm, tab_lds) : tail_chains11(Rm, tab_lds);
        } else if constexpr (kByteFold4) {
            // 4-wave blocks: the byte fold too, its last 8 steps on the byte
            // tables (32 lookups per segment instead of 128)
            return skip ? tail_bytes8<true, true>(Rm, tab_lds) : tail_bytes8<false, true>(Rm, tab_lds);
        } else {
            return skip ? tail_horner<8>(Rm, tab_lds) : tail_horner(Rm, tab_lds);
        }
    };
    if (threadIdx.x < (uint32_t)WPB) {
        one_prog[threadIdx.x] = 0u;
    }
    if (threadIdx.x == 0) {
        claim_ctr = WPB;
        claim2 = 0ull;
        long_n = 0;
    }

    // Prologue: every load that depends on nothing is issued before the first
    // wait -- the remainder tables, k_plan's block words and the first group's
    // descriptors as if segment = message (true for BMQCRC_F_WHOLE_MESSAGES
    // and for identity batches; discarded otherwise).
    constexpr int kTw = (kTab / 4) / (int)kThreads, kXw = 1024 / kThreads;  // table words per thread
    static_assert(kTw * (int)kThreads * 4 == kTab && kXw * kThreads == 1024, "table fill");
    // The one-segment kernel (kOneEarly) loads no table here: its first
    // group's descriptors go out first, then the group's data, and only then
    // the tables, LDS-DMA'd (see early_tables below), so the first data
    // load no longer waits behind 8-24 KiB of table loads and a barrier
    // (per-wave stamps, 20,000 x 256 B: prologue 0.8-1.0 us, first issue
    // 1.5 us later, profiles/r05/probe/fold_trace_small_batches.jsonl)
    constexpr bool kEarly = ONE && kOneEarly && WPB == 4;
    static_assert(!kEarly || kTab % (1024 * WPB) == 0, "early tables: whole KiB per wave");
    constexpr bool kNoVgprTab = kEarly;
    // the wave's first group (claim k = wave, see gid below), as if
    // segment = message: its descriptors are the kernel's first loads
    // (round 6; before, 8-24 KiB of table loads per block went out first
    // and every wave's first data load queued behind them)
    const uint32_t gfirst = a.spread ? wave * gridDim.x + blockIdx.x : blockIdx.x * WPB + wave;
    const uint32_t sid = gfirst * 64u + (uint32_t)lane;
    [[maybe_unused]] SegDesc spec = {0ull, 0u, 0u, 0u, 0u};
    if constexpr (kDescFirst) {
        spec = fetch_desc(a, SegRef{sid, 0u}, sid < a.n);
    }
    uint32_t tw[kNoVgprTab ? 1 : kTw];
#pragma unroll
    for (int i = 0; i < (kNoVgprTab ? 0 : kTw); ++i) {
        const uint32_t t = threadIdx.x + (uint32_t)i * kThreads;
        if constexpr (H11) {
            tw[i] = c_rtab11[t];
        } else {
            tw[i] = c_ty[t >> 8][t & 255u];
        }
    }
    uint32_t xw[kXw];
    if (!ONE) {
#pragma unroll
        for (int i = 0; i < kXw; ++i) {
            const uint32_t t = threadIdx.x + (uint32_t)i * kThreads;
            xw[i] = c_xbytes[t >> 8][t & 255u];
        }
    }
    const uint32_t whole = ONE ? 0u : a.whole;
    // speculative single launch (no planner ran): every message predicted to
    // have spec_u segments, spec_u dividing 64 (1: one segment per message)
    const uint32_t spec_mode = ONE ? 1u : a.spec;
    const uint32_t spec_u = spec_mode ? spec_mode : 1u;
    PlanWords pw = {0u, 0u, 0u, 0u};
    uint32_t map_void = 0u;  // k_plan_map gave up its map for this launch
    uint32_t ep = a.plan_epoch;  // the planner's launch tag (0: kept on the device)
    if (!whole && !spec_mode) {
        pw = plan_load(a);
        if (a.map_planned && a.plan_sync) {
            ep = launch_epoch(a);
            map_void = (uint32_t)a.plan_sync[2] == ep;
        }
    }
    // x^(-8p) un-shift table -> LDS too: a per-lane index, so from constant
    // memory it would be a vector load with a full memory latency per group
    __shared__ __attribute__((aligned(16))) uint32_t xneg8[136];
    const uint32_t xn = (!kNoVgprTab && threadIdx.x < 136u) ? c_xneg8[threadIdx.x] : 0u;
    [[maybe_unused]] const uint32_t g0 = blockIdx.x * WPB + wave;  // this wave's index in the grid
    FOLD_STAMP(0)
    if constexpr (!kDescFirst) {
        spec = fetch_desc(a, SegRef{sid, 0u}, sid < a.n);
    }
    // remainder-reduction tables -> LDS (8 KiB, once per block; no DMA in
    // flight yet; plan_reduce's barriers order them before any lookup)
#pragma unroll
    for (int i = 0; i < (kNoVgprTab ? 0 : kTw); ++i) {
        const uint32_t t = threadIdx.x + (uint32_t)i * kThreads;
        *(lds_u32*)(uintptr_t)(tab_lds + 4u * t) = tw[i];
    }
    if (!kNoVgprTab && threadIdx.x < 136u) {
        xneg8[threadIdx.x] = xn;
    }
    // kEarly: this wave's share of the tables, LDS-DMA'd after its first
    // group's loads (wave w: KiB w * kTab / 1024 / WPB ...; wave 0 also the
    // 544-byte x^-8p table).  Nothing reads them before early_barrier.
    auto early_tables = [&]() {
        if constexpr (kEarly) {
            constexpr int kKib = kTab / 1024 / WPB;
            const uint64_t src = H11 ? (uint64_t)(uintptr_t)&c_rtab11[0]
                                     : (uint64_t)(uintptr_t)&c_ty[0][0];
            dma_copy_kib<kKib>(tab_lds + 1024u * kKib * wave, src + 1024u * kKib * wave);
            if (wave == 0 && lane < 34) {
                dma_copy_kib<1>((uint32_t)(uintptr_t)xneg8, (uint64_t)(uintptr_t)&c_xneg8[0]);
            }
        }
    };
    // every wave once, before its first lookup: its own table loads have
    // landed (the counted waits of its first fold, or the explicit one
    // here), then the block meets, so every wave's share is visible
    auto early_barrier = [&](bool wait) {
        if constexpr (kEarly) {
            if (wait) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            __builtin_amdgcn_s_barrier();
        }
    };
    if (!ONE) {
#pragma unroll
        for (int i = 0; i < kXw; ++i) {
            const uint32_t t = threadIdx.x + (uint32_t)i * kThreads;
            *(lds_u32*)(uintptr_t)(xb_lds + 4u * t) = xw[i];
        }
    }

    // BMQCRC_F_WHOLE_MESSAGES and speculative launches: group g = messages
    // 64g..64g+63 (speculative uniform: 64g/u .. 64(g+1)/u - 1, u segments
    // each), no planner ran.  Otherwise the batch totals come from k_plan's
    // block words.
    __shared__ PlanLds pl;
    PlanTotals pt = {(uint32_t)a.n * spec_u, spec_u == 1u ? 1u : 0u, spec_u == 1u ? 0u : spec_u,
                     0u};
    if (!whole && !spec_mode) {
        pt = plan_reduce(a, &pl, pw);
    } else {
        __syncthreads();
    }
    // more segments than 32-bit indices hold: every message in one lane.  A
    // map k_plan_map gave up is not used; its seg_first is (binary search).
    const uint32_t wholef = whole | pt.overflow;
    const uint32_t hint_identity = pt.identity && !pt.overflow;
    const uint32_t hint_uni = pt.uni;
    if (pt.overflow) {
        pt.identity = 1u;
        pt.uni = 0u;
        pt.total = (uint32_t)a.n;
    }
    const uint32_t total = pt.total;
    const uint32_t identity = pt.identity;
    const uint32_t uni = pt.uni;
    // the size-class order exists only if the histogram and k_plan_sort ran
    // (and seginfo could hold every segment, and k_plan_map kept its map)
    const uint32_t sorted =
        (wholef || !a.map_planned || identity || uni || total > a.max_segs || map_void) ? 0u : 1u;
    const uint32_t ngroups = (total + 63u) / 64u;
    const uint32_t SEG = a.seg_bytes;
    const uint64_t arena = (uint64_t)(uintptr_t)a.arena;
    if (a.shape_hint && blockIdx.x == 0 && threadIdx.x == 0 && !whole && !spec_mode) {
        // batch shape for the host's next launch decision (host-mapped word);
        // a speculative launch keeps kHintIdentity unless a message is queued
        // (a closed-form batch whose u segments per message divide 64 also
        // records u: its successor can run speculatively, see kHintClosed)
        __hip_atomic_store(a.shape_hint,
                           hint_identity ? kHintIdentity
                           : (hint_uni && !pt.overflow && 64u % hint_uni == 0u)
                               ? (kHintClosed | (hint_uni << 8))
                           : (hint_uni || pt.overflow) ? kHintClosed
                                                  : kHintRagged,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (map_void) {  // the GPU was shared: the host plans with the pair for a while
            __hip_atomic_store(a.shape_hint + 1, ep, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }

    FOLD_STAMP(1)
    const uint32_t rd_off = (uint32_t)lane * 128u + (((uint32_t)lane >> 1) & 7u) * 16u;
    const uint64_t zero = (uint64_t)(uintptr_t)g_zero_line + 16u * ((uint32_t)lane & 7u);

    // Claim k of this block is group WPB (b_r + G r) + k % WPB, r = k / WPB
    // (G = gridDim.x; >= ngroups: none): chunks of WPB adjacent groups, one
    // per block and round -- one-group-per-wave batches keep round 3's
    // layout (mapping claim k to group blockIdx.x + G k instead cost the
    // headline 1.5-2 %, profiles/r04/ab/).  b_r = blockIdx.x in even rounds
    // and G - 1 - blockIdx.x in odd ones: in a size-class-sorted map the
    // chunks' work grows (or shrinks) along the map, so the same block taking
    // chunk b of every round got the largest chunk of each (the 1/8 Zipf
    // shard's block means fell with the block index, correlation -0.74,
    // 475-534 us, profiles/r04/fold_trace/).  gid grows with k.
    const uint32_t nbk = gridDim.x;
    auto gid = [&](uint32_t k) {
        if (a.spread) {
            return k * nbk + blockIdx.x;
        }
        const uint32_t r = k / (uint32_t)WPB;
        const uint32_t b = (kSnakeRounds && !ONE && (r & 1u)) ? nbk - 1u - blockIdx.x : blockIdx.x;
        return (b + nbk * r) * (uint32_t)WPB + k % (uint32_t)WPB;
    };
    // a claim in two halves: the LDS atomic (lane 0) is issued early and its
    // result read later, so its latency hides behind other LDS work
    // Two-ended claims (BMQCRC_TWO_ENDED, A/B): the block's K claims k =
    // 0 .. K-1 are taken from both ends at once, waves 0 .. WPB/2-1 from the
    // front (the map's first size classes), the others from the back (its
    // last), so that a CU folds large and small groups side by side instead
    // of one size class after another; one 64-bit LDS counter holds both
    // counts, and a claim is valid while they sum to less than K.
    const bool back = kTwoEnded && wave >= (uint32_t)WPB / 2u;
    uint32_t kb = 0;  // this block's claims (gid(k) < ngroups exactly for k < kb)
    if (kTwoEnded && a.spread) {
        kb = blockIdx.x < ngroups ? (ngroups - blockIdx.x - 1u) / nbk + 1u : 0u;
    } else if (kTwoEnded) {
        const uint32_t full = ngroups / (nbk * (uint32_t)WPB);
        kb = full * (uint32_t)WPB;
        const uint32_t b = (kSnakeRounds && !ONE && (full & 1u)) ? nbk - 1u - blockIdx.x : blockIdx.x;
        const uint64_t c = (uint64_t)(b + nbk * full) * WPB;
        if (c < ngroups) {
            kb += (uint32_t)min((uint64_t)WPB, (uint64_t)ngroups - c);
        }
    }
    auto claim_issue = [&]() {
        unsigned long long k = 0;
        if (lane == 0) {
            if (kTwoEnded) {
                k = atomicAdd(&claim2, back ? (1ull << 32) : 1ull);
            } else {
                k = atomicAdd(&claim_ctr, 1u);
            }
        }
        return k;
    };
    auto claim_take = [&](unsigned long long k) {
        if (kTwoEnded) {
            const uint32_t f = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)k);
            const uint32_t bk = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(k >> 32));
            if ((uint64_t)f + bk >= kb) {
                return ngroups;
            }
            return gid(back ? kb - 1u - bk : f);
        }
        return gid((uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)k));
    };
    auto claim = [&]() { return claim_take(claim_issue()); };
    const uint32_t seg_shift = (SEG & (SEG - 1u)) == 0 ? (uint32_t)__builtin_ctz(SEG) : 0u;

    // One group = 64 segments, one per lane.  Its per-lane geometry and the
    // DMA source of every instruction of its rounds (see dma_round).
    struct Group {
        uint64_t pbase[8];
        uint32_t plo[8], pcnt[8];
        uint64_t E, L0, mend;
        uint32_t msg, k, nseg, nl, R, r0, sl, jE, eE, c0, hskip;
        bool valid, first, lo_part, hi_part;
        bool whole_lines;  // every valid lane's [S, E) starts and ends on a 128-byte line
    };
    // Geometry of one lane's segment k of a message of nseg segments.
    auto setup_lane = [&](bool valid, uint32_t msg, uint32_t k, uint32_t nseg, uint64_t off,
                          uint32_t len, uint32_t seed, Group& G) {
        G.valid = valid;
        G.msg = msg;
        G.k = k;
        G.nseg = valid ? nseg : 0u;
        const uint64_t mstart = arena + off;
        G.mend = mstart + len;
        const SegGeom geo = seg_geom(mstart, len, G.k, G.nseg, SEG);
        G.E = geo.E;
        G.L0 = geo.L0;
        G.first = G.valid && G.k == 0;
        G.nl = G.valid ? geo.nl : 0u;
        // every lane invalid (a speculative group of queued messages): one
        // round of zeros, nothing stored
        G.R = max(wave_max(G.nl), 1u);
        // one-line group: the remainder is the line; its leading zero word
        // pairs (before the lowest S of the wave) need no remainder step
        G.hskip = 0u;
        if (kHornerSkip && G.R == 1u) {
            // every lane's S in the line's second half (one ballot: this sits
            // before the next group's loads)
            const uint32_t sl0 = G.valid ? (uint32_t)(geo.S - geo.L0) : 128u;
            G.hskip = __ballot(sl0 < 64u) == 0 ? 8u : 0u;
        }
        // right-aligned stream: this lane's line j is round r0 + j
        G.r0 = G.R - G.nl;
        G.sl = G.valid ? (uint32_t)(geo.S - G.L0) : 0u;  // S's offset in line 0
        const uint64_t el = G.valid ? G.E - G.L0 : 0u;   // E's offset in the stream
        G.lo_part = (G.sl & 15u) != 0;
        G.hi_part = (el & 15u) != 0;
        G.jE = (uint32_t)(el >> 7);    // line holding E's cut piece
        G.eE = (uint32_t)(el & 127u);  // E's offset in that line
        G.c0 = ~seed;
        G.whole_lines = __ballot(G.valid && (((geo.S | geo.E) & 127u) != 0)) == 0;
        // DMA source per instruction: pieces [gS, gE) of the stream overlap
        // [S, E); the stream piece index in round r is 8 (r - r0) + piece
        const uint32_t gS = G.sl >> 4;
        const uint32_t gE = (uint32_t)((el + 15u) >> 4);
        const uint32_t plo_l = 8u * G.r0 + gS;
        const uint32_t pcnt_l = G.valid ? gE - gS : 0u;
        const uint64_t pb_l = G.L0 - ((uint64_t)G.r0 << 7);
        // Instruction i reads segments 8i .. 8i+7 (lane l: segment 8i + l/8),
        // so each lane needs eight other lanes' sources: transposed through a
        // 1 KiB scratch at the start of slot 0 (free here: no DMA in flight,
        // and this wave's earlier reads of it complete first, LDS being in
        // order per wave).  Lane s writes record (s & 7) * 8 + ((s >> 3) ^
        // (s & 7)); lane l reads records (l >> 3) * 8 + (i ^ (l >> 3)), i =
        // 0..7 (the XOR spreads one read's eight addresses over the banks).
        const uint32_t ls = (uint32_t)lane;
        const uint32_t kq = ls >> 3;
        *(lds_u4*)(uintptr_t)(wave_lds + 16u * ((ls & 7u) * 8u + (kq ^ (ls & 7u)))) =
            u32x4{(uint32_t)pb_l, (uint32_t)(pb_l >> 32), plo_l, pcnt_l};
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const u32x4 v = *(lds_cu4*)(uintptr_t)(wave_lds + 16u * (kq * 8u + ((uint32_t)i ^ kq)));
            const uint32_t pp = ((uint32_t)lane & 7u) ^ ((4u * i + ((uint32_t)lane >> 4)) & 7u);
            G.pbase[i] = (((uint64_t)v.y << 32) | v.x) + 16u * pp;
            G.plo[i] = v.z - pp;
            G.pcnt[i] = v.w;
        }
    };
    auto segments = [&](uint32_t len) {
        return len ? (seg_shift ? ((len - 1u) >> seg_shift) : (len - 1u) / SEG) + 1u : 0u;
    };
    bool long_seen = false;  // ONE: a message of this wave's groups needs the second pass
    // The segment of group gg in this lane (planned or speculative mapping).
    auto setup = [&](const SegDesc& d, uint32_t gg, Group& G) {
        const uint32_t seg = gg * 64u + (uint32_t)lane;
        bool valid = seg < total;
        uint32_t nseg = !valid ? 0u : (wholef ? 1u : segments(d.len));
        if (spec_mode) {
            // a message of another segment count than predicted is left to
            // the wave's second pass (below); with u = 1 an empty message is
            // folded whole (its seed)
            const bool ok = spec_u == 1u ? nseg <= 1u : nseg == spec_u;
            if constexpr (ONE && !kOneClaims) {
                long_seen |= __ballot(valid && !ok) != 0;
            } else if (__ballot(valid && !ok) != 0 && lane == 0) {  // group gg on the block's list
                const uint32_t at = atomicAdd(&long_n, 1u);
                if (at < kLongListCap) {
                    long_list[at] = gg;
                }
            }
            valid = valid && ok;
            nseg = spec_u;
        }
        if (ONE) {
            setup_lane(valid, d.msg, 0u, 1u, d.off, d.len, d.seed, G);
        } else {
            // (a sorted map's last segment: k from the message's length)
            setup_lane(valid, d.msg, d.k == kKFromLength ? nseg - 1u : d.k, nseg, d.off, d.len,
                       d.seed, G);
        }
    };
    // Load policy per group: streams of three or more lines read
    // non-temporally; a group of one or two lines per lane does too when every
    // lane's segment is whole lines (no line shared with a neighbouring
    // message), else with the default policy, which keeps a line that two
    // messages share in L2 for the second.  Measured on MI355X batches read
    // from HBM (profiles/r05/ab/ntshort_ab.jsonl): non-temporal 256-byte
    // messages +13-15 % (4M: 0.640 -> 0.721 of the roofline), 128-byte +5 %,
    // 64-byte flat, 200-byte (lines shared) -8 %; long streams 8-10 % faster
    // non-temporal (round 2).  Round 2 chose the default policy for every
    // short group from a batch the Infinity Cache held (+3 %).
    auto issue_first_rounds = [&](const Group& G) {
        if (!NT || !kNtLoads || (kShortDefaultPolicy && G.R <= 2u && !(kShortNtWholeLines && G.whole_lines))) {
            dma_round<false>(wave_lds, G.pbase, G.plo, G.pcnt, zero, 0);
            if (G.R > 1) {
                dma_round<false>(wave_lds + kSlotBytes, G.pbase, G.plo, G.pcnt, zero, 1);
            }
            return;
        }
        dma_round<true>(wave_lds, G.pbase, G.plo, G.pcnt, zero, 0);
        if (G.R > 1) {
            dma_round<true>(wave_lds + kSlotBytes, G.pbase, G.plo, G.pcnt, zero, 1);
        }
    };

    // Rounds of a group whose first two rounds are in flight: rounds 0 .. R-2
    // fold into the ring; the last round (peeled, so no remainder array is
    // carried through the loop) gives the remainder words Rm.
    auto fold_rounds = [&](const Group& G, uint32_t (&Rm)[32]) {
        uint32_t q[32], p[32];
        [[maybe_unused]] uint32_t sink = 0;  // BMQCRC_ONE_DIAG & 2: keeps the line reads
        const uint32_t R = G.R;
        auto load_line = [&](uint32_t r, uint32_t slot, uint32_t (&m)[32]) {
            // Byte edges of this round's line: the piece cut by S (first line),
            // the piece cut by E, and the seed word (first segment only; it may
            // spill into the second line).  Lanes before their stream (j wraps)
            // match none of these.
            const uint32_t j = r - G.r0;
            const bool fx_lo = G.lo_part && j == 0u;
            const bool fx_hi = G.hi_part && j == G.jE;
            const bool fx_sd = G.first && (j == 0u || (j == 1u && G.sl > 124u));
            if (__ballot(fx_lo || fx_hi || fx_sd)) {
                if (fx_lo || fx_hi || fx_sd) {
                    line_fixup(slot, rd_off, fx_lo, G.sl, fx_hi, G.eE, fx_sd,
                               (int)(G.sl - 128u * j), G.c0);
                }
            }
#pragma unroll
            for (int kk = 0; kk < 8; ++kk) {
                const u32x4 v = *(lds_cu4*)(uintptr_t)(slot + (rd_off ^ (16u * kk)));
                m[4 * kk + 0] = v.x;
                m[4 * kk + 1] = v.y;
                m[4 * kk + 2] = v.z;
                m[4 * kk + 3] = v.w;
            }
        };
        for (uint32_t r = 0; r + 1 < R; ++r) {
            const uint32_t slot = wave_lds + (r & 1u) * kSlotBytes;
            if constexpr (kRoundWait0) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            }
            uint32_t m[32];
            load_line(r, slot, m);
            if (r + 2 < R) {
                dma_round<NT && kNtLoads>(slot, G.pbase, G.plo, G.pcnt, zero, r + 2);
            }
            if (ONE && (BMQCRC_ONE_DIAG & 2)) {
#pragma unroll
                for (int d = 0; d < 32; ++d) {
                    sink ^= m[d];
                }
            } else if (r == 0) {
                first_round(q, p, m);
            } else {
                fold_round(q, p, m);
            }
        }
        const uint32_t slot = wave_lds + ((R - 1u) & 1u) * kSlotBytes;
        // R_d = m_d ^ (taps into the previous round): the taps need only the
        // ring, so they are summed before the last line lands, and the path
        // from its arrival to the next group's loads is 32 XORs (one-line
        // streams: no history)
        // one-line streams read the line as is; the others XOR the taps into
        // the last line (no zeroed tap array for one-line groups: materialised
        // for every group it cost 32 VALU each, 1M x 256 B +1.8 %, 64 B +3 %,
        // profiles/r03/ab/ab7_split_tail_priority.jsonl)
        if (R == 1) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            load_line(0u, slot, Rm);
            return;
        }
        uint32_t H[32];
        if (ONE && (BMQCRC_ONE_DIAG & 2)) {
#pragma unroll
            for (int d = 0; d < 32; ++d) {
                H[d] = d == 0 ? sink : 0u;
            }
        } else {
            tail_taps(q, p, H);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        uint32_t m[32];
        load_line(R - 1u, slot, m);
#pragma unroll
        for (int d = 0; d < 32; ++d) {
            Rm[d] = m[d] ^ H[d];
        }
    };

    // Move + combine of a folded group: raw(stream) = raw(segment) * x^(8
    // padE): un-shift the zero padding (table x^-8p + one 160-VALU multiply),
    // then move the segment to the message end with x^(8 after) (sparse
    // exponent: bits no lane needs are skipped wave-uniformly).
    auto contribution = [&](const Group& C, uint32_t crc) {
        uint32_t contrib = 0;
        const uint32_t padE = C.valid ? (uint32_t)(C.L0 + ((uint64_t)C.nl << 7) - C.E) : 0u;
        if (__ballot(padE != 0) == 0) {
            contrib = C.valid ? crc : 0u;
        } else if (C.valid) {
            contrib = gmul(crc, xneg8[padE]);
        }
        if (ONE) {  // second pass only (mispredicted long messages)
            contrib = mul_xpow(contrib, C.valid ? mersenne31(8ull * (C.mend - C.E)) : 0u);
        } else {
            contrib = mul_xbytes(contrib, C.valid ? (uint32_t)(C.mend - C.E) : 0u, xb_lds);
        }
        if (C.first) {
            contrib ^= 0xffffffffu;
        }
        return contrib;
    };
    // A group's result: per lane nothing, a store or an XOR-atomic into
    // out[msg].  finish computes it; commit issues it one group later, after
    // the group after it has issued its loads (round 5).  A store issued
    // just before a wave's next s_waitcnt vmcnt is waited for there too
    // (stores share the load counter on gfx950), so its acknowledgement
    // latency sat on every group's critical path: a diagnostic build without
    // the stores ran 4M x 256 B 9 %, 64- and 128-byte messages 15 % faster.
    // Committed after the next group's loads are issued, same box: 2M x
    // 128 B +12 %, 4M x 64 B +9 %, 200 B +5 %, 4M x 256 B +2 %; committed
    // right after the wait instead, 64 B lost 5 % (the store then delays
    // the next loads) (profiles/r05/ab/deferred_commit_ab.jsonl).
    struct Pending {
        uint32_t msg, val, mode;  // mode: 0 none, 1 store, 2 atomic XOR
    };
    auto commit = [&](const Pending& P) {
        if (P.mode == 1u) {
            if (kNtResults) {
                __builtin_nontemporal_store(P.val, &a.out[P.msg]);
            } else {
                a.out[P.msg] = P.val;
            }
        } else if (P.mode == 2u) {
            atomicXor(&a.out[P.msg], P.val);
        }
    };
    auto finish = [&](const Group& C, uint32_t crc) -> Pending {
        Pending P = {C.msg, 0u, 0u};
        if (ONE) {
            // every segment is a whole message ending at E: un-shift the
            // padding, invert, store
            uint32_t contrib = C.valid ? crc : 0u;
            const uint32_t padE = C.valid ? (uint32_t)(C.L0 + ((uint64_t)C.nl << 7) - C.E) : 0u;
            if (__ballot(padE != 0) != 0 && C.valid) {
                contrib = gmul(crc, xneg8[padE]);
            }
            P.val = contrib ^ 0xffffffffu;
            P.mode = C.valid ? 1u : 0u;
            return P;
        }
        uint32_t contrib = contribution(C, crc);
        // XOR-reduce each run of adjacent lanes holding the same message, then
        // one store or atomic per run: the run head owns the result.  A
        // message may occupy several runs of one wave (the size-class sort
        // can split its segments across a bucket boundary inside the wave),
        // so runs are delimited by a head ballot, never by key equality, and
        // a head stores plainly only when its run is the whole message.
        if (__ballot(C.valid && C.nseg != 1u) == 0) {
            // every segment of this group is a whole message: no runs to combine
            P.val = contrib;
            P.mode = C.valid ? 1u : 0u;
            return P;
        }
        const uint32_t key = C.valid ? C.msg : 0xffffffffu;
        const uint32_t pkey = (uint32_t)__shfl_up((int)key, 1);
        const bool head = lane == 0 || pkey != key;
        const uint64_t heads = __ballot(head);
        const uint64_t upto = (lane == 63) ? ~0ull : ((2ull << lane) - 1ull);
        const uint64_t later = heads & ~upto;
        const uint32_t rend = later ? (uint32_t)__builtin_ctzll(later) : 64u;  // run end
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t ov = (uint32_t)__shfl_down((int)contrib, o);
            if ((uint32_t)lane + (uint32_t)o < rend) {
                contrib ^= ov;
            }
        }
        P.val = contrib;
        if (C.valid && head) {
            // a plain store when the whole message is this run
            P.mode = (C.k == 0 && rend - (uint32_t)lane == C.nseg) ? 1u : 2u;
        }
        return P;
    };

    // Speculative launches only: the block's messages of another segment
    // count than predicted, skipped by the first pass, folded with all 64
    // lanes of a wave (lane l: segment 64c + l of chunk c), one message at a
    // time; the chunks' contributions are XOR-accumulated in registers and
    // stored once.  The groups holding them are on the block's list (all the
    // block's groups are scanned if it overflowed), shared out over its
    // waves.  No wave waits on another block, and in the predicted case
    // (every message as predicted) no wave runs this pass.
    //
    // The speculative one-segment kernel (ONE) runs round 3's form: the wave
    // flags its own groups (long_seen) and scans them again.  (Sharing the
    // claiming kernels' block list there, or dropping the pass, changed
    // ONE's code generation and cost one-line groups 15 %: 64-byte messages
    // 96 against 82 us, profiles/r04/ab/small_msgs/.)
    auto second_pass = [&](uint32_t nlong) {
        bool any = false;
        const uint32_t mpg = 64u / spec_u;  // messages per group
        const bool listed = nlong <= kLongListCap;
        for (uint32_t j = wave;; j += WPB) {
            const uint32_t gg = (ONE && !kOneClaims) ? gfirst + (j / (uint32_t)WPB) * nbk * (uint32_t)WPB
                                : listed ? (j < nlong ? long_list[j] : ngroups) : gid(j);
            if (gg >= ngroups) {
                break;
            }
            const uint64_t i = (uint64_t)gg * mpg + (uint32_t)lane;
            const bool mine = (uint32_t)lane < mpg && i < a.n;
            const uint32_t len = mine ? a.lengths[i] : 0u;
            const uint32_t ns = segments(len);
            uint64_t todo = __ballot(mine && (spec_u == 1u ? ns > 1u : ns != spec_u));
            any = any || todo != 0;
            for (; todo; todo &= todo - 1ull) {
                const uint32_t msg = (uint32_t)((uint64_t)gg * mpg + __builtin_ctzll(todo));
                const uint64_t off = a.offsets[msg];
                const uint32_t mlen = a.lengths[msg];
                const uint32_t seed = a.seeds ? a.seeds[msg] : 0u;
                const uint32_t nseg = segments(mlen);
                uint32_t acc = mlen ? 0u : seed;  // an empty message's CRC is its seed
                for (uint32_t c = 0; 64u * c < nseg; ++c) {
                    const uint32_t k = 64u * c + (uint32_t)lane;
                    Group H;
                    setup_lane(k < nseg, msg, k, nseg, off, mlen, seed, H);
                    issue_first_rounds(H);
                    uint32_t Rm[32];
                    fold_rounds(H, Rm);
                    uint32_t x = contribution(H, remainder(Rm, false, H.R == 1u));
#pragma unroll
                    for (int o = 32; o > 0; o >>= 1) {
                        x ^= (uint32_t)__shfl_xor((int)x, o);
                    }
                    acc ^= x;
                }
                if (lane == 0) {
                    a.out[msg] = acc;
                }
            }
        }
        if (any && lane == 0 && a.shape_hint) {  // mispredicted: plan the next batch
            __hip_atomic_store(a.shape_hint, kHintRagged, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        }
    };

    // Descriptor pipeline: the (offset, length, seed) of the next group and
    // the (message, part) of the one after are loaded a group ahead, and a
    // group's first two rounds are in flight before the previous group's
    // remainder reduction, move and combine run -- a wave's LDS slots are
    // never idle while it computes.  g is the group in hand, g1 the next
    // (descriptors loading), g2 the one after (map entries loading); each
    // new one is claimed from the block's counter, so a wave that runs
    // faster takes more of the block's groups.
    Group G;
    SegDesc nxt = {0ull, 0u, 0u, 0u, 0u};
    SegRef ref2 = {0u, 0u};
    if constexpr (ONE && !kOneClaims) {
        // The speculative one-segment kernel: every group the same work, so
        // wave w of block b keeps round 3's static share, groups
        // g0 + j stride (the set its claims k = w, w + WPB, ... name, gid
        // without the reversed rounds), in the grid-stride loop of round 3.
        // (The claiming loop below compiled for ONE ran one-line groups
        // 15 % slower -- 64-byte messages 95 against 82 us, 128 B 70 against
        // 64, 256 B 50.7 against 49.5 -- with claims, list and layout each
        // ruled out, profiles/r04/ab/small_msgs/.)
        const uint32_t stride = nbk * (uint32_t)WPB;
        uint32_t g = gfirst;
        if (g < ngroups) {
            const uint32_t s0 = g * 64u + (uint32_t)lane;
            SegRef r0 = {0u, 0u};
            if (!identity) {
                r0 = map_segment(a, &pl, s0, s0 < total, identity, uni, sorted, ep);
                if (sorted) {
                    r0 = resolve_sorted(r0, s0 < total);
                }
            }
            const SegDesc d0 = identity ? spec : fetch_desc(a, r0, s0 < total);
            const uint32_t s1 = (g + stride) * 64u + (uint32_t)lane;
            const bool v1 = g + stride < ngroups && s1 < total;
            SegRef r1 = map_segment(a, &pl, s1, v1, identity, uni, sorted, ep);
            if (sorted) {
                r1 = resolve_sorted(r1, v1);
            }
            if constexpr (!kNoVgprTab) {
                nxt = fetch_desc(a, r1, v1);
            }
            const uint32_t s2 = (g + 2u * stride) * 64u + (uint32_t)lane;
            ref2 = map_segment(a, &pl, s2, g + 2u * stride < ngroups && s2 < total, identity, uni,
                               sorted, ep);
            setup(d0, g, G);
            if constexpr (kNoVgprTab) {
                // a wait the compiler sees (vmcnt(0), expcnt/lgkmcnt free)
                // before the first asm loads: nothing but this group's
                // descriptors is in flight yet, so it costs nothing
                __builtin_amdgcn_s_waitcnt(0x0F70);
            }
            issue_first_rounds(G);
            early_tables();
            if constexpr (kNoVgprTab) {
                nxt = fetch_desc(a, r1, v1);  // behind the first data, not in front of it
            }
            FOLD_STAMP(2)
        } else {
            early_tables();
            early_barrier(true);
        }
        [[maybe_unused]] bool first = true;
        bool meet = kEarly;  // early_barrier owed, after the first group's fold
        [[maybe_unused]] uint32_t it = 0;
        Pending pend = {0u, 0u, 0u};
        for (; g < ngroups; g += stride) {
            if constexpr (kOnePrio != 0 && WPB == 8) {
                // The two waves of a SIMD (w and w ^ WPB/2) take the same
                // number of groups, but the older one wins every issue tie:
                // per-wave stamps put the younger four waves of every block
                // 16 % behind at the end (1M x 256 B: 57.6 against 49.5 us,
                // profiles/r05/probe/fold_trace_one_raw.txt), the SIMD then
                // left to one wave.  The one behind in groups raises its
                // priority until even (groups of two or more lines: for one-line
                // groups the exchange costs more than the balance gains).
                // Same box, HBM-resident: 2M x 256 B +3.9 %, 4M x 256 B +2 %,
                // the rest unchanged (profiles/r05/ab/one_prio_ab.jsonl).
                // 8-wave blocks only: a 4-wave block's partner wave is in
                // another block (two per CU) or absent (one per CU).
                if (kOnePrio == 1 || G.R >= 2u) {
                    if (lane == 0) {
                        one_prog[wave] = it;
                    }
                    const uint32_t other = one_prog[wave ^ ((uint32_t)WPB / 2u)];
                    if (it > other) {
                        __builtin_amdgcn_s_setprio(0);
                    } else {
                        __builtin_amdgcn_s_setprio(1);
                    }
                    ++it;
                }
            }
            uint32_t Rm[32];
            fold_rounds(G, Rm);
            if (meet) {  // (fold_rounds ended on vmcnt(0): this wave's tables are in)
                early_barrier(false);
                meet = false;
            }
#if BMQCRC_FOLD_DIAG
            if (first) {
                FOLD_STAMP(3)
                first = false;
            }
            if (g + stride >= ngroups) {
                FOLD_STAMP(4)
            }
#endif
            const Group C = G;
            if (g + stride < ngroups) {
                setup(nxt, g + stride, G);
                const uint32_t s2 = (g + 2u * stride) * 64u + (uint32_t)lane;
                const bool v2 = g + 2u * stride < ngroups && s2 < total;
                nxt = fetch_desc(a, sorted ? resolve_sorted(ref2, v2) : ref2, v2);
                const uint32_t s3 = (g + 3u * stride) * 64u + (uint32_t)lane;
                ref2 = map_segment(a, &pl, s3, g + 3u * stride < ngroups && s3 < total, identity,
                                   uni, sorted, ep);
                issue_first_rounds(G);
            }
            // the previous group's results, after the next group's loads
            commit(pend);
            if (BMQCRC_ONE_DIAG & 1) {  // diagnostic: no remainder step (wrong CRCs)
                uint32_t x = 0;
#pragma unroll
                for (int d = 0; d < 32; ++d) {
                    x ^= Rm[d];
                }
                pend = finish(C, x);
            } else {
                pend = finish(C, remainder(Rm, C.hskip != 0u, C.R == 1u));
            }
        }
        commit(pend);
    } else {
    uint32_t g = kTwoEnded ? claim() : gid(wave), g1 = ngroups, g2 = ngroups;  // (= gfirst)
    if (g < ngroups) {
        g1 = claim();
        g2 = g1 < ngroups ? claim() : ngroups;
        const uint32_t s0 = g * 64u + (uint32_t)lane;
        SegRef r0 = {0u, 0u};
        if (!identity) {
            r0 = map_segment(a, &pl, s0, s0 < total, identity, uni, sorted, ep);
            if (sorted) {
                r0 = resolve_sorted(r0, s0 < total);
            }
        }
        // (the prologue's descriptors are gfirst's, the first claim's only
        // with one-ended claims)
        const SegDesc d0 = (identity && !kTwoEnded)
                               ? spec
                               : fetch_desc(a, identity ? SegRef{s0, 0u} : r0, s0 < total);
        const uint32_t s1 = g1 * 64u + (uint32_t)lane;
        const bool v1 = g1 < ngroups && s1 < total;
        SegRef r1 = map_segment(a, &pl, s1, v1, identity, uni, sorted, ep);
        if (sorted) {
            r1 = resolve_sorted(r1, v1);
        }
        nxt = fetch_desc(a, r1, v1);
        const uint32_t s2 = g2 * 64u + (uint32_t)lane;
        ref2 = map_segment(a, &pl, s2, g2 < ngroups && s2 < total, identity, uni, sorted, ep);
        setup(d0, g, G);
        issue_first_rounds(G);
        FOLD_STAMP(2)
    }
    bool first_group = true;
    Pending pend = {0u, 0u, 0u};
    while (g < ngroups) {
        // the claim of the group after g2, issued before this group's fold
        // (whose LDS reads cover the atomic's latency), taken below
        const bool more = g1 < ngroups && g2 < ngroups;  // claims only grow: none left
        const unsigned long long k3 = more ? claim_issue() : 0ull;
        uint32_t Rm[32];
        fold_rounds(G, Rm);
        if (first_group) {
            FOLD_STAMP(3)
            first_group = false;
        }
        if (g1 >= ngroups) {
            FOLD_STAMP(4)
        }
        // The slots are read: the next group's first rounds go out now, so
        // they load while this group's remainder is reduced and combined.
        const Group C = G;
        uint32_t g3 = ngroups;
        if (g1 < ngroups) {
            // setup first: it reads the descriptors loaded a group ago, and the
            // compiler's wait for them (which cannot see the DMA waits above)
            // must not also wait for the loads issued next
            setup(nxt, g1, G);
            const uint32_t s2 = g2 * 64u + (uint32_t)lane;
            const bool v2 = g2 < ngroups && s2 < total;
            nxt = fetch_desc(a, sorted ? resolve_sorted(ref2, v2) : ref2, v2);
            g3 = more ? claim_take(k3) : ngroups;
            const uint32_t s3 = g3 * 64u + (uint32_t)lane;
            ref2 = map_segment(a, &pl, s3, g3 < ngroups && s3 < total, identity, uni, sorted, ep);
            issue_first_rounds(G);
        }
        commit(pend);  // the previous group's results, after the next group's loads
        pend = finish(C, remainder(Rm, C.hskip != 0u, C.R == 1u));
        g = g1;
        g1 = g2;
        g2 = g3;
    }
    commit(pend);
    }
    FOLD_STAMP(5)
    if constexpr (ONE && !kOneClaims) {
        if (long_seen) {
            second_pass(0u);
        }
    } else if (spec_mode) {
        __syncthreads();  // the block's list of groups with skipped messages is complete
        const uint32_t nlong = long_n;
        if (nlong) {
            second_pass(nlong);
        }
    }
    FOLD_STAMP(6)
}

// ---------------------------------------------------------------- planner
// Two classes per octave of the line count (1, 2, 3, 4-5, 6-7, 8-11, 12-15,
// ..., 128-191, >= 192): lanes of a wave differ by at most 1.5x in rounds.
// 16 buckets cover the default 16 KiB segments (<= 129 lines).
__device__ __forceinline__ uint32_t size_class(uint32_t nl)
{
    nl |= 1u;
    const uint32_t b = 31u - __clz(nl);
    const uint32_t c = b ? 2u * b + ((nl >> (b - 1u)) & 1u) : 0u;
    return c < kBuckets - 1 ? c : kBuckets - 1;
}

// Segments of a message (offset off, length len) and the size class of its
// last (or only) one.  Every other segment spans exactly seg_bytes / 128
// lines (internal boundaries are 128-byte aligned and seg_bytes is a multiple
// of 128), so it is in class size_class(seg_bytes / 128).
__device__ __forceinline__ uint32_t msg_segments(const BatchArgs& a, uint64_t off, uint32_t len,
                                                 uint32_t seg_shift, uint32_t* c_last)
{
    *c_last = kBuckets;  // kBuckets: no segment
    if (len == 0) {
        return 0;
    }
    const uint32_t SEG = a.seg_bytes;
    const uint32_t nseg = (seg_shift ? ((len - 1u) >> seg_shift) : (len - 1u) / SEG) + 1u;
    // seg_geom's line count of the last segment in 32-bit arithmetic: it
    // depends only on the segment's start offset in its line (the message's
    // for k = 0, else 0: internal boundaries are line-aligned) and its
    // length D = E - S (for k > 0: len - k SEG + the message's offset in its
    // line), both < 2^31 (tests/test_fold_model.py::test_last_segment_class)
    const uint32_t k = nseg - 1u;
    const uint32_t s0 = ((uint32_t)(uintptr_t)a.arena + (uint32_t)off) & 127u;
    const uint32_t s = k ? 0u : s0;
    const uint32_t D = k ? len - (seg_shift ? k << seg_shift : k * SEG) + s0 : len;
    const uint32_t dn = (k == 0u && D < 4u) ? 4u : D;
    const uint32_t pe = (s + dn + 15u) & ~15u;
    const uint32_t nl_r = (pe - (s & ~15u) + 127u) >> 7;
    const uint32_t nl_l = (s + dn + 127u) >> 7;
    *c_last = size_class((kRightAlign && (nl_r < nl_l || nl_r <= kRightAlignLines)) ? nl_r : nl_l);
    return nseg;
}

// Lengths and offsets of messages i0 .. i0 + kPlanV - 1: one planner
// thread's quad of a tile.  A whole quad inside [lo, hi) is one dwordx4 load
// of lengths and two of offsets (the dword form, lanes 16 bytes apart, issued
// 4x the requests); any other quad loads zeros from g_zero_line, and the
// batch's last, partial quad (hi = n, n % 4 != 0) is patched from LDS where
// it is used (PlanTail).  No branch around the loads: a quad assembled in a
// branch made the compiler copy registers at the join, which waited for the
// loads there and serialized a block's tiles (phase 1 at ~4 us per tile,
// profiles/r03/ab/planner_stamps/).
struct Quad {
    u32x4 l;
    u64x2 o0, o1;
};

struct PlanTail {  // LDS: the last 1-3 messages of the batch, in the block that owns them
    uint64_t off[kPlanV - 1];
    uint32_t len[kPlanV - 1];
};

__device__ __forceinline__ Quad load_quad(const BatchArgs& a, uint64_t i0, uint64_t hi,
                                          bool offsets = true)
{
    static_assert(kPlanV == 4, "quad loads");
    const bool whole = i0 + kPlanV <= hi;
    const uint32_t* lp = whole ? a.lengths + i0 : (const uint32_t*)g_zero_line;
    const uint64_t* op = (whole && offsets) ? a.offsets + i0 : (const uint64_t*)g_zero_line;
    Quad q;
    q.l = *(const u32x4e*)lp;
    q.o0 = *(const u64x2e*)op;
    q.o1 = *(const u64x2e*)(op + 2);
    return q;
}

// Thread 0 of the block whose range ends the batch with a partial quad
// (before the block's first barrier).
__device__ __forceinline__ void load_tail(const BatchArgs& a, uint64_t hi, bool offsets,
                                          PlanTail* t)
{
    if (threadIdx.x == 0 && hi == a.n && (hi & 3u)) {
        const uint64_t i0 = hi & ~3ull;
        for (uint32_t v = 0; v < (uint32_t)(hi & 3u); ++v) {
            t->len[v] = a.lengths[i0 + v];
            t->off[v] = offsets ? a.offsets[i0 + v] : 0ull;
        }
    }
}

__device__ __forceinline__ void unpack_quad(const Quad& q, uint64_t i0, uint64_t hi,
                                            const PlanTail* t, uint32_t (&L)[kPlanV],
                                            uint64_t (&O)[kPlanV])
{
    L[0] = q.l.x;
    L[1] = q.l.y;
    L[2] = q.l.z;
    L[3] = q.l.w;
    O[0] = q.o0.x;
    O[1] = q.o0.y;
    O[2] = q.o1.x;
    O[3] = q.o1.y;
    if (i0 < hi && i0 + kPlanV > hi) {  // the batch's partial last quad
#pragma unroll
        for (uint32_t v = 0; v < kPlanV - 1; ++v) {
            if (i0 + v < hi) {
                L[v] = t->len[v];
                O[v] = t->off[v];
            }
        }
    }
}

// seg_first (exclusive prefix from r) and out[] initialisation of one
// planner thread's quad: one dwordx4 store each for a whole quad, out only
// when the quad holds a message of other than one segment.  out gets 0 for
// every non-empty message (a one-segment message is stored whole by its lane
// in k_fold, later on the stream; others XOR-accumulate from 0) and the seed
// for an empty one.
__device__ __forceinline__ void store_quad(const BatchArgs& a, uint64_t i0, uint64_t hi,
                                           const uint32_t (&L)[kPlanV], const uint32_t (&ns)[kPlanV],
                                           uint32_t r, bool write_sf)
{
    uint32_t sf[kPlanV], o[kPlanV];
#pragma unroll
    for (uint32_t v = 0; v < kPlanV; ++v) {
        sf[v] = r;
        r += ns[v];
        o[v] = 0u;
        if (L[v] == 0u && a.seeds && i0 + v < hi) {
            o[v] = a.seeds[i0 + v];
        }
    }
    if (i0 + kPlanV <= hi) {
        if (write_sf) {
            *(u32x4e*)(a.seg_first + i0) = u32x4{sf[0], sf[1], sf[2], sf[3]};
        }
        if ((ns[0] != 1u) | (ns[1] != 1u) | (ns[2] != 1u) | (ns[3] != 1u)) {
            *(u32x4e*)(a.out + i0) = u32x4{o[0], o[1], o[2], o[3]};
        }
        return;
    }
#pragma unroll
    for (uint32_t v = 0; v < kPlanV; ++v) {
        if (i0 + v < hi) {
            if (write_sf) {
                a.seg_first[i0 + v] = sf[v];
            }
            if (ns[v] != 1u) {
                a.out[i0 + v] = o[v];
            }
        }
    }
}

// K1: segment counts per message, the block-local exclusive prefix over the
// block's contiguous message range (seg_first), out[] initialisation, and
// three words per block (segments, messages with != 1 segment, the common
// segment count or ~0) that the consumer kernels reduce in their prologues
// (plan_totals).  No grid-wide step here.  Each thread takes kPlanV
// consecutive messages (a tile = 4096 messages, one block scan) and the next
// tile's lengths are loaded before the current tile is scanned, so a block
// pays one load latency, not one per tile.
template <bool CLASSES>
__global__ __launch_bounds__(kPlanBlock) void k_plan(BatchArgs a)
{
    __shared__ uint32_t wsum[40];
    __shared__ uint32_t sh[4];
    __shared__ uint32_t hist[kBuckets];
    __shared__ unsigned long long segs64;  // the block's segments without wrapping
    __shared__ PlanTail tail;
    constexpr bool classes = CLASSES;  // a ragged batch is expected: size-class histogram
    load_tail(a, min((uint64_t)blockIdx.x * a.per_msg + a.per_msg, a.n), classes, &tail);
    if (threadIdx.x == 0) {
        sh[1] = 0;            // messages with != 1 segment
        sh[2] = 0xffffffffu;  // min segments per message
        sh[3] = 0;            // max segments per message
        segs64 = 0;
    }
    if (threadIdx.x < kBuckets) {
        hist[threadIdx.x] = 0;
    }
    __syncthreads();
    constexpr uint64_t kTile = (uint64_t)kPlanBlock * kPlanV;
    const uint64_t lo = (uint64_t)blockIdx.x * a.per_msg;
    const uint64_t hi = min(lo + a.per_msg, a.n);
    const uint32_t seg = a.seg_bytes;
    const uint32_t seg_shift = (seg & (seg - 1u)) == 0 ? (uint32_t)__builtin_ctz(seg) : 0u;
    auto load = [&](uint64_t base) {
        return load_quad(a, base + (uint64_t)threadIdx.x * kPlanV, hi, classes);
    };
    Quad nq;
    if (lo < hi) {
        nq = load(lo);
    }
    uint32_t full = 0;  // this thread's non-last segments (all of class c_full)
    // A single-tile block (<= 4096 messages: every batch of <= 1M messages)
    // writes seg_first only if its messages differ in segment count; for a
    // uniform block consumers compute it (seg_first_g).
    const bool one_tile = hi - lo <= kTile;
    uint32_t carry = 0, mn = 0xffffffffu, mx = 0, non1 = 0;
    uint64_t mine64 = 0;  // this thread's segments (u32 tile scans may wrap: see kSegLimit)
    uint32_t ns[kPlanV], run0 = 0;
    for (uint64_t base = lo; base < hi; base += kTile) {
        uint32_t L[kPlanV];
        uint64_t O[kPlanV];
        unpack_quad(nq, base + (uint64_t)threadIdx.x * kPlanV, hi, &tail, L, O);
        if (base + kTile < hi) {
            nq = load(base + kTile);  // next tile in flight during this scan
        }
        if (classes) {
            // class of each message's last (or only) segment: one
            // returnless LDS atomic per message (a ballot and a conditional
            // atomic per class and wave measured 43 against 26 us on Zipf 4M)
#pragma unroll
            for (uint32_t v = 0; v < kPlanV; ++v) {
                uint32_t c;
                const uint32_t nseg = msg_segments(a, O[v], L[v], seg_shift, &c);
                full += nseg ? nseg - 1u : 0u;
                if (c < (uint32_t)kBuckets) {
                    atomicAdd(&hist[c], 1u);
                }
            }
        }
        uint32_t sum = 0;
#pragma unroll
        for (uint32_t v = 0; v < kPlanV; ++v) {
            const uint64_t i = base + (uint64_t)threadIdx.x * kPlanV + v;
            const uint32_t len = L[v];
            ns[v] = len ? (seg_shift ? ((len - 1u) >> seg_shift) : (len - 1u) / seg) + 1u : 0u;
            if (i < hi) {
                mn = min(mn, ns[v]);
                mx = max(mx, ns[v]);
                non1 += ns[v] != 1u ? 1u : 0u;
            }
            sum += ns[v];
        }
        mine64 += sum;
        uint32_t excl;
        const uint32_t tot = block_scan(sum, &excl, wsum);
        run0 = carry + excl;
        // seg_first (multi-tile blocks; a single tile's waits for the block's
        // shape below) and out[]
        store_quad(a, base + (uint64_t)threadIdx.x * kPlanV, hi, L, ns, run0, !one_tile);
        carry += tot;
    }
    // block-level min / max / count(!=1): wave reductions, then LDS atomics
    mn = wave_min(mn);
    mx = wave_max(mx);
    non1 = wave_sum(non1);
    if (classes) {
        full = wave_sum(full);
    }
    mine64 = wave_sum64(mine64);
    if ((threadIdx.x & 63) == 0) {
        atomicMin(&sh[2], mn);
        atomicMax(&sh[3], mx);
        atomicAdd(&sh[1], non1);
        atomicAdd(&segs64, (unsigned long long)mine64);
        if (full) {
            atomicAdd(&hist[size_class(seg >> 7)], full);
        }
    }
    __syncthreads();
    if (classes && threadIdx.x < kBuckets) {  // read by k_plan_sort (kernel boundary)
        a.bhist[(uint64_t)blockIdx.x * kBuckets + threadIdx.x] = hist[threadIdx.x];
    }
    if (one_tile && sh[2] != sh[3]) {
        uint32_t sf[kPlanV], run = run0;
#pragma unroll
        for (uint32_t v = 0; v < kPlanV; ++v) {
            sf[v] = run;
            run += ns[v];
        }
        const uint64_t i0 = lo + (uint64_t)threadIdx.x * kPlanV;
        if (i0 + kPlanV <= hi) {
            *(u32x4e*)(a.seg_first + i0) = u32x4{sf[0], sf[1], sf[2], sf[3]};
        } else {
#pragma unroll
            for (uint32_t v = 0; v < kPlanV; ++v) {
                if (i0 + v < hi) {
                    a.seg_first[i0 + v] = sf[v];
                }
            }
        }
    }
    if (threadIdx.x == 0) {  // read by the next launches (kernel boundary: plain stores)
        a.block_sum[blockIdx.x] = segs64 > kSegLimit ? 0xffffffffu : carry;
        a.block_sum[a.nblocks + blockIdx.x] = sh[1];
        a.block_sum[2u * a.nblocks + blockIdx.x] = sh[2] == sh[3] ? sh[2] : 0xffffffffu;
    }
}

// Lengths and offsets of a planner tile: kPlanV messages per thread, message
// base + v * kPlanBlock + threadIdx.x (coalesced per v).  The next tile is
// loaded while the current one is processed, so a block waits for one load
// latency, not one per tile.
struct TileDesc {
    uint64_t off[kPlanV];
    uint32_t len[kPlanV];
};

__device__ __forceinline__ void load_tile(const BatchArgs& a, uint64_t base, uint64_t hi,
                                          TileDesc& t)
{
#pragma unroll
    for (uint32_t v = 0; v < kPlanV; ++v) {
        const uint64_t i = base + (uint64_t)v * kPlanBlock + threadIdx.x;
        t.len[v] = i < hi ? a.lengths[i] : 0u;
        t.off[v] = i < hi ? a.offsets[i] : 0ull;
    }
}

// seginfo entries (round 3: 4 bytes per segment, was 8).  A message's last
// (or only) segment is stored as msg | kSegLast -- k_fold takes k from its
// length.  A full segment is stored as msg; its k is its distance from the
// head of its run (a message's full segments are one contiguous run, k
// ascending), and for a run that began in an earlier group of 64 the k of
// the group's first entry comes from firstk[group], written here by whoever
// writes an entry at a multiple of 64.
__device__ __forceinline__ void put_full(const BatchArgs& a, uint32_t pos, uint32_t msg, uint32_t k)
{
    a.seginfo[pos] = msg;
    if ((pos & 63u) == 0) {
        a.firstk[pos >> 6] = k;
    }
}

__device__ __forceinline__ void put_last(const BatchArgs& a, uint32_t pos, uint32_t msg)
{
    a.seginfo[pos] = msg | kSegLast;
}

// K3 (ragged batches): write (message, k) of every segment into seginfo in
// size-class order.  Each block fills its slice of every bucket (offsets from
// K2); a message's non-last segments go to one contiguous run (same class),
// so they stay adjacent in a wave and combine before their one atomic.
// Positions inside a block's slice are claimed with wave-aggregated LDS
// atomics: the order within a bucket may differ between runs, the CRCs do not
// (XOR combine).
// Runs of at most kShortRun full segments are written by their own lane
// (one claim each); longer runs by the whole wave, lane by lane.  Zipf 4M:
// 61.5 us with every run walked by the wave, 52 with 4-segment short runs,
// 49.5 with 8, 51.4 with 16 (same-box A/B, profiles/r02/ab/).
constexpr uint32_t kShortRun = 8u;
constexpr uint32_t kMapShortRun = 16u;  // k_plan_map: runs the wave writes through its search

__global__ __launch_bounds__(kPlanBlock) void k_plan_sort(BatchArgs a)
{
    __shared__ uint32_t run[kBuckets];
    __shared__ uint32_t part[2][kPlanBlock / kBuckets][kBuckets];
    __shared__ PlanLds pl;
    const PlanTotals pt = plan_totals(a, &pl);
    if (pt.identity || pt.uni || pt.overflow || pt.total > a.max_segs) {
        return;  // closed form, overflow, or more segments than seginfo holds (k_fold searches)
    }
    const int lane = threadIdx.x & 63;
    // This block's slice of every bucket, from k_plan's per-block histograms
    // (bhist[block][class]): bucket-major order, so slice(c) starts at the
    // segments of all smaller classes plus class c of the earlier blocks.
    {
        static_assert(kPlanBlock % kBuckets == 0, "bucket-base reduction layout");
        constexpr uint32_t kParts = kPlanBlock / kBuckets;
        const uint32_t c = threadIdx.x % kBuckets, pi = threadIdx.x / kBuckets;
        uint32_t tot = 0, pre = 0;
        for (uint32_t b = pi; b < a.nblocks; b += kParts) {
            const uint32_t h = a.bhist[(uint64_t)b * kBuckets + c];
            tot += h;
            pre += b < blockIdx.x ? h : 0u;
        }
        part[0][pi][c] = tot;
        part[1][pi][c] = pre;
        __syncthreads();
        if (threadIdx.x < kBuckets) {
            uint32_t t = 0, q = 0;
            for (uint32_t p = 0; p < kParts; ++p) {
                t += part[0][p][threadIdx.x];
                q += part[1][p][threadIdx.x];
            }
            part[0][0][threadIdx.x] = t;
            part[1][0][threadIdx.x] = q;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t acc = 0;
            for (int cc = 0; cc < kBuckets; ++cc) {
                run[cc] = acc + part[1][0][cc];
                acc += part[0][0][cc];
            }
        }
        __syncthreads();
    }
    const uint32_t SEG = a.seg_bytes;
    const uint32_t seg_shift = (SEG & (SEG - 1u)) == 0 ? (uint32_t)__builtin_ctz(SEG) : 0u;
    const uint32_t c_full = size_class(SEG >> 7);
    const uint64_t lo = (uint64_t)blockIdx.x * a.per_msg;
    const uint64_t hi = min(lo + a.per_msg, a.n);
    constexpr uint64_t kTile = (uint64_t)kPlanBlock * kPlanV;
    TileDesc nxt;
    if (lo < hi) {
        load_tile(a, lo, hi, nxt);
    }
    for (uint64_t base = lo; base < hi; base += kTile) {
        const TileDesc cur = nxt;
        if (base + kTile < hi) {
            load_tile(a, base + kTile, hi, nxt);
        }
        uint32_t c[kPlanV], nseg[kPlanV], nf_all = 0;
#pragma unroll
        for (uint32_t v = 0; v < kPlanV; ++v) {
            nseg[v] = msg_segments(a, cur.off[v], cur.len[v], seg_shift, &c[v]);
            const uint32_t nf = nseg[v] ? nseg[v] - 1u : 0u;
            if (nf && nf <= kShortRun) {
                // a short run of full segments: its lane claims and writes it
                const uint32_t at = atomicAdd(&run[c_full], nf);
                const uint32_t i = (uint32_t)(base + (uint64_t)v * kPlanBlock + threadIdx.x);
                for (uint32_t k = 0; k < nf; ++k) {
                    put_full(a, at + k, i, k);
                }
            } else {
                nf_all += nf;
            }
        }
        // long runs of full segments: one contiguous run per message in class
        // c_full, one LDS atomic per wave and tile
        uint32_t x = nf_all;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)x, o);
            if (lane >= o) {
                x += y;
            }
        }
        const uint32_t tf = (uint32_t)__shfl((int)x, 63);
        if (tf) {
            uint32_t pos = 0;
            if (lane == 0) {
                pos = atomicAdd(&run[c_full], tf);
            }
            pos = (uint32_t)__shfl((int)pos, 0) + (x - nf_all);
            // the whole wave writes each lane's runs in turn (coalesced),
            // instead of every lane looping over its own runs while the
            // others wait on the longest
            const uint32_t lane0 = threadIdx.x & ~63u;
            for (uint64_t busy = __ballot(nf_all != 0u); busy; busy &= busy - 1ull) {
                const int src = __builtin_ctzll(busy);
                uint32_t at = (uint32_t)__builtin_amdgcn_readlane((int)pos, src);
#pragma unroll
                for (uint32_t v = 0; v < kPlanV; ++v) {
                    const uint32_t nfv = nseg[v] ? nseg[v] - 1u : 0u;
                    const uint32_t nf = (uint32_t)__builtin_amdgcn_readlane(
                        (int)(nfv > kShortRun ? nfv : 0u), src);
                    const uint32_t i =
                        (uint32_t)(base + (uint64_t)v * kPlanBlock + lane0 + (uint32_t)src);
                    for (uint32_t k = (uint32_t)lane; k < nf; k += 64u) {
                        put_full(a, at + k, i, k);
                    }
                    at += nf;
                }
            }
        }
        // last (or only) segments: a returning LDS atomic per message claims
        // its slot in its class (the order inside a bucket is free; a ballot,
        // an atomic and a shuffle per class and wave measured 73 against 61 us
        // on Zipf 4M)
#pragma unroll
        for (uint32_t v = 0; v < kPlanV; ++v) {
            if (c[v] < (uint32_t)kBuckets) {
                const uint64_t i = base + (uint64_t)v * kPlanBlock + threadIdx.x;
                put_last(a, atomicAdd(&run[c[v]], 1u), (uint32_t)i);
            }
        }
    }
}

// ------------------------------------------------ single-pass planner
// k_plan_map (ragged batches, round 3): one launch does what k_plan<true>
// and k_plan_sort did in two.  Phase 1 (every block, its contiguous message
// range): segment counts, the size-class histogram and the block-local
// prefix, kept in registers; the block words and the histogram are published.
// The blocks then meet once, grid-wide; after that every block reads all
// histograms and writes the rest: (message, k) of its segments into its
// slice of every class -- exactly k_plan_sort's global class-major order --
// plus seg_first and the out[] initialisation, which phase 1 defers (they
// are not needed before the wait, and the deferred stores are one dwordx4
// per quad).  (A block-major
// order -- each block's slice sorted by class, offsets by a decoupled
// look-back, no grid-wide wait -- was measured first: k_fold's grid-stride
// waves then draw a binomial mix of 16-round and 1-round groups, and Zipf's
// k_fold ran 7 % slower, profiles/r03/ab/ab1_*.jsonl.)
//
// Safety of the wait: the host sizes the grid to what the GPU holds at once
// (occupancy x CUs), but nothing guarantees residency (other streams, other
// processes).  A block that has waited map_wait_ticks (bmqcrc_plan_wait)
// without seeing every arrival marks the map invalid for this launch
// (plan_sync[2] = epoch, plan_sync[3] counts such launches) and leaves; a
// block that finds the map already given up leaves at once.  Every block
// writes seg_first and the out[] initialisation in every path, so k_fold
// then maps segments by searching seg_first (message order instead of
// size-class order: exact, somewhat slower).  Arrival flags carry the
// launch's epoch, so nothing needs resetting between launches.
#ifndef BMQCRC_MAP_REG_TILES
#define BMQCRC_MAP_REG_TILES 4
#endif
constexpr uint32_t kMapRegTiles = BMQCRC_MAP_REG_TILES;  // tiles kept in registers across the wait
#ifndef BMQCRC_CLASS_DESC
#define BMQCRC_CLASS_DESC 0  // size-class order in seginfo: 0 by BatchArgs::class_desc (product),
                             // 1 always descending, 2 always ascending (A/B builds)
#endif
#ifndef BMQCRC_PLAN_SKIP
#define BMQCRC_PLAN_SKIP 0  // timing diagnostics with the map voided (wrong maps, exact CRCs):
                            // 1 no histogram atomics, 2 no last-segment claims, 4 no full-run
                            // writes, 8 no last-segment stores, 16 no long-run writes, 32 no
                            // short-run writes, 64 full-run slots mapped but not stored
#endif
#ifndef BMQCRC_PLAN_FLAGS
#define BMQCRC_PLAN_FLAGS 0  // 1: round 3's separate arrival flags (A/B)
#endif
#ifndef BMQCRC_PLAN_DIAG
#define BMQCRC_PLAN_DIAG 0  // 3: per-block phase stamps, 4: the same without seginfo stores,
                            // 6: every block's first read of the exchanged words is stale
                            // (timing diagnostics, tools/plan_trace_diag.py); product: 0
#endif

#if BMQCRC_PLAN_DIAG >= 3
// diagnostic build only: per-block wall-clock stamps of the last launch
// (start, first loads landed, first tile counted, phase 1 done, wait done,
// deferred writes issued, class bases done, end), read by
// bmqcrc_diag_plan_trace
__device__ unsigned long long g_plan_trace[kPlanMaxBlocks][8];
#define PLAN_STAMP(k)                                                        \
    if (threadIdx.x == 0) {                                                  \
        g_plan_trace[blockIdx.x][k] = wall_clock64();                        \
    }
#define PLAN_STAMP_LANDED(k)                                                 \
    if (threadIdx.x == 0) {                                                  \
        __builtin_amdgcn_s_waitcnt(0);                                       \
        g_plan_trace[blockIdx.x][k] = wall_clock64();                        \
    }
#else
#define PLAN_STAMP(k)
#define PLAN_STAMP_LANDED(k)
#endif

__global__ __launch_bounds__(kPlanBlock) void k_plan_map(BatchArgs a)
{
    PLAN_STAMP(0)
    __shared__ uint32_t wsum[40];
    __shared__ uint32_t sh[4];
    __shared__ uint32_t hist[kBuckets];
    __shared__ uint32_t run[kBuckets];
    __shared__ uint32_t part[2][2][kBuckets];  // per wave: class totals / prefix, block words
    __shared__ unsigned long long segs64;
    __shared__ uint32_t go;
    __shared__ PlanTail tail;
    __shared__ uint32_t sruns[kPlanBlock / 64][64 * kPlanV];  // per wave: short-run ends
#if BMQCRC_LONG_FLAT
    __shared__ uint32_t slong[kPlanBlock / 64][2][64 * kPlanV];  // per wave: long runs' starts, lengths
    __shared__ uint32_t smark[kPlanBlock / 64][64];             // per wave: item-run starts in a chunk
#endif
    const uint32_t nb = a.nblocks, ep = launch_epoch(a), bid = blockIdx.x;
    load_tail(a, min((uint64_t)bid * a.per_msg + a.per_msg, a.n), true, &tail);
    // epoch-tagged words the blocks exchange (plan_sync after the flags),
    // laid out for coalesced reads: [c * kPlanMaxBlocks + b] histograms,
    // [kTagWords + i * kPlanMaxBlocks + b] block words
    unsigned long long* const tags = a.plan_sync + kSyncFlags + kPlanMaxBlocks;
    constexpr uint32_t kTagWords = kPlanMaxBlocks * kBuckets;
    // mark this launch's map given up (one thread): k_fold folds every
    // message whole; the first block to give up counts the launch
    auto give_up = [&]() {
        if (__hip_atomic_exchange(&a.plan_sync[2], (unsigned long long)ep, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT) != ep) {
            __hip_atomic_fetch_add(&a.plan_sync[3], 1ull, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
    };
    unsigned long long* const sync = a.plan_sync;
    if (threadIdx.x == 0) {
        sh[1] = 0;            // messages with != 1 segment
        sh[2] = 0xffffffffu;  // min segments per message
        sh[3] = 0;            // max segments per message
        segs64 = 0;
    }
    if (threadIdx.x < kBuckets) {
        hist[threadIdx.x] = 0;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    constexpr uint64_t kTile = (uint64_t)kPlanBlock * kPlanV;
    const uint64_t lo = (uint64_t)bid * a.per_msg;
    const uint64_t hi = min(lo + a.per_msg, a.n);
    const uint32_t ntiles = hi > lo ? (uint32_t)((hi - lo + kTile - 1) / kTile) : 0u;
    const uint32_t seg = a.seg_bytes;
    const uint32_t seg_shift = (seg & (seg - 1u)) == 0 ? (uint32_t)__builtin_ctz(seg) : 0u;
    const uint32_t c_full = size_class(seg >> 7);
    const bool one_tile = ntiles <= 1u;
    auto segments = [&](uint32_t len) {
        return len ? (seg_shift ? ((len - 1u) >> seg_shift) : (len - 1u) / seg) + 1u : 0u;
    };

    // Thread t of tile [base, base + kTile) owns messages base + 4t .. base + 4t + 3.
    auto load = [&](uint32_t t) {
        return load_quad(a, lo + (uint64_t)t * kTile + (uint64_t)threadIdx.x * kPlanV, hi);
    };
    // seg_first (the block-local prefix from run0) and out[] for one tile
    auto tile_words = [&](uint64_t base, const uint32_t (&L)[kPlanV], uint32_t run0,
                          bool write_sf) {
        uint32_t ns[kPlanV];
#pragma unroll
        for (uint32_t v = 0; v < kPlanV; ++v) {
            ns[v] = segments(L[v]);
        }
        store_quad(a, base + (uint64_t)threadIdx.x * kPlanV, hi, L, ns, run0, write_sf);
    };
    // Phase 1.  The first kMapRegTiles tiles are loaded at once (all in
    // flight together) and keep their lengths, classes and prefix in
    // registers, deferring their writes; later tiles load one ahead and
    // write as k_plan does.
    uint32_t Lr[kMapRegTiles][kPlanV], Cr[kMapRegTiles], R0[kMapRegTiles];
    uint32_t full = 0, carry = 0, mn = 0xffffffffu, mx = 0, non1 = 0;
    uint64_t mine64 = 0;
    Quad rq[kMapRegTiles];
#pragma unroll
    for (uint32_t t = 0; t < kMapRegTiles; ++t) {
        rq[t] = load(t);  // unguarded: a tile past the range loads the zero line
    }
    auto count_tile = [&](uint32_t t, const Quad& q, uint32_t (&L)[kPlanV], uint32_t& cls,
                          uint32_t& run0, bool defer) {
        const uint64_t base = lo + (uint64_t)t * kTile;
        uint64_t O[kPlanV];
        unpack_quad(q, base + (uint64_t)threadIdx.x * kPlanV, hi, &tail, L, O);
        if (t == 0) {
            PLAN_STAMP_LANDED(1)
        }
        cls = 0;
        uint32_t sum = 0;
#pragma unroll
        for (uint32_t v = 0; v < kPlanV; ++v) {
            uint32_t c;
            const uint32_t ns = msg_segments(a, O[v], L[v], seg_shift, &c);
            full += ns ? ns - 1u : 0u;
            if (c < (uint32_t)kBuckets && !(BMQCRC_PLAN_SKIP & 1)) {
                atomicAdd(&hist[c], 1u);
            }
            cls |= c << (8u * v);  // kBuckets (no segment) fits a byte
            const uint64_t i = base + (uint64_t)threadIdx.x * kPlanV + v;
            if (i < hi) {
                mn = min(mn, ns);
                mx = max(mx, ns);
                non1 += ns != 1u ? 1u : 0u;
            }
            sum += ns;
        }
        mine64 += sum;
        uint32_t excl;
        const uint32_t tot = block_scan(sum, &excl, wsum);
        run0 = carry + excl;
        carry += tot;
        if (!defer) {
            tile_words(base, L, run0, true);
        }
        if (t == 0) {
            PLAN_STAMP(2)
        }
    };
#pragma unroll
    for (uint32_t t = 0; t < kMapRegTiles; ++t) {
        if (t < ntiles) {
            count_tile(t, rq[t], Lr[t], Cr[t], R0[t], true);
        }
    }
    if (ntiles > kMapRegTiles) {
        Quad nq = load(kMapRegTiles);
        for (uint32_t t = kMapRegTiles; t < ntiles; ++t) {
            const Quad q = nq;
            if (t + 1u < ntiles) {
                nq = load(t + 1u);  // the next tile in flight during this one
            }
            uint32_t L[kPlanV], c, r0;
            count_tile(t, q, L, c, r0, false);
        }
    }
    // wave reductions by DPP (the bpermute butterflies were a 6-deep chain
    // of LDS round trips per value)
    mn = wave_min(mn);
    mx = wave_max(mx);
    non1 = wave_sum(non1);
    full = wave_sum(full);
    mine64 = wave_sum64(mine64);
    if ((threadIdx.x & 63) == 0) {
        atomicMin(&sh[2], mn);
        atomicMax(&sh[3], mx);
        atomicAdd(&sh[1], non1);
        atomicAdd(&segs64, (unsigned long long)mine64);
        if (full) {
            atomicAdd(&hist[c_full], full);
        }
    }
    __syncthreads();
    // a single-tile block whose messages all have the same segment count
    // leaves seg_first to the consumers (seg_first_g), as in k_plan
    const bool write_sf = !one_tile || sh[2] != sh[3];
    // the register tiles' deferred writes: out[], and seg_first when there
    // is no map to use
    auto deferred = [&](bool sf) {
#pragma unroll
        for (uint32_t t = 0; t < kMapRegTiles; ++t) {
            if (t < ntiles) {
                tile_words(lo + (uint64_t)t * kTile, Lr[t], R0[t], sf && write_sf);
            }
        }
    };
    // Publish the block words and the histogram, then arrive and wait.
    PLAN_STAMP(3)
    if (threadIdx.x < 64) {
        // Wave 0 publishes the block words and the histogram as
        // device-scope 64-bit stores, each word tagged with this launch's
        // epoch (they write through to memory, visible on every XCD once
        // complete), waits for them, then arrives: one flag word per block,
        // set to the epoch.  The readers load everything with device-scope
        // loads and check every word's tag, reading a stale one again, so no
        // visibility order is assumed between the flag and the words and
        // neither side needs an agent-scope fence (an L2 write-back /
        // invalidate: ~3 us of the wait, profiles/r03/ab/planner_stamps/).
        // No shared counter -- 256 atomics on one word serialize at the
        // memory side (11-16 us measured,
        // profiles/r03/ab/planner_phases_counter_wait/) -- and no reset: a
        // word of an older launch holds an older epoch.
        const unsigned long long tagv = (unsigned long long)ep << 32;
        if (lane < kBuckets) {
            __hip_atomic_store(&tags[lane * kPlanMaxBlocks + bid], tagv | hist[lane],
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane < 3) {
            const uint32_t wv = lane == 0   ? (segs64 > kSegLimit ? 0xffffffffu : carry)
                                : lane == 1 ? sh[1]
                                            : (sh[2] == sh[3] ? sh[2] : 0xffffffffu);
            __hip_atomic_store(&tags[kTagWords + lane * kPlanMaxBlocks + bid], tagv | wv,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            a.block_sum[lane * nb + bid] = wv;  // for k_fold (the next launch)
        }
#if BMQCRC_PLAN_FLAGS
        __builtin_amdgcn_s_waitcnt(0);  // the stores above are complete (vmcnt 0)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) {
            __hip_atomic_store(&sync[kSyncFlags + bid], (unsigned long long)ep, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        // poll the blocks' arrival flags
        const unsigned long long* const arrive = sync + kSyncFlags;
        constexpr int kArriveShift = 0;
#else
        // round 4: no separate flag.  The poll reads each block's tagged
        // third block word (published beside its histogram, in no particular
        // order: the tag check below re-reads any word still stale), so the
        // wait for the stores' completion and the flag's own store and
        // visibility latency are gone from the meeting.
        const unsigned long long* const arrive = tags + kTagWords + 2u * kPlanMaxBlocks;
        constexpr int kArriveShift = 32;
#endif
        const uint64_t t0 = wall_clock64();
        uint32_t ok = 1u;
        static_assert(kPlanMaxBlocks <= 4 * 64, "four flags per lane");
        // a zero limit gives the map up before the first poll (the test hook
        // of bmqcrc_plan_wait(0): every such launch takes the fallback)
        bool waiting = a.map_wait_ticks != 0;
        if (!waiting) {
            ok = 0u;
            if (lane == 0) {
                give_up();
            }
        }
        while (waiting) {
            // all four loads in flight at once (a short-circuit chain made
            // them four round trips per poll), plus the launch's give-up word:
            // a block arriving after another gave the map up leaves at once
            // instead of waiting out its own limit
            unsigned long long f[4];
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) {
                const uint32_t b = (uint32_t)lane + 64u * k;
                f[k] = b < nb ? __hip_atomic_load(&arrive[b], __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT) >> kArriveShift
                              : (unsigned long long)ep;
            }
            const unsigned long long gone =
                __hip_atomic_load(&sync[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const bool mine = f[0] == ep && f[1] == ep && f[2] == ep && f[3] == ep;
            if (__ballot(!mine) == 0) {
                break;
            }
            if (gone == (unsigned long long)ep) {
                ok = 0u;  // another block gave this launch's map up
                break;
            }
            if (wall_clock64() - t0 >= a.map_wait_ticks) {
                ok = 0u;  // not all blocks running: give up the map, keep correctness
                if (lane == 0) {
                    give_up();
                }
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        if (lane == 0) {
            go = ok;
        }
    }
    __syncthreads();
    PLAN_STAMP(4)
    // false: no map for k_fold (given up, or a closed form / past capacity
    // below); it then searches seg_first, and multi-segment messages
    // XOR-combine into out[] -- both written by deferred() in every path
    bool map = go != 0;
    // Batch shape and size from every block's words (closed-form batches
    // and those past seginfo's capacity or 32-bit indices need no map), and
    // this block's slice of every class (k_plan_sort's class-major order):
    // every load goes out at once, each wave reduces its share by DPP, and
    // one LDS exchange combines the waves.  Wave c sums class c over all
    // blocks (lane l: blocks l + 64 k); the block words are in waves 0-3.
    static_assert(kPlanBlock / 64 == kBuckets && kPlanMaxBlocks <= 4 * 64,
                  "one wave per size class, four blocks per lane");
    const uint32_t cw = threadIdx.x >> 6;
    const uint32_t j = threadIdx.x;
    uint32_t u0 = 0;
    if (map) {  // block-uniform (go is in LDS)
        const uint64_t t1 = wall_clock64();
        auto tagged = [&](const unsigned long long* p, uint32_t& val, bool& stale) {
            const unsigned long long x = __hip_atomic_load(p, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT);
            stale = stale || (uint32_t)(x >> 32) != ep;
            val = (uint32_t)x;
        };
#if BMQCRC_PLAN_DIAG == 6
        bool forced = true;  // diagnostic: the first read counts as stale (re-read path)
#endif
        while (true) {
            bool stale = false;
#if BMQCRC_PLAN_DIAG == 6
            stale = forced;
            forced = false;
#endif
            uint32_t hb[4], v = 0, nn = 0, u;
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) {
                const uint32_t b = (uint32_t)lane + 64u * k;
                hb[k] = 0u;
                if (b < nb) {
                    tagged(&tags[cw * kPlanMaxBlocks + b], hb[k], stale);
                }
            }
            tagged(&tags[kTagWords + 2u * kPlanMaxBlocks], u0, stale);
            u = u0;
            if (j < nb) {
                tagged(&tags[kTagWords + j], v, stale);
                tagged(&tags[kTagWords + kPlanMaxBlocks + j], nn, stale);
                tagged(&tags[kTagWords + 2u * kPlanMaxBlocks + j], u, stale);
            }
            uint32_t tot = 0, pre = 0;
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) {
                tot += hb[k];
                pre += (uint32_t)lane + 64u * k < bid ? hb[k] : 0u;
            }
            tot = wave_sum(tot);
            pre = wave_sum(pre);
            // (a block over the limit stores ~0: its wave's sum passes any capacity)
            const uint64_t segs = wave_sum64(v);
            const bool w_ragged = __ballot(nn != 0u) != 0, w_mixed = __ballot(u != u0) != 0;
            const bool w_stale = __ballot(stale) != 0;
            if (lane == 0) {
                part[0][0][cw] = tot;
                part[1][0][cw] = pre;
                part[0][1][cw] = (uint32_t)min(segs, (uint64_t)0xffffffffu);
                part[1][1][cw] = (w_ragged ? 1u : 0u) | (w_mixed ? 2u : 0u) | (w_stale ? 4u : 0u) |
                                 ((threadIdx.x == 0 && wall_clock64() - t1 >= a.map_wait_ticks)
                                      ? 8u : 0u);
            }
            __syncthreads();
            uint32_t f = 0;
#pragma unroll
            for (uint32_t w = 0; w < (uint32_t)kBuckets; ++w) {
                f |= part[1][1][w];
            }
            if (!(f & 4u)) {
                break;
            }
            // a word not yet visible: read again, within the same time limit
            if (f & 8u) {
                if (threadIdx.x == 0) {
                    give_up();
                }
                map = false;
                break;
            }
            __syncthreads();  // part[] read by all before the next round
        }
    }
    if (map) {
        uint32_t flags = 0;
        unsigned long long all = 0;
#pragma unroll
        for (uint32_t w = 0; w < (uint32_t)kBuckets; ++w) {
            flags |= part[1][1][w];
            all += part[0][1][w];
        }
        const bool ragged = flags & 1u, mixed = flags & 2u;
        if (!ragged || (!mixed && u0 != 0xffffffffu)) {
            map = false;  // identity or uniform: k_fold uses closed forms
        } else {
            // past seginfo's capacity: k_fold searches seg_first (or folds
            // whole messages past 32-bit segment indices)
            map = all <= min((unsigned long long)a.max_segs, (unsigned long long)kSegLimit);
        }
        if (threadIdx.x < kBuckets) {
            uint32_t acc = 0;
            const bool desc = BMQCRC_CLASS_DESC == 1 || (BMQCRC_CLASS_DESC == 0 && a.class_desc);
            for (uint32_t c = 0; c < (uint32_t)kBuckets; ++c) {
                acc += (desc ? c > threadIdx.x : c < threadIdx.x) ? part[0][0][c] : 0u;
            }
            run[threadIdx.x] = acc + part[1][0][threadIdx.x];
        }
    }
    // seg_first in every path: should another block give the map up after
    // this one saw every arrival (its timer ran out between two polls),
    // k_fold searches seg_first for every segment of the batch (16 MB of
    // stores on Zipf 4M; round 3 skipped them and fell back to one lane per
    // message, a cliff of up to the longest message per wave).
    deferred(true);
    PLAN_STAMP(5)
    if (!map) {
        return;
    }
    __syncthreads();  // run[]
    PLAN_STAMP(6)
    // Phase 2: (message, k) of every segment.
    auto write_tile = [&](uint32_t t, const uint32_t (&L)[kPlanV], uint32_t cls) {
        const uint64_t base = lo + (uint64_t)t * kTile;
        // Full segments: one claim per wave for all its runs, short ones
        // (at most kMapShortRun segments) first, then long ones; each kind
        // in (lane, v) order.  The wave writes the short runs' range
        // together, 64 consecutive entries per store: slot j finds its run
        // by a binary search over the runs' ends, staged in LDS.  (Each lane
        // writing its own runs issued up to 4 kShortRun scattered stores per
        // tile: 16 of the planner's 58 us on Zipf 4M,
        // profiles/r03/ab/planner_stamps/sk1_component_skips.jsonl.)
        // Each long run is written by the whole wave, coalesced.
        uint32_t nf[kPlanV], ns_all = 0, nl_all = 0;
#pragma unroll
        for (uint32_t v = 0; v < kPlanV; ++v) {
            const uint32_t nseg = segments(L[v]);
            nf[v] = nseg ? nseg - 1u : 0u;
            ns_all += nf[v] <= kMapShortRun ? nf[v] : 0u;
            nl_all += nf[v] > kMapShortRun ? nf[v] : 0u;
        }
        const uint32_t xs = wave_incl_scan(ns_all), xl = wave_incl_scan(nl_all);
        const uint32_t ts = (uint32_t)__builtin_amdgcn_readlane((int)xs, 63);
        const uint32_t tl = (uint32_t)__builtin_amdgcn_readlane((int)xl, 63);
        if (ts + tl) {
            uint32_t pos = 0;
            if (lane == 0) {
                pos = atomicAdd(&run[c_full], ts + tl);
            }
            pos = (uint32_t)__builtin_amdgcn_readfirstlane((int)pos);
#if BMQCRC_PLAN_DIAG != 4 && !(BMQCRC_PLAN_SKIP & 4)
            const uint32_t w = threadIdx.x >> 6;
            const uint64_t wbase = base + (uint64_t)(threadIdx.x & ~63u) * kPlanV;
            if (ts && !(BMQCRC_PLAN_SKIP & 32)) {
                uint32_t e = xs - ns_all, ends[kPlanV];
#pragma unroll
                for (uint32_t v = 0; v < kPlanV; ++v) {
                    e += nf[v] <= kMapShortRun ? nf[v] : 0u;
                    ends[v] = e;
                }
                *(u32x4*)&sruns[w][lane * kPlanV] = u32x4{ends[0], ends[1], ends[2], ends[3]};
                for (uint32_t j = (uint32_t)lane; j < ts; j += 64u) {
                    uint32_t q = 0;  // runs ending at or before j
#pragma unroll
                    for (uint32_t st = 32u * kPlanV; st; st >>= 1) {
                        q += sruns[w][q + st - 1u] <= j ? st : 0u;
                    }
                    const uint32_t k = j - (q ? sruns[w][q - 1u] : 0u);
#if BMQCRC_PLAN_SKIP & 64
                    if (k == 0xfffffff0u) {  // never: keeps the slot's search live
                        a.firstk[0] = q;
                    }
#else
                    put_full(a, pos + j, (uint32_t)(wbase + q), k);
#endif
                }
            }
            uint64_t longs = 0;
#pragma unroll
            for (uint32_t v = 0; v < kPlanV; ++v) {
                longs |= __ballot(nf[v] > kMapShortRun);
            }
            if (BMQCRC_PLAN_SKIP & 16) {
                longs = 0;
            }
            const uint32_t lpos = pos + ts + (xl - nl_all);
#if BMQCRC_LONG_FLAT
            if (longs) {
                // Every long run of the wave at once: its head and tail
                // entries (the partial groups at either end) are one list of
                // items over the wave, its whole groups another, each walked
                // 64 items per store.  (Run by run, a wave issued two to four
                // partly filled stores per run, and the long runs' stores
                // were 5.3 of the 1/8 shard's 21.5 us planner,
                // profiles/r05/ab/planner/phase_stamps_fullrun_split.jsonl.)
                // An item finds its run by a mark at the run's first item and
                // a max-scan over the wave (run indices grow with their
                // items); a wave's LDS operations complete in order, so
                // marks, reads and clearing need no barrier.  The shard's
                // planner 21.6 -> 20.7 us traced, the whole batch flat
                // (profiles/r05/ab/planner/long_flat_ab.jsonl): the bytes
                // stored, not the store count, are what remains.
                uint32_t atv[kPlanV], nv[kPlanV], ni[kPlanV], ng[kPlanV];
                uint32_t p = lpos;
#pragma unroll
                for (uint32_t v = 0; v < kPlanV; ++v) {
                    const uint32_t n = nf[v] > kMapShortRun ? nf[v] : 0u;
                    const uint32_t gf = (p + 63u) >> 6, ge = (p + n) >> 6;
                    const bool whole = kGroupDesc && gf < ge;
                    atv[v] = p;
                    nv[v] = n;
                    if constexpr (kRunRecords) {
                        // entries only for a run inside one group touching
                        // neither of its ends; a run's head (the group's
                        // last lanes) and tail (its first lanes) are records
                        const bool inner = n && (p >> 6) == ((p + n - 1u) >> 6) && (p & 63u) &&
                                           ((p + n) & 63u);
                        ni[v] = inner ? n : 0u;
                    } else {
                        ni[v] = whole ? (64u * gf - p) + (p + n - 64u * ge) : n;
                    }
                    ng[v] = whole ? ge - gf : 0u;
                    p += n;
                }
                *(u32x4*)&slong[w][0][lane * kPlanV] = u32x4{atv[0], atv[1], atv[2], atv[3]};
                *(u32x4*)&slong[w][1][lane * kPlanV] = u32x4{nv[0], nv[1], nv[2], nv[3]};
                if constexpr (kRunRecords) {
                    // Run records (round 6): a long run's partial groups
                    // are described per group, not per slot -- its head
                    // (lanes ho..63 of group at/64) by the group's suffix
                    // record, its tail (lanes 0..te-1 of the last group) by
                    // the prefix record and firstk; each side of a group has
                    // one owner (the run covering lane 63, or lane 0).
                    // Round 5 wrote up to 63 + 63 entries per long run, ~3 MB
                    // on Zipf's 1/8 shard: 5.3 of its planner's 20.7 us
                    // (profiles/r05/ab/planner/phase_stamps_fullrun_split.jsonl).
#pragma unroll
                    for (uint32_t v = 0; v < kPlanV; ++v) {
                        const uint32_t at = atv[v], n = nv[v];
                        if (n == 0u) {
                            continue;
                        }
                        const uint32_t hb = at >> 6, tb = (at + n - 1u) >> 6;
                        const uint32_t ho = at & 63u, te = (at + n) & 63u;
                        const uint32_t msg = (uint32_t)(wbase + (uint32_t)lane * kPlanV + v);
                        if (ho != 0u && (hb < tb || te == 0u)) {
                            *(u32x4*)&a.grec[8u * hb + 4u] = u32x4{ep, msg, 64u - ho, 0u};
                        }
                        if (te != 0u && (hb < tb || ho == 0u)) {
                            *(u32x4*)&a.grec[8u * tb] = u32x4{ep, msg, te, 0u};
                            a.firstk[tb] = 64u * tb - at;
                        }
                    }
                }
                auto flat = [&](const uint32_t (&cnt)[kPlanV], auto&& body) {
                    const uint32_t mine = cnt[0] + cnt[1] + cnt[2] + cnt[3];
                    const uint32_t x = wave_incl_scan(mine);
                    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
                    uint32_t s0 = x - mine, st[kPlanV];
#pragma unroll
                    for (uint32_t v = 0; v < kPlanV; ++v) {
                        st[v] = cnt[v] ? s0 : 0xffffffffu;
                        s0 += cnt[v];
                    }
                    *(u32x4*)&sruns[w][lane * kPlanV] = u32x4{st[0], st[1], st[2], st[3]};
                    smark[w][lane] = 0u;
                    uint32_t open = 0u;
                    for (uint32_t j0 = 0; j0 < total; j0 += 64u) {
#pragma unroll
                        for (uint32_t v = 0; v < kPlanV; ++v) {
                            if (st[v] - j0 < 64u) {
                                smark[w][st[v] - j0] = (uint32_t)lane * kPlanV + v + 1u;
                            }
                        }
                        uint32_t o = smark[w][lane];
                        smark[w][lane] = 0u;
                        o = max(wave_incl_max(o), open);
                        open = (uint32_t)__builtin_amdgcn_readlane((int)o, 63);
                        const uint32_t j = j0 + (uint32_t)lane;
                        if (j < total) {
                            const uint32_t q = o - 1u;  // o >= 1: a run's items start at 0
                            body(q, j - sruns[w][q]);
                        }
                    }
                };
                if (!(BMQCRC_PLAN_SKIP & 64)) {
                    flat(ni, [&](uint32_t q, uint32_t e) {
                        const uint32_t at = slong[w][0][q], n = slong[w][1][q];
                        const uint32_t gf = (at + 63u) >> 6, ge = (at + n) >> 6;
                        const uint32_t h = kGroupDesc && gf < ge ? 64u * gf - at : n;
                        const uint32_t slot = e < h ? at + e : 64u * ge + (e - h);
                        put_full(a, slot, (uint32_t)(wbase + q), slot - at);
                    });
                    if (kGroupDesc) {
                        flat(ng, [&](uint32_t q, uint32_t e) {
                            const uint32_t at = slong[w][0][q];
                            const uint32_t g = ((at + 63u) >> 6) + e;
                            a.gdesc[g] = (unsigned long long)ep << 32 | (uint32_t)(wbase + q);
                            a.firstk[g] = 64u * g - at;
                        });
                    }
                }
            }
#else
            for (; longs; longs &= longs - 1ull) {
                const int src = __builtin_ctzll(longs);
                uint32_t at2 = (uint32_t)__builtin_amdgcn_readlane((int)lpos, src);
#pragma unroll
                for (uint32_t v = 0; v < kPlanV; ++v) {
                    const uint32_t n = (uint32_t)__builtin_amdgcn_readlane((int)nf[v], src);
                    if (n > kMapShortRun) {
                        const uint32_t i = (uint32_t)(wbase + (uint32_t)src * kPlanV + v);
                        // groups wholly inside [at2, at2 + n): one tagged
                        // descriptor each (and its firstk) instead of 64
                        // entries; the entries of the partial groups at
                        // either end as before
                        const uint32_t gf = (at2 + 63u) >> 6, ge = (at2 + n) >> 6;
                        const uint32_t kh = kGroupDesc && gf < ge ? 64u * gf - at2 : n;
                        const uint32_t kt = kGroupDesc && gf < ge ? 64u * ge - at2 : n;
                        for (uint32_t k = (uint32_t)lane; k < kh && !(BMQCRC_PLAN_SKIP & 64); k += 64u) {
                            put_full(a, at2 + k, i, k);
                        }
                        if (kGroupDesc && !(BMQCRC_PLAN_SKIP & 64)) {
                            const unsigned long long tag = (unsigned long long)ep << 32 | i;
                            for (uint32_t g = gf + (uint32_t)lane; g < ge; g += 64u) {
                                a.gdesc[g] = tag;
                                a.firstk[g] = 64u * g - at2;
                            }
                        }
                        for (uint32_t k = kt + (uint32_t)lane; k < n && !(BMQCRC_PLAN_SKIP & 64); k += 64u) {
                            put_full(a, at2 + k, i, k);
                        }
                        at2 += n;
                    }
                }
            }
#endif
#endif
        }
        // last (or only) segments: one returning LDS atomic per message
#pragma unroll
        for (uint32_t v = 0; v < kPlanV; ++v) {
            const uint32_t c = (cls >> (8u * v)) & 0xffu;
            if (c < (uint32_t)kBuckets) {
                const uint64_t i = base + (uint64_t)threadIdx.x * kPlanV + v;
#if BMQCRC_PLAN_SKIP & 2
                const uint32_t at = run[c] + (uint32_t)threadIdx.x * kPlanV + v;
#else
                const uint32_t at = atomicAdd(&run[c], 1u);
#endif
#if BMQCRC_PLAN_DIAG != 4 && !(BMQCRC_PLAN_SKIP & 8)
                put_last(a, at, (uint32_t)i);
#else
                (void)at;
                (void)i;
#endif
            }
        }
    };
#pragma unroll
    for (uint32_t t = 0; t < kMapRegTiles; ++t) {
        if (t < ntiles) {
            write_tile(t, Lr[t], Cr[t]);
        }
    }
    for (uint32_t t = kMapRegTiles; t < ntiles; ++t) {
        uint32_t L[kPlanV];
        uint64_t O[kPlanV];
        unpack_quad(load(t), lo + (uint64_t)t * kTile + (uint64_t)threadIdx.x * kPlanV, hi, &tail,
                    L, O);
        uint32_t cls = 0;
#pragma unroll
        for (uint32_t v = 0; v < kPlanV; ++v) {
            uint32_t c;
            (void)msg_segments(a, O[v], L[v], seg_shift, &c);
            cls |= c << (8u * v);
        }
        write_tile(t, L, cls);
    }
    __syncthreads();
    PLAN_STAMP(7)
#if BMQCRC_PLAN_DIAG == 4 || BMQCRC_PLAN_SKIP
    // diagnostic (timing only): no seginfo stores, so no map
    if (threadIdx.x == 0) {
        __hip_atomic_store(&sync[2], (unsigned long long)ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#endif
}

// ------------------------------------------------- verify / blob combine
// Mismatch detection for journal recovery: count and record indices
// (unordered; the host sorts the short list).
__global__ void k_compare(const uint32_t* got, const uint32_t* expected, uint64_t n,
                          uint32_t* bad_count, uint32_t* bad_idx, uint32_t bad_cap)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        if (got[i] != expected[i]) {
            const uint32_t slot = atomicAdd(bad_count, 1u);
            if (slot < bad_cap) {
                bad_idx[slot] = (uint32_t)i;
            }
        }
    }
}

// Ordered mismatch list, used when more messages mismatch than the caller's
// bad_cap: block b owns indices [b*chunk, (b+1)*chunk); pass 1 counts its
// mismatches, the host scans the counts, pass 2 writes each mismatch at its
// global rank so the list holds exactly the bad_cap LOWEST indices (the
// reference's walks stop at / report the first corrupt record).
__global__ void k_compare_count(const uint32_t* got, const uint32_t* expected, uint64_t n,
                                uint64_t chunk, uint32_t* block_cnt)
{
    const uint64_t lo = (uint64_t)blockIdx.x * chunk;
    const uint64_t hi = min(n, lo + chunk);
    uint32_t cnt = 0;
    for (uint64_t base = lo; base < hi; base += blockDim.x) {
        const uint64_t i = base + threadIdx.x;
        cnt += __syncthreads_count(i < hi && got[i] != expected[i]);
    }
    if (threadIdx.x == 0) {
        block_cnt[blockIdx.x] = cnt;
    }
}

// Ranks [skip, skip + bad_cap) of the ordered list go to bad_idx[rank - skip]
// (the host takes a long list in windows of a fixed device buffer).
__global__ void k_compare_emit(const uint32_t* got, const uint32_t* expected, uint64_t n,
                               uint64_t chunk, const uint32_t* block_off, uint32_t* bad_idx,
                               uint32_t skip, uint32_t bad_cap)
{
    __shared__ uint32_t wave_cnt[16];
    const uint64_t lo = (uint64_t)blockIdx.x * chunk;
    const uint64_t hi = min(n, lo + chunk);
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t nwaves = blockDim.x >> 6;
    uint32_t run = block_off[blockIdx.x];
    const uint64_t end = (uint64_t)skip + bad_cap;
    for (uint64_t base = lo; base < hi && run < end; base += blockDim.x) {
        const uint64_t i = base + threadIdx.x;
        const bool bad = i < hi && got[i] != expected[i];
        const uint64_t m = __ballot(bad);
        const uint32_t below = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        if (lane == 0) {
            wave_cnt[wave] = (uint32_t)__popcll(m);
        }
        __syncthreads();
        uint32_t before = run, total = 0;
        for (uint32_t w = 0; w < nwaves; ++w) {
            before += (w < wave) ? wave_cnt[w] : 0u;
            total += wave_cnt[w];
        }
        const uint64_t rank = (uint64_t)before + below;
        if (bad && rank >= skip && rank < end) {
            bad_idx[rank - skip] = (uint32_t)i;
        }
        run += total;
        __syncthreads();
    }
}

// Blob chaining (bmqp_crc32c.cpp:47-67): acc = seed; for each buffer j of
// blob m: acc = calculate(buf_j, acc) = acc * x^(8 len_j) ^ crc0(buf_j).
// x^e is applied with the 31 constant matrices (per-lane, no ballots: the
// trip counts differ between lanes).
__device__ uint32_t mul_xpow_lane(uint32_t v, uint32_t e)
{
    for (int j = 0; j < 31; ++j) {
        if ((e >> j) & 1u) {
            uint32_t a0 = 0, a1 = 0;
#pragma unroll
            for (int t = 0; t < 32; t += 2) {
                a0 = xand(a0, bitmask(v, t), c_x2col[j][t]);
                a1 = xand(a1, bitmask(v, t + 1), c_x2col[j][t + 1]);
            }
            v = a0 ^ a1;
        }
    }
    return v;
}

__global__ void k_blob_combine(const uint32_t* buf_crc, const uint32_t* buf_len,
                               const uint64_t* msg_first_buf, const uint32_t* seeds,
                               uint32_t* out, uint64_t n)
{
    for (uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; m < n;
         m += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t acc = seeds ? seeds[m] : 0u;
        const uint64_t b1 = msg_first_buf[m + 1];
        for (uint64_t b = msg_first_buf[m]; b < b1; ++b) {
            const uint32_t len = buf_len[b];
            if (len) {
                acc = mul_xpow_lane(acc, mersenne31(8ull * len)) ^ buf_crc[b];
            }
        }
        out[m] = acc;
    }
}

// ------------------------------------------------------- synthetic payload
__device__ __forceinline__ uint64_t splitmix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// byte i of the payload stream = byte (i % 8) of splitmix64(seed*golden + i/8);
// identical to oracle_fill_payload().  dst must be 8-byte aligned.
__global__ void k_fill(uint8_t* dst, uint64_t nbytes, uint64_t seed, uint64_t begin)
{
    const uint64_t nw = nbytes >> 3;
    const uint64_t key = seed * 0x9E3779B97F4A7C15ull + (begin >> 3);
    uint64_t* d64 = (uint64_t*)dst;
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw;
         w += (uint64_t)gridDim.x * blockDim.x) {
        d64[w] = splitmix64(key + w);
    }
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < (nbytes & 7)) {
        const uint64_t g = (nw << 3) + t;
        dst[g] = (uint8_t)(splitmix64(key + (g >> 3)) >> (8 * (g & 7)));  // begin % 8 == 0
    }
}

}  // namespace bmqcrc

using namespace bmqcrc;

extern "C" int bmqcrc_launch_batch(const BatchArgs* a, void* stream, int num_cus, void* ev_start,
                                   void* ev_stop)
{
    hipStream_t s = (hipStream_t)stream;
    if (a->n == 0) {
        return 0;
    }
    if (!a->whole && !a->spec && a->map_planned && a->plan_epoch == 0) {
        // whichever planner runs: k_fold's sorted path takes a gdesc word in
        // place of seginfo when its tag equals the launch's, so a captured
        // pair-planned batch needs a tag no earlier word carries too (left at
        // plan_sync[1] it could be 0 -- every zeroed word -- or the tag of an
        // earlier captured k_plan_map whose words name stale messages)
        hipLaunchKernelGGL(k_epoch_advance, dim3(1), dim3(1), 0, s, a->plan_sync);
    }
    if (!a->whole && !a->spec) {
        // Ragged batch expected: the single-pass planner when its blocks
        // hold more than one tile (it keeps them in registers across its
        // grid-wide wait instead of reloading them); with one tile per block
        // the round-2 pair is as fast (Zipf's 1/8 shard: 26.5 against 27.8
        // us traced; the whole batch 75.3 against 70.2 us,
        // profiles/r03/ab/planner_traces.txt).
        const bool single_pass = single_pass_planner(*a);
        if (a->map_planned && single_pass) {
            hipLaunchKernelGGL(k_plan_map, dim3(a->nblocks), dim3(kPlanBlock), 0, s, *a);
        } else if (a->map_planned) {
            hipLaunchKernelGGL(k_plan<true>, dim3(a->nblocks), dim3(kPlanBlock), 0, s, *a);
        } else {
            hipLaunchKernelGGL(k_plan<false>, dim3(a->nblocks), dim3(kPlanBlock), 0, s, *a);
        }
        if (a->map_planned && !single_pass) {
            hipLaunchKernelGGL(k_plan_sort, dim3(a->nblocks), dim3(kPlanBlock), 0, s, *a);
        }
    }
    const uint64_t max_groups = (a->max_segs + 63) / 64;
    const uint32_t per_cu = (a->tune & 2u) ? 1u : (a->tune & 8u) ? 2u : a->blocks_per_cu;
    const uint64_t cus = (uint64_t)(num_cus > 0 ? num_cus : 256);
    // Two waves per SIMD as ONE block of 8 waves per CU whose waves claim
    // the block's groups dynamically, when the batch gives every wave at
    // least two groups; otherwise (one wave per SIMD, or small batches that
    // should reach more CUs) 4-wave blocks, per_cu of them per CU.
    const bool wide = per_cu == 2u && !(a->tune & 1024u) && max_groups >= 2u * 8u * cus;
    const uint32_t wpb = wide ? 8u : 4u;
    uint64_t grid = (max_groups + wpb - 1) / wpb;
    const uint64_t cap = wide ? cus : cus * (per_cu ? per_cu : 2u);
    if (grid > cap) {
        grid = cap;
    }
    if (grid < 1) {
        grid = 1;
    }
    if (ev_start) {
        (void)hipEventRecord((hipEvent_t)ev_start, s);
    }
    const bool one = a->spec == 1u && !a->whole && !(a->tune & 64u);
    // few groups: one per block over every CU first (BatchArgs::spread)
    BatchArgs b = *a;
    b.spread = 0u;
    if (kSpread && !wide && grid < cus && max_groups > grid) {
        grid = std::min<uint64_t>(max_groups, cus);
        b.spread = 1u;
    }
    const dim3 gd((unsigned)grid), bd(wpb * 64u);
    if (a->tune & 1u) {  // A/B: default-policy LDS-DMA for long streams too
        if (wide) {
            hipLaunchKernelGGL((k_fold<false, false, 8>), gd, bd, 0, s, b);
        } else {
            hipLaunchKernelGGL((k_fold<false, false, 4>), gd, bd, 0, s, b);
        }
    } else if (one) {  // default: non-temporal LDS-DMA for long streams (once-read)
        if (wide) {
            hipLaunchKernelGGL((k_fold<true, true, 8>), gd, bd, 0, s, b);
        } else {
            hipLaunchKernelGGL((k_fold<true, true, 4>), gd, bd, 0, s, b);
        }
    } else if (wide) {
        hipLaunchKernelGGL((k_fold<true, false, 8>), gd, bd, 0, s, b);
    } else {
        hipLaunchKernelGGL((k_fold<true, false, 4>), gd, bd, 0, s, b);
    }
    if (ev_stop) {
        (void)hipEventRecord((hipEvent_t)ev_stop, s);
    }
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int bmqcrc_plan_map_occupancy(int* blocks_per_cu)
{
    int per = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reinterpret_cast<const void*>(&k_plan_map),
                                                     kPlanBlock, 0) != hipSuccess) {
        return -5;
    }
    *blocks_per_cu = per;
    return 0;
}

#if BMQCRC_FOLD_DIAG
extern "C" __attribute__((visibility("default"))) int bmqcrc_diag_fold_trace(unsigned long long* out)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fold_trace), sizeof(g_fold_trace)) == hipSuccess
               ? 0
               : -5;
}
#endif

#if BMQCRC_PLAN_DIAG >= 3
extern "C" __attribute__((visibility("default"))) int bmqcrc_diag_plan_trace(unsigned long long* out)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_plan_trace), sizeof(g_plan_trace)) == hipSuccess
               ? 0
               : -5;
}
#endif

extern "C" int bmqcrc_launch_compare(const uint32_t* got, const uint32_t* expected, uint64_t n,
                                     uint32_t* bad_count, uint32_t* bad_idx, uint32_t bad_cap,
                                     void* stream)
{
    if (n == 0) {
        return 0;
    }
    const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_compare, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, got,
                       expected, n, bad_count, bad_idx, bad_cap);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int bmqcrc_launch_compare_ordered(const uint32_t* got, const uint32_t* expected,
                                            uint64_t n, uint32_t* block_cnt, uint32_t nblocks,
                                            uint32_t* bad_idx, uint32_t skip, uint32_t bad_cap,
                                            int pass, void* stream)
{
    if (n == 0 || nblocks == 0) {
        return 0;
    }
    const uint64_t chunk = (n + nblocks - 1) / nblocks;
    if (pass == 0) {
        hipLaunchKernelGGL(k_compare_count, dim3(nblocks), dim3(256), 0, (hipStream_t)stream,
                           got, expected, n, chunk, block_cnt);
    } else {
        hipLaunchKernelGGL(k_compare_emit, dim3(nblocks), dim3(256), 0, (hipStream_t)stream, got,
                           expected, n, chunk, block_cnt, bad_idx, skip, bad_cap);
    }
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int bmqcrc_launch_blob_combine(const uint32_t* buf_crc, const uint32_t* buf_len,
                                         const uint64_t* msg_first_buf, const uint32_t* seeds,
                                         uint32_t* out, uint64_t n, void* stream)
{
    if (n == 0) {
        return 0;
    }
    const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_blob_combine, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                       buf_crc, buf_len, msg_first_buf, seeds, out, n);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int bmqcrc_launch_fill(uint8_t* dst, uint64_t nbytes, uint64_t seed, uint64_t begin,
                                  void* stream)
{
    if (nbytes == 0) {
        return 0;
    }
    uint64_t blocks = (nbytes / 8 + 255) / 256;
    if (blocks > 65536) {
        blocks = 65536;
    }
    if (blocks < 1) {
        blocks = 1;
    }
    hipLaunchKernelGGL(k_fill, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, dst,
                       nbytes, seed, begin);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}
