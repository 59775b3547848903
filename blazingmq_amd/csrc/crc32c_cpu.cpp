// crc32c_cpu.cpp -- host-CPU scalar CRC32C behind the unchanged
// bmqp::Crc32c::calculate(const void*, unsigned, unsigned) signature
// (/root/reference/src/groups/bmq/bmqp/bmqp_crc32c.h:244-246).
//
// The reference answers a single-buffer call synchronously on the calling
// thread (bmqp_crc32c.cpp:41-45 -> BDE, SSE4.2 when available).  A single
// buffer is latency-bound, so the scalar path stays on the CPU; the GPU serves
// batches (bmqcrc_crc32c_batch).  It must not be slower than what it replaces
// at any size (bmqp_crc32c.h:109-132 publishes the reference's per-size
// times), so the buffer length picks the method:
//   * with AVX-512 VPCLMULQDQ, from kFoldMin bytes: carry-less folding of
//     64-byte accumulators (four of them, 256 bytes per step, from 256 bytes),
//     reduced to 16 bytes that two crc32q finish;
//   * without it, from kThreeWayMin bytes: three crc32q chains over the
//     buffer's thirds, stitched with two carry-less multiplies -- one pass,
//     one stitch, the lane length chosen per call;
//   * shorter buffers: one crc32q chain (3-cycle latency per word);
//   * no SSE4.2: slicing-by-8 tables.
//
// Representation.  A CRC register is "reflected": bit j holds the coefficient
// of x^(31-j).  A carry-less product of two such values has bit m on
// x^(62-m); read by crc32q as a message word (bit m on x^(63-m), then times
// x^32) it gives a*b*x^33 mod P.  So with K = x^(e-33) mod P,
// crc32q(0, clmul(c, K)) = c * x^e mod P: the register shifted over e/8 zero
// bytes, in two instructions.  The folding constants follow the same rule
// (derivation in DESIGN.md, "Scalar CRC").
#include <stdint.h>
#include <string.h>

#include "../../include/bmqcrc.h"

#if defined(__x86_64__)
#include <cpuid.h>
#include <immintrin.h>
#endif

namespace bmqcrc {
namespace {

constexpr uint32_t kPoly = 0x82F63B78u;  // 0x1EDC6F41 reflected
constexpr uint32_t kOne = 1u << 31;      // x^0
constexpr uint32_t kFoldMin = 256;       // bytes, with AVX-512 VPCLMULQDQ (EPYC 9575F: serial
                                         // crc32q is faster to 224 B, profiles/r05/scalar)
constexpr uint32_t kThreeWayMin = 256;   // bytes, without it ("Scalar CRC")
constexpr uint32_t kMaxLane = 4096;      // longest 3-way lane (bytes): 12 KiB per stitch

uint32_t gf2_mul(uint32_t a, uint32_t b)  // a*b mod P (init only)
{
    uint32_t p = 0;
    for (uint32_t m = kOne; m; m >>= 1) {
        if (a & m) {
            p ^= b;
        }
        b = (b >> 1) ^ (kPoly & (0u - (b & 1u)));
    }
    return p;
}

uint32_t div_x(uint32_t y)  // y / x mod P: P's constant term is 1, so x is invertible
{
    return (y & kOne) ? (((y ^ kPoly) << 1) | 1u) : (y << 1);
}

uint32_t xpow(int64_t e)  // x^e mod P, e may be negative (init only)
{
    uint32_t r = kOne;
    if (e < 0) {
        for (; e < 0; ++e) {
            r = div_x(r);
        }
        return r;
    }
    for (uint32_t sq = kOne >> 1; e; e >>= 1) {
        if (e & 1) {
            r = gf2_mul(r, sq);
        }
        sq = gf2_mul(sq, sq);
    }
    return r;
}

struct Tables {
    uint32_t t8[8][256];
    uint32_t lane_k[kMaxLane / 8 + 1][2];  // lane of 8i bytes: x^(8*2*8i-33), x^(8*8i-33)
    uint32_t pow2_k[64];                   // x^(8*2^k-33): cpu_combine
    uint64_t fold256[2], fold192[2], fold128[2], fold64[2], fold16[2];
    uint64_t fold_lanes[8];                // the last 64 bytes' lanes 0..2 to lane 3
    bool sse42 = false, clmul = false, avx512 = false;

    static void fold_k(uint64_t* k, uint32_t dist)  // fold a 16-byte block over dist bytes
    {
        k[0] = xpow(8ll * dist + 31);  // the block's first 8 bytes (x^64 higher)
        k[1] = xpow(8ll * dist - 33);  // its last 8 bytes
    }

    Tables()
    {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = i;
            for (int k = 0; k < 8; ++k) {
                c = (c >> 1) ^ (kPoly & (0u - (c & 1u)));
            }
            t8[0][i] = c;
        }
        for (int s = 1; s < 8; ++s) {
            for (uint32_t i = 0; i < 256; ++i) {
                t8[s][i] = (t8[s - 1][i] >> 8) ^ t8[0][t8[s - 1][i] & 0xFFu];
            }
        }
        // x^(8*8i - 33) for i = 0..512, by stepping x^64 from x^-33
        const uint32_t x64 = xpow(64);
        uint32_t k = xpow(-33);
        for (uint32_t i = 0; i <= kMaxLane / 8; ++i) {
            lane_k[i][1] = k;
            k = gf2_mul(k, x64);
        }
        for (uint32_t i = 0; 2 * i <= kMaxLane / 8; ++i) {
            lane_k[i][0] = lane_k[2 * i][1];
        }
        for (uint32_t i = kMaxLane / 16 + 1; i <= kMaxLane / 8; ++i) {
            lane_k[i][0] = gf2_mul(lane_k[i][1], xpow(64ll * i));
        }
        uint32_t p = xpow(8);  // x^(8*2^k)
        const uint32_t inv33 = xpow(-33);
        for (int b = 0; b < 64; ++b) {
            pow2_k[b] = gf2_mul(p, inv33);
            p = gf2_mul(p, p);
        }
        fold_k(fold256, 256);
        fold_k(fold192, 192);
        fold_k(fold128, 128);
        fold_k(fold64, 64);
        fold_k(fold16, 16);
        fold_k(fold_lanes + 0, 48);
        fold_k(fold_lanes + 2, 32);
        fold_k(fold_lanes + 4, 16);
        fold_lanes[6] = fold_lanes[7] = 0;
#if defined(__x86_64__)
        unsigned a, b, c, d;
        if (__get_cpuid(1, &a, &b, &c, &d)) {
            sse42 = (c & bit_SSE4_2) != 0;
            clmul = sse42 && (c & bit_PCLMUL) != 0;
            const bool osxsave = (c & bit_OSXSAVE) != 0;
            unsigned a7 = 0, b7 = 0, c7 = 0, d7 = 0;
            if (clmul && osxsave && __get_cpuid_count(7, 0, &a7, &b7, &c7, &d7)) {
                uint32_t xlo, xhi;
                __asm__("xgetbv" : "=a"(xlo), "=d"(xhi) : "c"(0));
                const bool zmm_state = (xlo & 0xE6u) == 0xE6u;  // SSE, AVX, opmask, ZMM
                avx512 = zmm_state && (b7 & bit_AVX512F) && (b7 & bit_AVX512VL) &&
                         (c7 & bit_VPCLMULQDQ);
            }
        }
#endif
    }
};

const Tables& tables()
{
    static const Tables t;
    return t;
}

uint32_t raw_soft(const Tables& T, const uint8_t* p, size_t n, uint32_t c)
{
    for (; n && (reinterpret_cast<uintptr_t>(p) & 7u); --n) {
        c = T.t8[0][(c ^ *p++) & 0xFFu] ^ (c >> 8);
    }
    for (; n >= 8; n -= 8, p += 8) {
        uint64_t w;
        memcpy(&w, p, 8);
        w ^= c;
        c = T.t8[7][w & 0xFF] ^ T.t8[6][(w >> 8) & 0xFF] ^ T.t8[5][(w >> 16) & 0xFF] ^
            T.t8[4][(w >> 24) & 0xFF] ^ T.t8[3][(w >> 32) & 0xFF] ^ T.t8[2][(w >> 40) & 0xFF] ^
            T.t8[1][(w >> 48) & 0xFF] ^ T.t8[0][w >> 56];
    }
    for (; n; --n) {
        c = T.t8[0][(c ^ *p++) & 0xFFu] ^ (c >> 8);
    }
    return c;
}

#if defined(__x86_64__)
#define BMQCRC_SSE42 __attribute__((target("sse4.2")))
#define BMQCRC_CLMUL __attribute__((target("sse4.2,pclmul")))
#define BMQCRC_AVX512 __attribute__((target("sse4.2,pclmul,avx512f,avx512vl,vpclmulqdq")))

inline uint64_t load64(const uint8_t* p)  // one unaligned scalar load
{
    uint64_t w;
    memcpy(&w, p, 8);
    return w;
}

BMQCRC_SSE42 inline uint32_t serial_tail(const uint8_t* p, size_t n, uint32_t c)  // n < 8
{
    if (n & 4) {
        uint32_t w;
        memcpy(&w, p, 4);
        c = _mm_crc32_u32(c, w);
        p += 4;
    }
    if (n & 2) {
        uint16_t w;
        memcpy(&w, p, 2);
        c = _mm_crc32_u16(c, w);
        p += 2;
    }
    if (n & 1) {
        c = _mm_crc32_u8(c, *p);
    }
    return c;
}

BMQCRC_SSE42 __attribute__((always_inline)) inline uint32_t serial_body(const uint8_t* p, size_t n,
                                                                      uint32_t c)
{
    uint64_t c64 = c;
    for (; n >= 32; n -= 32, p += 32) {
        c64 = _mm_crc32_u64(c64, load64(p));
        c64 = _mm_crc32_u64(c64, load64(p + 8));
        c64 = _mm_crc32_u64(c64, load64(p + 16));
        c64 = _mm_crc32_u64(c64, load64(p + 24));
    }
    for (; n >= 8; n -= 8, p += 8) {
        c64 = _mm_crc32_u64(c64, load64(p));
    }
    return serial_tail(p, n, (uint32_t)c64);
}

BMQCRC_SSE42 uint32_t raw_serial(const uint8_t* p, size_t n, uint32_t c)
{
    return serial_body(p, n, c);
}

// c0 * x^(8*2L) + c1 * x^(8L) + c2 with K = lane_k[L/8]: two carry-less
// multiplies and one crc32q (their sum is linear, so one reduction serves both)
BMQCRC_CLMUL inline uint32_t stitch3(const uint32_t* K, uint64_t c0, uint64_t c1, uint32_t c2)
{
    const __m128i k = _mm_set_epi64x(K[1], K[0]);
    const __m128i a = _mm_set_epi64x((long long)c1, (long long)c0);
    const __m128i m = _mm_xor_si128(_mm_clmulepi64_si128(a, k, 0x00), _mm_clmulepi64_si128(a, k, 0x11));
    return (uint32_t)_mm_crc32_u64(0, (uint64_t)_mm_cvtsi128_si64(m)) ^ c2;
}

// Three crc32q chains over consecutive lanes of L bytes (L a multiple of 8,
// at most kMaxLane), stitched once; the remainder (< 24 bytes when n fits one
// pass) runs serially.
BMQCRC_CLMUL uint32_t raw_three_way(const Tables& T, const uint8_t* p, size_t n, uint32_t c)
{
    while (n >= 24) {
        size_t lane = (n / 24) * 8;
        if (lane > kMaxLane) {
            lane = kMaxLane;
        }
        const uint8_t* p1 = p + lane;
        const uint8_t* p2 = p + 2 * lane;
        uint64_t c0 = c, c1 = 0, c2 = 0;
        size_t i = 0;
        for (; i + 16 <= lane; i += 16) {
            c0 = _mm_crc32_u64(c0, load64(p + i));
            c1 = _mm_crc32_u64(c1, load64(p1 + i));
            c2 = _mm_crc32_u64(c2, load64(p2 + i));
            c0 = _mm_crc32_u64(c0, load64(p + i + 8));
            c1 = _mm_crc32_u64(c1, load64(p1 + i + 8));
            c2 = _mm_crc32_u64(c2, load64(p2 + i + 8));
        }
        if (i < lane) {
            c0 = _mm_crc32_u64(c0, load64(p + i));
            c1 = _mm_crc32_u64(c1, load64(p1 + i));
            c2 = _mm_crc32_u64(c2, load64(p2 + i));
        }
        c = stitch3(T.lane_k[lane / 8], c0, c1, (uint32_t)c2);
        p += 3 * lane;
        n -= 3 * lane;
    }
    return raw_serial(p, n, c);
}

BMQCRC_AVX512 inline __m512i fold512(__m512i x, __m512i k, __m512i data)
{
    return _mm512_ternarylogic_epi64(_mm512_clmulepi64_epi128(x, k, 0x00),
                                     _mm512_clmulepi64_epi128(x, k, 0x11), data, 0x96);
}

BMQCRC_AVX512 inline __m128i fold128(__m128i x, __m128i k, __m128i data)
{
    return _mm_ternarylogic_epi64(_mm_clmulepi64_si128(x, k, 0x00), _mm_clmulepi64_si128(x, k, 0x11),
                                  data, 0x96);
}

BMQCRC_AVX512 inline __m512i bcast(const uint64_t* k)
{
    return _mm512_broadcast_i32x4(_mm_loadu_si128(reinterpret_cast<const __m128i*>(k)));
}

// n >= 64.  The register c enters as the first four message bytes XOR c
// (raw(c, M) = raw(0, M with c XORed into its first 32 bits)); the 16 bytes
// left after folding are finished by crc32q from 0, then the < 16 tail bytes.
// Four accumulators (256 bytes per step, independent chains) from 256 bytes,
// one below.
BMQCRC_AVX512 uint32_t raw_fold(const Tables& T, const uint8_t* p, size_t n, uint32_t c)
{
    const __m512i cz = _mm512_zextsi128_si512(_mm_cvtsi32_si128((int)c));
    __m512i x;
    if (n >= 256) {
        __m512i x0 = _mm512_xor_si512(_mm512_loadu_si512(p), cz);
        __m512i x1 = _mm512_loadu_si512(p + 64);
        __m512i x2 = _mm512_loadu_si512(p + 128);
        __m512i x3 = _mm512_loadu_si512(p + 192);
        p += 256;
        n -= 256;
        if (n >= 256) {
            const __m512i k256 = bcast(T.fold256);
            do {
                x0 = fold512(x0, k256, _mm512_loadu_si512(p));
                x1 = fold512(x1, k256, _mm512_loadu_si512(p + 64));
                x2 = fold512(x2, k256, _mm512_loadu_si512(p + 128));
                x3 = fold512(x3, k256, _mm512_loadu_si512(p + 192));
                p += 256;
                n -= 256;
            } while (n >= 256);
        }
        // four accumulators -> one: x0, x1, x2 over 192, 128, 64 bytes onto x3
        x = fold512(x0, bcast(T.fold192), x3);
        x = fold512(x1, bcast(T.fold128), x);
        x = fold512(x2, bcast(T.fold64), x);
    } else {
        x = _mm512_xor_si512(_mm512_loadu_si512(p), cz);
        p += 64;
        n -= 64;
    }
    const __m512i k64 = bcast(T.fold64);
    for (; n >= 64; n -= 64, p += 64) {
        x = fold512(x, k64, _mm512_loadu_si512(p));
    }
    // 64 bytes -> 16: lanes 0, 1, 2 over 48, 32, 16 bytes onto lane 3
    const __m512i kl = _mm512_loadu_si512(T.fold_lanes);
    const __m512i t = _mm512_xor_si512(_mm512_clmulepi64_epi128(x, kl, 0x00),
                                       _mm512_clmulepi64_epi128(x, kl, 0x11));
    __m128i a = _mm_ternarylogic_epi64(_mm512_castsi512_si128(t), _mm512_extracti32x4_epi32(t, 1),
                                       _mm512_extracti32x4_epi32(t, 2), 0x96);
    a = _mm_xor_si128(a, _mm512_extracti32x4_epi32(x, 3));
    const __m128i k16 = _mm_loadu_si128(reinterpret_cast<const __m128i*>(T.fold16));
    for (; n >= 16; n -= 16, p += 16) {
        a = fold128(a, k16, _mm_loadu_si128(reinterpret_cast<const __m128i*>(p)));
    }
    uint64_t c64 = _mm_crc32_u64(0, (uint64_t)_mm_cvtsi128_si64(a));
    c64 = _mm_crc32_u64(c64, (uint64_t)_mm_extract_epi64(a, 1));
    if (n >= 8) {
        c64 = _mm_crc32_u64(c64, load64(p));
        p += 8;
        n -= 8;
    }
    return serial_tail(p, n, (uint32_t)c64);
}

// c * x^(8*lenB) mod P with K = pow2_k: lenB's set bits, one clmul + crc32q each
BMQCRC_CLMUL uint32_t shift_clmul(const Tables& T, uint32_t c, uint64_t lenB)
{
    for (int b = 0; lenB; ++b, lenB >>= 1) {
        if (lenB & 1u) {
            const __m128i m = _mm_clmulepi64_si128(_mm_cvtsi32_si128((int)c),
                                                   _mm_cvtsi32_si128((int)T.pow2_k[b]), 0x00);
            c = (uint32_t)_mm_crc32_u64(0, (uint64_t)_mm_cvtsi128_si64(m));
        }
    }
    return c;
}
#endif

// The method per host, chosen once: short buffers run the serial chain
// inlined in the chosen function, so a call costs one predicted indirect call
// on top of the arithmetic.
using RawFn = uint32_t (*)(const uint8_t*, size_t, uint32_t);

#if defined(__x86_64__)
BMQCRC_AVX512 uint32_t raw_host_avx512(const uint8_t* p, size_t n, uint32_t c)
{
    return n < kFoldMin ? serial_body(p, n, c) : raw_fold(tables(), p, n, c);
}

BMQCRC_CLMUL uint32_t raw_host_clmul(const uint8_t* p, size_t n, uint32_t c)
{
    return n < kThreeWayMin ? serial_body(p, n, c) : raw_three_way(tables(), p, n, c);
}
#endif

uint32_t raw_host_soft(const uint8_t* p, size_t n, uint32_t c)
{
    return raw_soft(tables(), p, n, c);
}

RawFn pick_raw()
{
    const Tables& T = tables();
#if defined(__x86_64__)
    if (T.avx512) {
        return raw_host_avx512;
    }
    if (T.clmul) {
        return raw_host_clmul;
    }
    if (T.sse42) {
        return raw_serial;
    }
#endif
    (void)T;
    return raw_host_soft;
}

// Set at load time (g_init); a call from another static initializer that
// runs first picks it itself (the same value, so the race is benign).
RawFn g_raw = nullptr;

__attribute__((noinline, cold)) RawFn init_raw()
{
    const RawFn f = pick_raw();
    __atomic_store_n(&g_raw, f, __ATOMIC_RELAXED);
    return f;
}

struct Init {
    Init() { init_raw(); }
} g_init;

}  // namespace

uint32_t cpu_crc32c(const void* data, uint32_t length, uint32_t crc)
{
    if (length == 0) {
        return crc;
    }
    RawFn f = __atomic_load_n(&g_raw, __ATOMIC_RELAXED);
    if (__builtin_expect(f == nullptr, 0)) {
        f = init_raw();
    }
    return ~f(static_cast<const uint8_t*>(data), length, ~crc);
}

uint32_t cpu_combine(uint32_t crcA, uint32_t crcB, uint64_t lenB)
{
    const Tables& T = tables();
#if defined(__x86_64__)
    if (T.clmul) {
        return shift_clmul(T, crcA, lenB) ^ crcB;
    }
#endif
    uint32_t sq = xpow(8), r = crcA;  // x^(8*2^b), squared per bit of lenB
    for (; lenB; lenB >>= 1) {
        if (lenB & 1u) {
            r = gf2_mul(r, sq);
        }
        sq = gf2_mul(sq, sq);
    }
    return r ^ crcB;
}

}  // namespace bmqcrc

#if !defined(BMQCRC_CPU_AB)
// The scalar entry points of include/bmqcrc.h (defined here so the
// reference-signature call bmqp::Crc32c::calculate -> bmqcrc_crc32c reaches
// the arithmetic through one indirect call).
extern "C" {

uint32_t bmqcrc_crc32c(const void* data, uint32_t length, uint32_t crc)
{
    return bmqcrc::cpu_crc32c(data, length, crc);
}

uint32_t bmqcrc_crc32c_blob(const void* const* bufs, const uint32_t* lens, uint32_t nbuf,
                            uint32_t crc)
{
    // bmqp_crc32c.cpp:47-67: an empty blob returns crc; otherwise chain.
    for (uint32_t i = 0; i < nbuf; ++i) {
        crc = bmqcrc::cpu_crc32c(bufs[i], lens[i], crc);
    }
    return crc;
}

uint32_t bmqcrc_combine(uint32_t crcA, uint32_t crcB, uint64_t lenB)
{
    return bmqcrc::cpu_combine(crcA, crcB, lenB);
}

}  // extern "C"
#endif

namespace bmqcrc {

#if defined(BMQCRC_CPU_AB)
// Same-box A/B of the methods at one length (tools/scalar_ab.cpp includes
// this file with BMQCRC_CPU_AB defined; the library never exports these).
uint32_t cpu_crc32c_method(int method, const void* data, uint32_t length, uint32_t crc)
{
    const Tables& T = tables();
    const uint8_t* p = static_cast<const uint8_t*>(data);
    if (length == 0) {
        return crc;
    }
    switch (method) {
#if defined(__x86_64__)
    case 1: return ~raw_serial(p, length, ~crc);
    case 2: return T.clmul ? ~raw_three_way(T, p, length, ~crc) : 0u;
    case 3: return (T.avx512 && length >= 64) ? ~raw_fold(T, p, length, ~crc) : 0u;
#endif
    case 4: return ~raw_soft(T, p, length, ~crc);
    default: return cpu_crc32c(data, length, crc);
    }
}

bool cpu_has(int method)
{
    const Tables& T = tables();
    return method == 0 || method == 4 || (method == 1 && T.sse42) || (method == 2 && T.clmul) ||
           (method == 3 && T.avx512);
}
#endif

}  // namespace bmqcrc
