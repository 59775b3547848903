// crc32c_cpu.cpp -- host-CPU scalar CRC32C behind the unchanged
// bmqp::Crc32c::calculate(const void*, unsigned, unsigned) signature
// (/root/reference/src/groups/bmq/bmqp/bmqp_crc32c.h:244-246).
//
// The reference answers a single-buffer call synchronously on the calling
// thread (bmqp_crc32c.cpp:41-45 -> BDE, SSE4.2 when available).  A single
// small buffer is latency-bound, so the scalar path stays on the CPU; the GPU
// serves batches (bmqcrc_crc32c_batch).  SSE4.2 crc32q in three interleaved
// lanes, stitched with a GF(2) shift; slicing-by-8 tables without SSE4.2.
#include <stdint.h>
#include <string.h>

#include <mutex>

#if defined(__x86_64__)
#include <cpuid.h>
#include <nmmintrin.h>
#endif

namespace bmqcrc {
namespace {

constexpr uint32_t kPoly = 0x82F63B78u;

uint32_t gf2_mul(uint32_t a, uint32_t b)  // a*b mod P, reflected
{
    uint32_t p = 0;
    for (uint32_t m = 1u << 31; m; m >>= 1) {
        if (a & m) {
            p ^= b;
        }
        b = (b >> 1) ^ (kPoly & (0u - (b & 1u)));
    }
    return p;
}

uint32_t x_pow_8n(uint64_t n)  // x^(8n) mod P, reflected
{
    uint32_t result = 1u << 31, sq = 1u << 30;
    for (uint64_t e = n * 8u; e; e >>= 1) {
        if (e & 1u) {
            result = gf2_mul(result, sq);
        }
        sq = gf2_mul(sq, sq);
    }
    return result;
}

struct Tables {
    uint32_t t8[8][256];
    uint32_t lane_shift[3][2];  // per tier: x^(8*blk), x^(8*2*blk)
    bool sse42;
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
        static const uint32_t blk[3] = {4096u, 512u, 64u};
        for (int t = 0; t < 3; ++t) {
            lane_shift[t][0] = x_pow_8n(blk[t]);
            lane_shift[t][1] = x_pow_8n(2ull * blk[t]);
        }
#if defined(__x86_64__)
        unsigned a, b, c, d;
        sse42 = __get_cpuid(1, &a, &b, &c, &d) && (c & bit_SSE4_2);
#else
        sse42 = false;
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
__attribute__((target("sse4.2"))) uint32_t raw_sse42(const Tables& T, const uint8_t* p, size_t n,
                                                    uint32_t c)
{
    for (; n && (reinterpret_cast<uintptr_t>(p) & 7u); --n) {
        c = _mm_crc32_u8(c, *p++);
    }
    static const uint32_t blk[3] = {4096u, 512u, 64u};
    for (int t = 0; t < 3; ++t) {
        const size_t b = blk[t];
        for (; n >= 3 * b; n -= 3 * b, p += 3 * b) {
            uint64_t a0 = c, a1 = 0, a2 = 0;
            for (size_t i = 0; i < b; i += 8) {
                uint64_t w0, w1, w2;
                memcpy(&w0, p + i, 8);
                memcpy(&w1, p + b + i, 8);
                memcpy(&w2, p + 2 * b + i, 8);
                a0 = _mm_crc32_u64(a0, w0);
                a1 = _mm_crc32_u64(a1, w1);
                a2 = _mm_crc32_u64(a2, w2);
            }
            c = gf2_mul((uint32_t)a0, T.lane_shift[t][1]) ^ gf2_mul((uint32_t)a1, T.lane_shift[t][0]) ^
                (uint32_t)a2;
        }
    }
    uint64_t c64 = c;
    for (; n >= 8; n -= 8, p += 8) {
        uint64_t w;
        memcpy(&w, p, 8);
        c64 = _mm_crc32_u64(c64, w);
    }
    c = (uint32_t)c64;
    for (; n; --n) {
        c = _mm_crc32_u8(c, *p++);
    }
    return c;
}
#endif

}  // namespace

uint32_t cpu_crc32c(const void* data, uint32_t length, uint32_t crc)
{
    if (length == 0) {
        return crc;
    }
    const Tables& T = tables();
    const uint8_t* p = static_cast<const uint8_t*>(data);
#if defined(__x86_64__)
    if (T.sse42) {
        return ~raw_sse42(T, p, length, ~crc);
    }
#endif
    return ~raw_soft(T, p, length, ~crc);
}

uint32_t cpu_combine(uint32_t crcA, uint32_t crcB, uint64_t lenB)
{
    return gf2_mul(crcA, x_pow_8n(lenB)) ^ crcB;
}

}  // namespace bmqcrc
