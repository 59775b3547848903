/*
 * crc32c_oracle.c -- CPU restatement of the reference CRC32C path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the checker for the MI355X HIP
 * path and the CPU baseline timed beside it in bench.py.  It is imported
 * only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg;
 * the shipped library (blazingmq_amd/) never links or calls it.
 *
 * What it restates
 * ----------------
 * bmqp::Crc32c::calculate(const void*, unsigned, unsigned crc)
 *     /root/reference/src/groups/bmq/bmqp/bmqp_crc32c.cpp:41-45 forwards to
 *     bdlde::Crc32c::calculate (BDE tag 4.39.0.0, pinned in
 *     /root/reference/bin/build-ubuntu.sh:71; BDE is NOT vendored in the
 *     reference and is absent from this image).  Semantics pinned by the
 *     reference's own tests (bmqp_crc32c.t.cpp:282-390, 416-434, 598-671):
 *       - CRC-32C (Castagnoli), reflected polynomial 0x82F63B78
 *         (normal 0x1EDC6F41), register initialised to ~crc, result ~register;
 *       - calculate(p, 0, c) == c, calculate(0, 0, c) == c;
 *       - calculate(b, len_b, calculate(a, len_a)) == calculate(a||b).
 * bmqp::Crc32c::calculate(const bdlbb::Blob&, unsigned crc)
 *     bmqp_crc32c.cpp:47-67: chain the above over the blob's data buffers
 *     (full size() for all but the last, lastDataBufferLength() for the
 *     last); an empty blob returns crc.
 *
 * Variants (BASELINE.md section 2 -- BDE's own code cannot be built here, so
 * these are the published algorithms BDE's implementation names follow):
 *   oracle_crc32c_bitwise    bit-at-a-time definition (ground truth)
 *   oracle_crc32c_sw         slicing-by-8 tables  (Crc32c_Impl::calculateSoftware)
 *   oracle_crc32c_hw_serial  SSE4.2 crc32q serial (Crc32c_Impl::calculateHardwareSerial)
 *   oracle_crc32c_hw         SSE4.2 3-way interleaved + table shift-combine
 *                            (bdlde::Crc32c::calculate default)
 * Parity of all variants is pinned by tests/golden/ (the reference's golden
 * vectors) in tests/test_oracle_golden.py.
 */
#define _GNU_SOURCE 1 /* pthread_setaffinity_np: the pinned CPU-baseline pool */
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#include <pthread.h>
#include <sched.h>
#include <time.h>

#if defined(__x86_64__)
#include <cpuid.h>
#include <nmmintrin.h>
#define ORACLE_HAVE_X86 1
#endif

#define POLY 0x82F63B78u

/* ---------------------------------------------------------------- bitwise */
uint32_t oracle_crc32c_bitwise(const void *data, uint32_t len, uint32_t crc)
{
    const uint8_t *p = (const uint8_t *)data;
    uint32_t c = ~crc;
    for (uint32_t i = 0; i < len; ++i) {
        c ^= p[i];
        for (int k = 0; k < 8; ++k) {
            c = (c >> 1) ^ (POLY & (0u - (c & 1u)));
        }
    }
    return ~c;
}

/* ------------------------------------------------------------ slicing-by-8 */
static uint32_t g_tab[8][256];
static pthread_once_t g_tab_once = PTHREAD_ONCE_INIT;

static void init_tables(void)
{
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int k = 0; k < 8; ++k) {
            c = (c >> 1) ^ (POLY & (0u - (c & 1u)));
        }
        g_tab[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i) {
        for (int t = 1; t < 8; ++t) {
            uint32_t prev = g_tab[t - 1][i];
            g_tab[t][i] = (prev >> 8) ^ g_tab[0][prev & 0xFF];
        }
    }
}

static uint32_t sw_raw(const uint8_t *p, size_t len, uint32_t c)
{
    while (len && ((uintptr_t)p & 7)) {
        c = g_tab[0][(c ^ *p++) & 0xFF] ^ (c >> 8);
        --len;
    }
    while (len >= 8) {
        uint64_t w;
        memcpy(&w, p, 8);
        w ^= c;
        c = g_tab[7][w & 0xFF] ^ g_tab[6][(w >> 8) & 0xFF] ^
            g_tab[5][(w >> 16) & 0xFF] ^ g_tab[4][(w >> 24) & 0xFF] ^
            g_tab[3][(w >> 32) & 0xFF] ^ g_tab[2][(w >> 40) & 0xFF] ^
            g_tab[1][(w >> 48) & 0xFF] ^ g_tab[0][w >> 56];
        p += 8;
        len -= 8;
    }
    while (len--) {
        c = g_tab[0][(c ^ *p++) & 0xFF] ^ (c >> 8);
    }
    return c;
}

uint32_t oracle_crc32c_sw(const void *data, uint32_t len, uint32_t crc)
{
    pthread_once(&g_tab_once, init_tables);
    if (len == 0) {
        return crc;
    }
    return ~sw_raw((const uint8_t *)data, len, ~crc);
}

/* ------------------------------------------------- GF(2) helpers (combine) */
/* a * b mod P, reflected convention (bit 31 <-> x^0). */
static uint32_t multmodp(uint32_t a, uint32_t b)
{
    uint32_t m = 1u << 31, p = 0;
    for (;;) {
        if (a & m) {
            p ^= b;
            if ((a & (m - 1)) == 0) {
                break;
            }
        }
        m >>= 1;
        b = (b & 1) ? (b >> 1) ^ POLY : b >> 1;
    }
    return p;
}

/* x^(8*n) mod P by square-and-multiply. */
static uint32_t x8nmodp(uint64_t n)
{
    uint32_t xp = 1u << 30; /* x^1 */
    uint32_t p = 1u << 31;  /* x^0 */
    uint64_t e = n * 8u;
    while (e) {
        if (e & 1) {
            p = multmodp(xp, p);
        }
        xp = multmodp(xp, xp);
        e >>= 1;
    }
    return p;
}

/* crc(A||B) from crc(A), crc(B), |B| (finalised CRCs, zlib-style). */
uint32_t oracle_crc32c_combine(uint32_t crcA, uint32_t crcB, uint64_t lenB)
{
    return multmodp(x8nmodp(lenB), crcA) ^ crcB;
}

/* ---------------------------------------------------------------- SSE4.2 */
static int g_have_sse42 = -1;

int oracle_have_sse42(void)
{
#ifdef ORACLE_HAVE_X86
    if (g_have_sse42 < 0) {
        unsigned a, b, c, d;
        g_have_sse42 = (__get_cpuid(1, &a, &b, &c, &d) && (c & bit_SSE4_2)) ? 1 : 0;
    }
    return g_have_sse42;
#else
    return 0;
#endif
}

#ifdef ORACLE_HAVE_X86
__attribute__((target("sse4.2"))) static uint32_t hw_raw(const uint8_t *p, size_t len, uint32_t c)
{
    uint64_t c64 = c;
    while (len && ((uintptr_t)p & 7)) {
        c64 = _mm_crc32_u8((uint32_t)c64, *p++);
        --len;
    }
    while (len >= 8) {
        uint64_t w;
        memcpy(&w, p, 8);
        c64 = _mm_crc32_u64(c64, w);
        p += 8;
        len -= 8;
    }
    while (len--) {
        c64 = _mm_crc32_u8((uint32_t)c64, *p++);
    }
    return (uint32_t)c64;
}

/* Three independent crc32q chains over consecutive thirds of a block, then a
 * GF(2) shift-combine: the standard way to fill the 3-cycle-latency /
 * 1-per-cycle-throughput crc32 pipeline.  Two block tiers (8 KiB, 256 B) so
 * mid-size buffers also run interleaved.  The combine shifts a register over
 * a lane of zero bytes with four 256-entry tables per tier (one lookup per
 * register byte), as in the published SSE4.2 CRC-32C code this family of
 * implementations follows (Mark Adler's crc32c.c: LONG = 8192, SHORT = 256,
 * crc32c_zeros / crc32c_shift); BDE's own source is absent (header comment). */
static uint32_t g_zeros[2][4][256]; /* [tier][register byte][value]: shift over one lane */
static const uint32_t g_blk[2] = {8192u, 256u};
static pthread_once_t g_shift_once = PTHREAD_ONCE_INIT;
static void init_shift(void)
{
    for (int t = 0; t < 2; ++t) {
        const uint32_t op = x8nmodp(g_blk[t]);
        for (int k = 0; k < 4; ++k) {
            for (uint32_t n = 0; n < 256; ++n) {
                g_zeros[t][k][n] = multmodp(op, n << (8 * k));
            }
        }
    }
}

static inline uint32_t zeros_shift(const uint32_t (*z)[256], uint32_t c)
{
    return z[0][c & 0xff] ^ z[1][(c >> 8) & 0xff] ^ z[2][(c >> 16) & 0xff] ^ z[3][c >> 24];
}

__attribute__((target("sse4.2"))) static uint32_t hw3_raw(const uint8_t *p, size_t len, uint32_t c)
{
    while (len && ((uintptr_t)p & 7)) {
        c = _mm_crc32_u8(c, *p++);
        --len;
    }
    for (int t = 0; t < 2; ++t) {
        const uint32_t blk = g_blk[t];
        while (len >= 3 * (size_t)blk) {
            uint64_t c0 = c, c1 = 0, c2 = 0;
            const uint8_t *p1 = p + blk, *p2 = p + 2 * blk;
            for (uint32_t i = 0; i < blk; i += 8) {
                uint64_t w0, w1, w2;
                memcpy(&w0, p + i, 8);
                memcpy(&w1, p1 + i, 8);
                memcpy(&w2, p2 + i, 8);
                c0 = _mm_crc32_u64(c0, w0);
                c1 = _mm_crc32_u64(c1, w1);
                c2 = _mm_crc32_u64(c2, w2);
            }
            c = zeros_shift(g_zeros[t], (uint32_t)c0) ^ (uint32_t)c1;
            c = zeros_shift(g_zeros[t], c) ^ (uint32_t)c2;
            p += 3 * (size_t)blk;
            len -= 3 * (size_t)blk;
        }
    }
    return hw_raw(p, len, c);
}
#endif

uint32_t oracle_crc32c_hw_serial(const void *data, uint32_t len, uint32_t crc)
{
    if (len == 0) {
        return crc;
    }
#ifdef ORACLE_HAVE_X86
    if (oracle_have_sse42()) {
        return ~hw_raw((const uint8_t *)data, len, ~crc);
    }
#endif
    return oracle_crc32c_sw(data, len, crc);
}

uint32_t oracle_crc32c_hw(const void *data, uint32_t len, uint32_t crc)
{
    if (len == 0) {
        return crc;
    }
#ifdef ORACLE_HAVE_X86
    if (oracle_have_sse42()) {
        pthread_once(&g_shift_once, init_shift);
        return ~hw3_raw((const uint8_t *)data, len, ~crc);
    }
#endif
    return oracle_crc32c_sw(data, len, crc);
}

/* ------------------------------------------------------------ Blob chain */
/* bmqp_crc32c.cpp:47-67: empty blob -> crc; otherwise chain per buffer. */
uint32_t oracle_crc32c_blob(const void *const *bufs, const uint32_t *lens, uint32_t nbuf,
                            uint32_t crc)
{
    for (uint32_t i = 0; i < nbuf; ++i) {
        crc = oracle_crc32c_bitwise(bufs[i], lens[i], crc);
    }
    return crc;
}

/* ------------------------------------------------------------ batch (CPU) */
typedef uint32_t (*crc_fn)(const void *, uint32_t, uint32_t);

static crc_fn pick(int variant)
{
    switch (variant) {
    case 0: return oracle_crc32c_hw;
    case 1: return oracle_crc32c_hw_serial;
    case 2: return oracle_crc32c_sw;
    default: return oracle_crc32c_bitwise;
    }
}

struct batch_job {
    const uint8_t *arena;
    const uint64_t *off;
    const uint32_t *len;
    const uint32_t *seed;
    uint32_t *out;
    size_t lo, hi;
    crc_fn fn;
};

static void *batch_worker(void *arg)
{
    struct batch_job *j = (struct batch_job *)arg;
    for (size_t i = j->lo; i < j->hi; ++i) {
        j->out[i] = j->fn(j->arena + j->off[i], j->len[i], j->seed ? j->seed[i] : 0u);
    }
    return NULL;
}

/* Contiguous byte-balanced slices of a batch, one per thread (the
 * reference's test5 pattern, bmqp_crc32c.t.cpp:705-760). */
static void split_jobs(struct batch_job *jobs, int nthreads, const uint8_t *arena,
                       const uint64_t *off, const uint32_t *len, const uint32_t *seed,
                       uint32_t *out, size_t n, int variant)
{
    uint64_t total = 0;
    for (size_t i = 0; i < n; ++i) {
        total += len[i];
    }
    size_t i = 0;
    uint64_t acc = 0;
    for (int t = 0; t < nthreads; ++t) {
        jobs[t].arena = arena;
        jobs[t].off = off;
        jobs[t].len = len;
        jobs[t].seed = seed;
        jobs[t].out = out;
        jobs[t].fn = pick(variant);
        jobs[t].lo = i;
        uint64_t target = total * (uint64_t)(t + 1) / (uint64_t)nthreads;
        while (i < n && (acc < target || t == nthreads - 1)) {
            acc += len[i];
            ++i;
        }
        jobs[t].hi = i;
    }
}

enum { MAXT = 256 };

static int clamp_threads(int nthreads)
{
    return nthreads < 1 ? 1 : nthreads > MAXT ? MAXT : nthreads;
}

/* CRC every message of a batch on `nthreads` host threads, messages split
 * into contiguous byte-balanced slices.  variant: 0 hw 3-way, 1 hw serial,
 * 2 slicing-by-8, 3 bitwise.  Returns 0. */
int oracle_crc32c_batch(const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                        const uint32_t *seed, uint32_t *out, size_t n, int nthreads, int variant)
{
    nthreads = clamp_threads(nthreads);
    pthread_once(&g_tab_once, init_tables);
    struct batch_job jobs[MAXT];
    pthread_t th[MAXT];
    split_jobs(jobs, nthreads, arena, off, len, seed, out, n, variant);
    for (int t = 1; t < nthreads; ++t) {
        pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
    }
    batch_worker(&jobs[0]);
    for (int t = 1; t < nthreads; ++t) {
        pthread_join(th[t], NULL);
    }
    return 0;
}

/* Timing pool: the worker threads are created once, before the clock
 * starts, and every pass is bracketed by two barrier waits, so a pass times
 * the CRCs (and one barrier), not thread start-up. */
struct pool_arg {
    struct batch_job *job;
    pthread_barrier_t *bar;
    int passes;
    int cpu; /* < 0: not pinned */
};

static void pin_self(int cpu)
{
    if (cpu >= 0 && cpu < CPU_SETSIZE) {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(cpu, &set);
        pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
    }
}

static void *pool_worker(void *arg)
{
    struct pool_arg *p = (struct pool_arg *)arg;
    pin_self(p->cpu);
    for (int r = 0; r < p->passes; ++r) {
        pthread_barrier_wait(p->bar);
        batch_worker(p->job);
        pthread_barrier_wait(p->bar);
    }
    return NULL;
}

static double now_s(void)
{
    struct timespec a;
    clock_gettime(CLOCK_MONOTONIC, &a);
    return (double)a.tv_sec + 1e-9 * (double)a.tv_nsec;
}

/* Wall-clock seconds for `reps` passes over the batch on `nthreads` threads
 * (bench helper): threads created before the clock starts and one untimed
 * warm-up pass first.  cpus (may be NULL): thread t runs pinned to cpus[t]
 * (thread 0 is the caller, whose affinity is restored afterwards). */
double oracle_time_batch_pinned(const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                                const uint32_t *seed, uint32_t *out, size_t n, int nthreads,
                                int variant, int reps, const int *cpus)
{
    nthreads = clamp_threads(nthreads);
    pthread_once(&g_tab_once, init_tables);
    struct batch_job jobs[MAXT];
    pthread_t th[MAXT];
    struct pool_arg args[MAXT];
    pthread_barrier_t bar;
    split_jobs(jobs, nthreads, arena, off, len, seed, out, n, variant);
    pthread_barrier_init(&bar, NULL, (unsigned)nthreads);
    const int passes = reps + 1;
    for (int t = 1; t < nthreads; ++t) {
        args[t].job = &jobs[t];
        args[t].bar = &bar;
        args[t].passes = passes;
        args[t].cpu = cpus ? cpus[t] : -1;
        pthread_create(&th[t], NULL, pool_worker, &args[t]);
    }
    cpu_set_t saved;
    const int restore = cpus && pthread_getaffinity_np(pthread_self(), sizeof(saved), &saved) == 0;
    if (cpus) {
        pin_self(cpus[0]);
    }
    double t0 = 0;
    for (int r = 0; r < passes; ++r) {
        if (r == 1) {
            t0 = now_s();  /* after the warm-up pass */
        }
        pthread_barrier_wait(&bar);
        batch_worker(&jobs[0]);
        pthread_barrier_wait(&bar);
    }
    const double dt = now_s() - t0;
    for (int t = 1; t < nthreads; ++t) {
        pthread_join(th[t], NULL);
    }
    pthread_barrier_destroy(&bar);
    if (restore) {
        pthread_setaffinity_np(pthread_self(), sizeof(saved), &saved);
    }
    return dt;
}

double oracle_time_batch(const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                         const uint32_t *seed, uint32_t *out, size_t n, int nthreads,
                         int variant, int reps)
{
    return oracle_time_batch_pinned(arena, off, len, seed, out, n, nthreads, variant, reps, NULL);
}

/* The reference's own benchmark loop (bmqp_crc32c.t.cpp:1116-1120): one
 * buffer CRC'd `iters` times on the calling thread after one untimed call.
 * Returns wall-clock seconds; *crc_out = the last CRC (keeps the loop live). */
double oracle_time_repeat(const uint8_t *buf, uint32_t length, int iters, int variant,
                          uint32_t *crc_out)
{
    pthread_once(&g_tab_once, init_tables);
    crc_fn fn = pick(variant);
    uint32_t c = fn(buf, length, 0u);
    const double t0 = now_s();
    for (int l = 0; l < iters; ++l) {
        c ^= fn(buf, length, 0u);
    }
    const double dt = now_s() - t0;
    *crc_out = c;
    return dt;
}

/* Deterministic synthetic payload bytes shared with the device generator:
 * byte i of the stream seeded by `seed` is the low byte of
 * splitmix64(seed * 0x9E3779B97F4A7C15 + (i / 8)) >> (8 * (i % 8)). */
static uint64_t splitmix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

void oracle_fill_payload(uint8_t *dst, uint64_t begin, uint64_t nbytes, uint64_t seed)
{
    for (uint64_t i = 0; i < nbytes; ++i) {
        uint64_t g = begin + i;
        uint64_t w = splitmix64(seed * 0x9E3779B97F4A7C15ull + (g >> 3));
        dst[i] = (uint8_t)(w >> (8 * (g & 7)));
    }
}
