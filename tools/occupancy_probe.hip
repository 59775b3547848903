// Occupancy probe (diagnostic, not product code): would k_fold's small-message
// regime (groups of 64 two-line segments, a fixed amount of per-group work)
// stream faster with more waves per SIMD?  k_fold is held at two waves per
// SIMD by LDS (two 8 KiB slots per wave) and VGPRs (227).  This probe keeps
// the LDS-DMA access pattern and replaces the fold by `work` dependent VALU
// operations per group in four independent chains, then varies
//   HALF   0: a round is one 128-byte line per lane (8 x 1 KiB instructions,
//             8 lanes per line, 8 KiB slots) -- k_fold's shape;
//          1: a round is half a line per lane (4 x 1 KiB instructions, 4 lanes
//             per half line, 4 KiB slots), so twice the waves fit in LDS;
//          2: k_fold's bytes and slots, but each 1 KiB instruction reads 4
//             consecutive two-line segments (contiguous), i.e. an LDS layout
//             [segment][line] instead of [line][segment];
//   blocks per CU (256-thread blocks = 4 waves), i.e. 2, 3 or 4 waves per SIMD;
//   NT     the non-temporal load policy (k_fold's) or the default one (a half
//          line's other half may then still be in L2).
// Build: hipcc --offload-arch=gfx950 -O3 tools/occupancy_probe.hip -o tools/bin_occupancy_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <bool NT, int N>
__device__ __forceinline__ void issue(uint32_t lds_dst, const uint64_t (&s)[8])
{
    uint32_t keep;
#define OP(CP, K) "global_load_lds_dwordx4 %" #K ", off" CP "\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
    if (N == 8) {
        if (NT) {
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                         OP(" nt", 2) OP(" nt", 3) OP(" nt", 4) OP(" nt", 5) OP(" nt", 6)
                         OP(" nt", 7) OP(" nt", 8) OP(" nt", 9) "s_mov_b32 m0, %0\n\t"
                         : "=&s"(keep) : "s"(lds_dst), "v"(s[0]), "v"(s[1]), "v"(s[2]), "v"(s[3]),
                           "v"(s[4]), "v"(s[5]), "v"(s[6]), "v"(s[7]) : "memory", "scc");
        } else {
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                         OP("", 2) OP("", 3) OP("", 4) OP("", 5) OP("", 6) OP("", 7) OP("", 8)
                         OP("", 9) "s_mov_b32 m0, %0\n\t"
                         : "=&s"(keep) : "s"(lds_dst), "v"(s[0]), "v"(s[1]), "v"(s[2]), "v"(s[3]),
                           "v"(s[4]), "v"(s[5]), "v"(s[6]), "v"(s[7]) : "memory", "scc");
        }
    } else {
        if (NT) {
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                         OP(" nt", 2) OP(" nt", 3) OP(" nt", 4) OP(" nt", 5) "s_mov_b32 m0, %0\n\t"
                         : "=&s"(keep) : "s"(lds_dst), "v"(s[0]), "v"(s[1]), "v"(s[2]), "v"(s[3])
                         : "memory", "scc");
        } else {
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                         OP("", 2) OP("", 3) OP("", 4) OP("", 5) "s_mov_b32 m0, %0\n\t"
                         : "=&s"(keep) : "s"(lds_dst), "v"(s[0]), "v"(s[1]), "v"(s[2]), "v"(s[3])
                         : "memory", "scc");
        }
    }
#undef OP
}

// A Horner-shaped chain of table lookups like k_fold's remainder step:
// 16 steps x 8 lookups of 8-bit indices into eight 1 KiB tables (bank
// conflicts as random bytes give them), or 16 steps x 16 lookups of 4-bit
// indices into sixteen 64-byte tables (conflict-free: 16 entries = 16 banks,
// equal addresses broadcast).  tab: LDS byte address of the tables.
template <int KIND>
__device__ __forceinline__ uint32_t horner_lookups(uint32_t c, uint32_t tab)
{
    typedef __attribute__((address_space(3))) uint32_t lds_u32;
#pragma unroll
    for (int d = 0; d < 16; ++d) {
        const uint32_t v = c ^ (0x9E3779B9u * (uint32_t)(d + 1));
        if (KIND == 1) {
            uint32_t acc = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint32_t b = (k < 4 ? v : (v * 0x85EBCA6Bu)) >> (8 * (k & 3)) & 0xffu;
                acc ^= *(lds_u32*)(uintptr_t)(tab + 1024u * k + 4u * b);
            }
            c = acc;
        } else {
            uint32_t acc = 0;
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const uint32_t b = (k < 8 ? v : (v * 0x85EBCA6Bu)) >> (4 * (k & 7)) & 0xfu;
                acc ^= *(lds_u32*)(uintptr_t)(tab + 64u * k + 4u * b);
            }
            c = acc;
        }
    }
    return c;
}

__device__ __forceinline__ void work4(uint32_t (&v)[4], uint32_t work)
{
    for (uint32_t k = 0; k < work; k += 16) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                v[c] = __builtin_amdgcn_bitop3_b32(v[c], v[(c + 1) & 3], v[c] << 3, 0x96);
            }
        }
    }
}

// HALF: rounds of 64 B per lane; ROUNDS per group = 2 lines * (HALF ? 2 : 1)
template <bool NT, int HALF, int BPC, int KIND = 0>
__global__ __launch_bounds__(256, BPC) void probe(const uint8_t* base, uint64_t ngroups,
                                                   uint32_t work, uint32_t* sink)
{
    // HALF 2: the same 16 KiB per group, each instruction 1 KiB contiguous
    // (4 consecutive two-line segments), i.e. an LDS layout [segment][line]
    constexpr uint32_t kSlot = HALF == 1 ? 4096u : 8192u;
    constexpr int kInstr = HALF == 1 ? 4 : 8;
    constexpr uint32_t kLanesPerPiece = HALF == 1 ? 4u : 8u;  // lanes sharing one 64/128 B unit
    constexpr uint32_t kRounds = HALF == 1 ? 4u : 2u;
    constexpr uint32_t kRoundBytes = HALF == 1 ? 64u : 128u;
    __shared__ __attribute__((aligned(16))) uint8_t lds[4 * 2 * kSlot + 8192];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wl = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)lds +
                        wave * 2u * kSlot;
    const uint64_t stride = (uint64_t)gridDim.x * 4u;
    uint32_t v[4] = {threadIdx.x, lane * 3u, lane ^ 0x55u, 7u};
    auto src = [&](uint64_t g, uint32_t r, uint64_t (&s)[8]) {
        const uint64_t gb = (uint64_t)(uintptr_t)base + g * (64ull * 256u);
#pragma unroll
        for (int i = 0; i < kInstr; ++i) {
            if (HALF == 2) {  // instruction i of "round" r: segments 4(8r+i) .. +3, both lines
                s[i] = gb + (uint64_t)(32u * r + 4u * i) * 256u + 16u * lane;
                continue;
            }
            const uint32_t seg = (uint32_t)i * (64u / kInstr) + lane / kLanesPerPiece;
            s[i] = gb + (uint64_t)seg * 256u + (uint64_t)r * kRoundBytes +
                   16u * (lane % kLanesPerPiece);
        }
    };
    for (uint64_t g = blockIdx.x * 4u + wave; g < ngroups; g += stride) {
        uint64_t s[8];
        src(g, 0, s);
        issue<NT, kInstr>(wl, s);
        src(g, 1, s);
        issue<NT, kInstr>(wl + kSlot, s);
        for (uint32_t r = 0; r < kRounds; ++r) {
            if (r + 1 < kRounds) {
                if (kInstr == 8) {
                    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                } else {
                    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                }
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            const uint32_t slot = wl + (r & 1u) * kSlot;
            v[0] ^= *(__attribute__((address_space(3))) uint32_t*)(uintptr_t)(slot + 4u * lane);
            if (r + 2 < kRounds) {
                src(g, r + 2, s);
                issue<NT, kInstr>(slot, s);
            }
        }
        if (KIND == 0) {
            work4(v, work);
        } else {
            const uint32_t tab = (uint32_t)(uintptr_t)(
                __attribute__((address_space(3))) uint8_t*)lds + 4u * 2u * kSlot;
            for (uint32_t k = 0; k < work; k += 400u) {  // one remainder-step chain per 400
                v[1] = horner_lookups<KIND>(v[1] ^ v[0], tab);
            }
        }
    }
    if ((v[0] ^ v[1] ^ v[2] ^ v[3]) == 0x12345678u) {
        sink[0] = 1;
    }
}

template <bool NT, int HALF, int BPC, int KIND = 0>
void run(const uint8_t* buf, uint64_t bytes, uint32_t work, uint32_t* sink, int cus,
         hipEvent_t a, hipEvent_t b)
{
    const uint64_t ngroups = bytes / (64ull * 256u);
    const int grid = BPC * cus;
    for (int w = 0; w < 3; ++w) {
        hipLaunchKernelGGL((probe<NT, HALF, BPC, KIND>), dim3(grid), dim3(256), 0, 0, buf, ngroups, work,
                           sink);
    }
    const int reps = 20;
    hipEventRecord(a, 0);
    for (int r = 0; r < reps; ++r) {
        hipLaunchKernelGGL((probe<NT, HALF, BPC, KIND>), dim3(grid), dim3(256), 0, 0, buf, ngroups, work,
                           sink);
    }
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double us = 1000.0 * ms / reps;
    printf("{\"mode\": %d, \"waves_per_simd\": %d, \"nt\": %d, \"work\": %u, \"kind\": %d, "
           "\"us\": %.2f, \"TBps\": %.3f}\n",
           HALF, BPC, NT ? 1 : 0, work, KIND, us, bytes / us / 1e6);
    fflush(stdout);
}

int main()
{
    const uint64_t bytes = 256ull << 20;
    uint8_t* buf;
    uint32_t* sink;
    hipMalloc(&buf, bytes);
    hipMalloc(&sink, 64);
    hipMemset(buf, 1, bytes);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    // kind 0: VALU chains; 1: byte-table Horner (128 lookups per 400); 2: nibble tables (256)
    for (uint32_t work : {400u, 800u}) {
        run<false, 0, 2, 0>(buf, bytes, work, sink, cus, a, b);
        run<false, 0, 2, 1>(buf, bytes, work, sink, cus, a, b);
        run<false, 0, 2, 2>(buf, bytes, work, sink, cus, a, b);
    }
    run<false, 0, 2, 0>(buf, bytes, 0, sink, cus, a, b);
    return 0;
}
