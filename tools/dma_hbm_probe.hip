// LDS-DMA access-pattern probe on HBM-resident data (diagnostic, not product
// code).  round 2's tools/dma_pattern_probe.hip read one 256 MiB buffer over
// and over, which the 256 MiB Infinity Cache holds; this one cycles four 1 GiB
// regions, so every launch streams from HBM.
//
// A wave owns groups of 64 segments with k_fold's two 8 KiB LDS slots (round
// r carries line r of every segment; instruction i covers segments 8i..8i+7),
// then `work` dependent VALU ops per group (a stand-in for fold + remainder).
// Shapes: contiguous 256-byte and 128-byte segments (1M x 256 B, 128-byte
// messages) and 2 KiB of segments 64 KiB apart (the headline's shape); 8 or 4
// waves per CU; default or non-temporal loads.  A first run (round 5) found
// k_fold's piece order and a segment-major order (1 KiB contiguous per
// instruction) equal: 6.05 / 6.04 TB/s with no work.
// Build: hipcc --offload-arch=gfx950 -O3 tools/dma_hbm_probe.hip -o /tmp/dma_hbm_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kSlotBytes = 8192;

#define PROBE_DMA(CP)                                                                         \
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

__device__ __forceinline__ void dma_round(uint32_t lds_dst, const uint64_t (&s)[8], bool nt)
{
    uint32_t keep;
    if (nt) {
        asm volatile(PROBE_DMA(" nt")
                     : "=&s"(keep)
                     : "s"(lds_dst), "v"(s[0]), "v"(s[1]), "v"(s[2]), "v"(s[3]), "v"(s[4]),
                       "v"(s[5]), "v"(s[6]), "v"(s[7])
                     : "memory", "scc");
        return;
    }
    asm volatile(PROBE_DMA("")
                 : "=&s"(keep)
                 : "s"(lds_dst), "v"(s[0]), "v"(s[1]), "v"(s[2]), "v"(s[3]), "v"(s[4]), "v"(s[5]),
                   "v"(s[6]), "v"(s[7])
                 : "memory", "scc");
}

// segment s of a group at gbase + s * sstride (sstride = 128 * seglines:
// contiguous, like 1M x 256 B; or 64 KiB: one message per lane, like the
// headline's segments); round r reads line r of every segment
__device__ __forceinline__ void round_src(uint64_t gbase, uint64_t sstride, uint32_t r,
                                          uint64_t (&s)[8])
{
    const uint32_t lane = __lane_id();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t seg = 8u * i + (lane >> 3);
        s[i] = gbase + (uint64_t)seg * sstride + (uint64_t)r * 128u + 16u * (lane & 7u);
    }
}

__device__ __forceinline__ uint32_t fake_work(uint32_t v, uint32_t work)
{
    for (uint32_t k = 0; k < work; k += 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            v = __builtin_amdgcn_bitop3_b32(v, v >> 1, v << 3, 0x96);
        }
    }
    return v;
}

__global__ __launch_bounds__(512, 1) void probe(const uint8_t* base, uint64_t ngroups,
                                                 uint32_t seglines, uint64_t sstride,
                                                 uint64_t gstride, uint32_t nt, uint32_t work,
                                                 uint32_t* sink)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[8 * 2 * kSlotBytes];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t wpb = blockDim.x / 64;
    const uint32_t wl = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)lds +
                        wave * 2 * kSlotBytes;
    const uint32_t stride = gridDim.x * wpb;
    uint32_t acc = threadIdx.x;
    uint64_t s[8];
    for (uint64_t g = blockIdx.x * wpb + wave; g < ngroups; g += stride) {
        // group g: 64 segments from gbase (contiguous groups for contiguous
        // segments; for 64 KiB-spaced segments the groups interleave)
        const uint64_t gb = (uint64_t)(uintptr_t)base + (g / 32u) * gstride + (g % 32u) * 128u * seglines;
        const uint64_t gbc = sstride == 128u * seglines ? (uint64_t)(uintptr_t)base + g * 64u * sstride : gb;
        round_src(gbc, sstride, 0, s);
        dma_round(wl, s, nt);
        if (seglines > 1) {
            round_src(gbc, sstride, 1, s);
            dma_round(wl + kSlotBytes, s, nt);
        }
        for (uint32_t r = 0; r < seglines; ++r) {
            if (r + 1 < seglines) {
                asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            const uint32_t slot = wl + (r & 1u) * kSlotBytes;
            acc ^= *(__attribute__((address_space(3))) uint32_t*)(uintptr_t)(slot + 4u * __lane_id());
            if (r + 2 < seglines) {
                round_src(gbc, sstride, r + 2, s);
                dma_round(slot, s, nt);
            }
        }
        acc = fake_work(acc, work);
    }
    if (acc == 0x12345678u) {
        sink[0] = acc;
    }
}

int main()
{
    const uint64_t region = 1ull << 30;
    const int nreg = 4;
    uint8_t* buf;
    uint32_t* sink;
    if (hipMalloc(&buf, region * nreg) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    hipMemset(buf, 1, region * nreg);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    struct Shape {
        uint32_t seglines;
        uint64_t sstride;
        const char* name;
    };
    // 2-line contiguous segments (1M x 256 B), 1-line (128 B), and 16-line
    // segments 64 KiB apart (the headline's access shape, one message per lane)
    const Shape shapes[] = {{2, 256, "256B_contig"}, {1, 128, "128B_contig"}, {16, 65536, "2KiB_of_64KiB"}};
    for (const Shape& sh : shapes) {
        const uint64_t gbytes = 64ull * 128u * sh.seglines;
        const uint64_t ngroups = region / gbytes;
        // 64 KiB-spaced: 32 groups share a 64-segment x 64 KiB window (4 MiB)
        const uint64_t gstride = 64ull * sh.sstride;
        for (uint32_t wpb : {8u, 4u}) {
            for (uint32_t nt = 0; nt < 2; ++nt) {
                for (uint32_t work : {0u, 400u}) {
                    auto launch = [&](int r) {
                        hipLaunchKernelGGL(probe, dim3(cus), dim3(64 * wpb), 0, 0,
                                           buf + (r % nreg) * region, ngroups, sh.seglines,
                                           sh.sstride, gstride, nt, work, sink);
                    };
                    for (int w = 0; w < nreg; ++w) {
                        launch(w);
                    }
                    const int reps = 20;
                    hipEventRecord(a, 0);
                    for (int r = 0; r < reps; ++r) {
                        launch(r);
                    }
                    hipEventRecord(b, 0);
                    hipEventSynchronize(b);
                    float ms = 0;
                    hipEventElapsedTime(&ms, a, b);
                    const double us = 1000.0 * ms / reps;
                    printf("{\"shape\": \"%s\", \"waves_per_cu\": %u, \"nt\": %u, \"work\": %u, "
                           "\"us_per_GiB\": %.2f, \"TBps\": %.3f}\n",
                           sh.name, wpb, nt, work, us, region / us / 1e6);
                    fflush(stdout);
                }
            }
        }
    }
    return 0;
}
