// LDS-DMA access-pattern probe on HBM-resident data (diagnostic, not product
// code).  round 2's tools/dma_pattern_probe.hip read one 256 MiB buffer over
// and over, which the 256 MiB Infinity Cache holds; this one cycles four 1 GiB
// regions, so every launch streams from HBM.
//
// A wave owns groups of 64 two-line (256-byte) segments, contiguous in
// memory like 1M x 256 B, with k_fold's two 8 KiB LDS slots:
//   layout 0  k_fold's: round r carries line r of every segment; instruction
//             i covers segments 8i..8i+7 (8 lines 256 bytes apart)
//   layout 1  segment-major: instruction i of round r covers segments
//             32r + 4i .. 32r + 4i + 3, both lines (1 KiB contiguous)
// then `work` dependent VALU ops per group (a stand-in for fold + remainder).
// Build: hipcc --offload-arch=gfx950 -O3 tools/dma_hbm_probe.hip -o /tmp/dma_hbm_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kSlotBytes = 8192;

__device__ __forceinline__ void dma_round(uint32_t lds_dst, const uint64_t (&s)[8])
{
    uint32_t keep;
    asm volatile(
        "s_waitcnt lgkmcnt(0)\n\t"
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %1\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %2, off\n\t"
        "s_add_u32 m0, m0, 0x400\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %3, off\n\t"
        "s_add_u32 m0, m0, 0x400\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %4, off\n\t"
        "s_add_u32 m0, m0, 0x400\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %5, off\n\t"
        "s_add_u32 m0, m0, 0x400\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %6, off\n\t"
        "s_add_u32 m0, m0, 0x400\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %7, off\n\t"
        "s_add_u32 m0, m0, 0x400\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %8, off\n\t"
        "s_add_u32 m0, m0, 0x400\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %9, off\n\t"
        "s_mov_b32 m0, %0\n\t"
        : "=&s"(keep)
        : "s"(lds_dst), "v"(s[0]), "v"(s[1]), "v"(s[2]), "v"(s[3]), "v"(s[4]), "v"(s[5]),
          "v"(s[6]), "v"(s[7])
        : "memory", "scc");
}

__device__ __forceinline__ void round_src(uint64_t gbase, uint32_t layout, uint32_t r,
                                          uint64_t (&s)[8])
{
    const uint32_t lane = __lane_id();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        if (layout == 0) {
            const uint32_t seg = 8u * i + (lane >> 3);
            s[i] = gbase + (uint64_t)seg * 256u + (uint64_t)r * 128u + 16u * (lane & 7u);
        } else {
            s[i] = gbase + (uint64_t)(r * 8u + i) * 1024u + 16u * lane;
        }
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
                                                 uint32_t layout, uint32_t work, uint32_t* sink)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[8 * 2 * kSlotBytes];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t wl = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)lds +
                        wave * 2 * kSlotBytes;
    const uint32_t stride = gridDim.x * 8;
    uint32_t acc = threadIdx.x;
    uint64_t s[8];
    for (uint64_t g = blockIdx.x * 8 + wave; g < ngroups; g += stride) {
        const uint64_t gb = (uint64_t)(uintptr_t)base + g * 16384u;
        round_src(gb, layout, 0, s);
        dma_round(wl, s);
        round_src(gb, layout, 1, s);
        dma_round(wl + kSlotBytes, s);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        acc ^= *(__attribute__((address_space(3))) uint32_t*)(uintptr_t)(wl + 4u * __lane_id());
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        acc ^= *(__attribute__((address_space(3))) uint32_t*)(uintptr_t)(wl + kSlotBytes +
                                                                        4u * __lane_id());
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
    const uint64_t ngroups = region / 16384u;
    for (uint32_t work : {0u, 400u, 800u}) {
        for (uint32_t layout = 0; layout < 2; ++layout) {
            for (int w = 0; w < nreg; ++w) {
                hipLaunchKernelGGL(probe, dim3(cus), dim3(512), 0, 0, buf + w * region, ngroups,
                                   layout, work, sink);
            }
            const int reps = 20;
            hipEventRecord(a, 0);
            for (int r = 0; r < reps; ++r) {
                hipLaunchKernelGGL(probe, dim3(cus), dim3(512), 0, 0, buf + (r % nreg) * region,
                                   ngroups, layout, work, sink);
            }
            hipEventRecord(b, 0);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            const double us = 1000.0 * ms / reps;
            printf("{\"layout\": %u, \"work\": %u, \"us_per_GiB\": %.2f, \"TBps\": %.3f}\n", layout,
                   work, us, region / us / 1e6);
            fflush(stdout);
        }
    }
    return 0;
}
