// LDS-DMA access-pattern probe (diagnostic, not product code): how fast can
// k_fold's data movement go for groups of 64 short segments, with and without
// keeping the DMA stream running across group boundaries?
//
// A wave owns groups of 64 consecutive segments of `seglines` 128-byte lines
// (k_fold's layout: per round 8 x global_load_lds_dwordx4, instruction i
// carries one full line of segments 8i..8i+7, two LDS slots).
//   mode 0  group-synchronous: the last round of a group waits vmcnt(0), then
//           a synthetic "remainder step" of `work` VALU ops, then the next
//           group starts (k_fold today).
//   mode 1  continuous: rounds run across group boundaries with two always in
//           flight; the synthetic work of a group runs while the next group's
//           first rounds load.
// Build: hipcc --offload-arch=gfx950 -O3 tools/dma_pattern_probe.hip -o /tmp/dma_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

constexpr int kSlotBytes = 8192;

__device__ __forceinline__ void dma_round(uint32_t lds_dst, const uint64_t (&s)[8])
{
    uint32_t keep;
    asm volatile(
        "s_waitcnt lgkmcnt(0)\n\t"
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %1\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %2, off nt\n\t"
        "s_add_u32 m0, m0, 0x400\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %3, off nt\n\t"
        "s_add_u32 m0, m0, 0x400\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %4, off nt\n\t"
        "s_add_u32 m0, m0, 0x400\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %5, off nt\n\t"
        "s_add_u32 m0, m0, 0x400\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %6, off nt\n\t"
        "s_add_u32 m0, m0, 0x400\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %7, off nt\n\t"
        "s_add_u32 m0, m0, 0x400\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %8, off nt\n\t"
        "s_add_u32 m0, m0, 0x400\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %9, off nt\n\t"
        "s_mov_b32 m0, %0\n\t"
        : "=&s"(keep)
        : "s"(lds_dst), "v"(s[0]), "v"(s[1]), "v"(s[2]), "v"(s[3]), "v"(s[4]), "v"(s[5]),
          "v"(s[6]), "v"(s[7])
        : "memory", "scc");
}

__device__ __forceinline__ void round_src(uint64_t gbase, uint32_t seglines, uint32_t r,
                                          uint64_t (&s)[8])
{
    const uint32_t lane = __lane_id();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t seg = 8u * i + (lane >> 3);
        s[i] = gbase + (uint64_t)seg * seglines * 128u + (uint64_t)r * 128u + 16u * (lane & 7u);
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

__global__ __launch_bounds__(256, 2) void probe(const uint8_t* base, uint64_t ngroups,
                                                 uint32_t seglines, uint32_t mode, uint32_t work,
                                                 uint32_t* sink)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[4 * 2 * kSlotBytes + 8192];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t wl = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)lds +
                        wave * 2 * kSlotBytes;
    const uint32_t stride = gridDim.x * 4;
    const uint64_t gbytes = 64ull * seglines * 128u;
    uint32_t acc = threadIdx.x;
    uint64_t s[8];
    if (mode == 0) {
        for (uint64_t g = blockIdx.x * 4 + wave; g < ngroups; g += stride) {
            const uint64_t gb = (uint64_t)(uintptr_t)base + g * gbytes;
            round_src(gb, seglines, 0, s);
            dma_round(wl, s);
            if (seglines > 1) {
                round_src(gb, seglines, 1, s);
                dma_round(wl + kSlotBytes, s);
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
                    round_src(gb, seglines, r + 2, s);
                    dma_round(slot, s);
                }
            }
            acc = fake_work(acc, work);
        }
    } else {
        // continuous round stream over this wave's groups
        const uint64_t g0 = blockIdx.x * 4 + wave;
        const uint64_t my = g0 < ngroups ? (ngroups - g0 + stride - 1) / stride : 0;
        const uint64_t total = my * seglines;
        auto src_of = [&](uint64_t t) {
            const uint64_t gi = seglines == 1 ? t : t / seglines;
            const uint32_t r = (uint32_t)(t - gi * seglines);
            round_src((uint64_t)(uintptr_t)base + (g0 + gi * stride) * gbytes, seglines, r, s);
        };
        if (total > 0) {
            src_of(0);
            dma_round(wl, s);
        }
        if (total > 1) {
            src_of(1);
            dma_round(wl + kSlotBytes, s);
        }
        for (uint64_t t = 0; t < total; ++t) {
            if (t + 1 < total) {
                asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            const uint32_t slot = wl + (uint32_t)(t & 1u) * kSlotBytes;
            acc ^= *(__attribute__((address_space(3))) uint32_t*)(uintptr_t)(slot + 4u * __lane_id());
            if (t + 2 < total) {
                src_of(t + 2);
                dma_round(slot, s);
            }
            if (seglines == 1 || (t + 1) % seglines == 0) {
                acc = fake_work(acc, work);
            }
        }
    }
    if (acc == 0x12345678u) {
        sink[0] = acc;
    }
}

int main(int argc, char** argv)
{
    const uint64_t bytes = 256ull << 20;
    uint8_t* buf;
    uint32_t* sink;
    hipMalloc(&buf, bytes);
    hipMalloc(&sink, 64);
    hipMemset(buf, 1, bytes);
    int dev = 0, cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const uint32_t seglines_list[] = {1, 2, 4, 16};
    const uint32_t work_list[] = {0, 200, 400, 800};
    for (uint32_t sl : seglines_list) {
        for (uint32_t work : work_list) {
            for (uint32_t mode = 0; mode < 2; ++mode) {
                const uint64_t ngroups = bytes / (64ull * sl * 128u);
                const int grid = 2 * cus;
                for (int w = 0; w < 3; ++w) {
                    hipLaunchKernelGGL(probe, dim3(grid), dim3(256), 0, 0, buf, ngroups, sl, mode,
                                       work, sink);
                }
                const int reps = 20;
                hipEventRecord(a, 0);
                for (int r = 0; r < reps; ++r) {
                    hipLaunchKernelGGL(probe, dim3(grid), dim3(256), 0, 0, buf, ngroups, sl, mode,
                                       work, sink);
                }
                hipEventRecord(b, 0);
                hipEventSynchronize(b);
                float ms = 0;
                hipEventElapsedTime(&ms, a, b);
                const double us = 1000.0 * ms / reps;
                printf("{\"seglines\": %u, \"work\": %u, \"mode\": %u, \"us\": %.2f, \"TBps\": %.3f}\n",
                       sl, work, mode, us, bytes / us / 1e6);
                fflush(stdout);
            }
        }
    }
    return 0;
}
