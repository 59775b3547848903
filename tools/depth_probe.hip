// Pipeline-depth probe for one-line groups on HBM-resident data (diagnostic,
// not product code).  k_fold folds a group of 64 one-line segments (messages
// of at most 128 bytes, right-aligned in a 128-byte stream) with ONE round of
// LDS-DMA in flight per wave: the next group's round is issued after this
// group's line is read, and its remainder step runs under that load.  Groups
// of two or more lines keep both 8 KiB slots in flight.  This probe measures
// what a second one-line group in flight (the slot the previous group used)
// is worth, with `work` dependent VALU ops per group standing in for the
// remainder step, and what loading only the pieces a 64-byte message
// occupies is worth (the other half of each line read from a zero line, as
// k_fold does, or not loaded at all: lanes masked off in the DMA).
//   depth 1: k_fold's schedule (wait, read, issue the next group, work)
//   depth 2: two groups in flight (wait for the older, read, issue the group
//            after the next into the freed slot, work)
//   depth 3: two ADJACENT groups issued together and waited for together
//            (twice the contiguous bytes per wave request; the work doubled)
//   depth 4: the same with the two groups half the batch apart
// Shapes: 128-byte messages (every piece from HBM) and 64-byte messages
// (pieces 0-3 from a zero line, or masked off).  Four 1 GiB regions are
// cycled so that every launch reads HBM, not the Infinity Cache.
// Build: hipcc --offload-arch=gfx950 -O3 tools/depth_probe.hip -o tools/bin/depth_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kSlotBytes = 8192;

__device__ __attribute__((aligned(128))) uint8_t g_zero[128];

#define DEPTH_DMA(CP)                                                                         \
    "s_waitcnt lgkmcnt(0)\n\t"                                                              \
    "s_mov_b32 %0, m0\n\t"                                                                  \
    "s_mov_b32 m0, %2\n\t"                                                                  \
    "s_mov_b64 %1, exec\n\t"                                                                \
    "s_mov_b64 exec, %3\n\t"                                                                \
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
    "s_add_u32 m0, m0, 0x400\n\t"                                                           \
    "s_nop 0\n\t"                                                                           \
    "global_load_lds_dwordx4 %10, off" CP "\n\t"                                            \
    "s_add_u32 m0, m0, 0x400\n\t"                                                           \
    "s_nop 0\n\t"                                                                           \
    "global_load_lds_dwordx4 %11, off" CP "\n\t"                                            \
    "s_mov_b64 exec, %1\n\t"                                                                \
    "s_mov_b32 m0, %0\n\t"

// one round: instruction i carries segment 8i + lane/8, piece lane%8; exec
// selects the lanes that load (all, or only the pieces a 64-byte message uses)
__device__ __forceinline__ void dma_round(uint32_t lds_dst, const uint64_t (&s)[8],
                                          uint64_t exec_mask)
{
    uint32_t keep;
    uint64_t save;
    asm volatile(DEPTH_DMA(" nt")
                 : "=&s"(keep), "=&s"(save)
                 : "s"(lds_dst), "s"(exec_mask), "v"(s[0]), "v"(s[1]), "v"(s[2]), "v"(s[3]),
                   "v"(s[4]), "v"(s[5]), "v"(s[6]), "v"(s[7])
                 : "memory", "scc");
}

// msg_bytes 128: the line is the message; 64: pieces 4-7 are the message,
// pieces 0-3 the zero line (mode 0) or not loaded (mode 1)
__device__ __forceinline__ void round_src(uint64_t gbase, uint32_t msg_bytes, uint64_t (&s)[8])
{
    const uint32_t lane = __lane_id();
    const uint32_t pp = lane & 7u;
    const uint64_t zero = (uint64_t)(uintptr_t)g_zero + 16u * pp;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t seg = 8u * i + (lane >> 3);
        if (msg_bytes == 128u) {
            s[i] = gbase + (uint64_t)seg * 128u + 16u * pp;
        } else {
            s[i] = pp < 4u ? zero : gbase + (uint64_t)seg * 64u + 16u * (pp - 4u);
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
                                                 uint32_t msg_bytes, uint32_t masked,
                                                 uint32_t depth, uint32_t work, uint32_t* sink)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[8 * 2 * kSlotBytes];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t wpb = blockDim.x / 64;
    const uint32_t wl = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)lds +
                        wave * 2 * kSlotBytes;
    const uint64_t stride = (uint64_t)gridDim.x * wpb;
    const uint64_t gbytes = 64ull * msg_bytes;
    const uint64_t exec_mask = (msg_bytes == 64u && masked) ? 0xF0F0F0F0F0F0F0F0ull : ~0ull;
    const uint32_t lane = __lane_id();
    uint32_t acc = threadIdx.x;
    uint64_t s[8];
    auto issue = [&](uint64_t g, uint32_t slot) {
        round_src((uint64_t)(uintptr_t)base + g * gbytes, msg_bytes, s);
        dma_round(slot, s, exec_mask);
    };
    if (depth >= 3) {
        // two groups issued together into both slots, waited for together,
        // then the next pair: adjacent (depth 3: 8 KiB of 64-byte messages
        // contiguous) or half the batch apart (depth 4)
        const uint64_t half = ngroups / 2;
        const uint64_t g0 = depth == 3 ? 2 * (blockIdx.x * wpb + wave) : blockIdx.x * wpb + wave;
        const uint64_t gstep = depth == 3 ? 2 * stride : stride;
        for (uint64_t g = g0; depth == 3 ? g + 1 < ngroups : g < half; g += gstep) {
            issue(g, wl);
            issue(depth == 3 ? g + 1 : g + half, wl + kSlotBytes);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            uint32_t x = 0;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
#pragma unroll
                for (int kk = 0; kk < 8; ++kk) {
                    const uint32_t off = h * kSlotBytes + lane * 128u + 16u * (uint32_t)kk;
                    x ^= *(const __attribute__((address_space(3))) uint32_t*)(uintptr_t)(wl + off);
                }
            }
            acc ^= x;
            acc = fake_work(acc, 2 * work);
        }
        if (acc == 0x12345678u) {
            sink[0] = acc;
        }
        return;
    }
    uint64_t g = blockIdx.x * wpb + wave;
    if (g >= ngroups) {
        return;
    }
    issue(g, wl);
    if (depth == 2 && g + stride < ngroups) {
        issue(g + stride, wl + kSlotBytes);
    }
    for (uint32_t j = 0; g < ngroups; g += stride, ++j) {
        const uint32_t slot = depth == 2 ? wl + (j & 1u) * kSlotBytes : wl;
        if (depth == 2 && g + stride < ngroups) {
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        // read the lane's 128-byte line (8 x 16 bytes) like k_fold's load_line
        uint32_t x = 0;
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {
            const uint32_t off = lane * 128u + 16u * (uint32_t)kk;
            const uint32_t v =
                *(const __attribute__((address_space(3))) uint32_t*)(uintptr_t)(slot + off);
            x ^= v;
        }
        acc ^= x;
        const uint64_t nxt = depth == 2 ? g + 2 * stride : g + stride;
        if (nxt < ngroups) {
            issue(nxt, slot);
        }
        acc = fake_work(acc, work);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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
        uint32_t msg_bytes, masked;
        const char* name;
    };
    const Shape shapes[] = {{128, 0, "128B"}, {64, 0, "64B_zero_half"}, {64, 1, "64B_masked_half"}};
    // per wave and group: 64 messages of msg_bytes; 256 MiB of messages per
    // launch region slice (4 launches cycle the four regions)
    for (const Shape& sh : shapes) {
        const uint64_t ngroups = (256ull << 20) / (64ull * sh.msg_bytes);
        for (uint32_t depth : {1u, 2u, 3u, 4u}) {
            for (uint32_t work : {0u, 200u}) {
                auto launch = [&](int r) {
                    hipLaunchKernelGGL(probe, dim3(cus), dim3(512), 0, 0, buf + (r % nreg) * region,
                                       ngroups, sh.msg_bytes, sh.masked, depth, work, sink);
                };
                for (int w = 0; w < nreg; ++w) {
                    launch(w);
                }
                const int reps = 40;
                hipEventRecord(a, 0);
                for (int r = 0; r < reps; ++r) {
                    launch(r);
                }
                hipEventRecord(b, 0);
                hipEventSynchronize(b);
                float ms = 0;
                hipEventElapsedTime(&ms, a, b);
                const double us = 1000.0 * ms / reps;
                const double bytes = 256.0 * (1 << 20);  // message bytes per launch
                printf("{\"shape\": \"%s\", \"depth\": %u, \"work\": %u, \"us\": %.2f, "
                       "\"msg_TBps\": %.3f, \"frac_of_8TBps\": %.3f}\n",
                       sh.name, depth, work, us, bytes / us / 1e6, bytes / us / 1e6 / 8.0);
                fflush(stdout);
            }
        }
    }
    return 0;
}
