// stream_probe.hip -- read-only HBM streaming ceiling on this MI355X
// ("report a measured read-only streaming kernel ceiling on the
// same box as context").  Diagnostic only; not part of the product.
//   probe_read_x4:   global_load_dwordx4 grid-stride, XOR-reduced per thread
//   probe_read_glds: per-wave LDS-DMA ring with no compute, 8 x 1 KiB
//                    global_load_lds_dwordx4 per round: contiguous chunks, or
//                    k_fold's headline shape (64 segments per wave, one line of
//                    each per round), default or non-temporal policy
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void probe_read_x4(const u32x4* __restrict__ p, uint64_t n16,
                                                     uint32_t* out, int nt)
{
    u32x4 acc = {0, 0, 0, 0};
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (nt) {
        for (; i + 3 * stride < n16; i += 4 * stride) {
            u32x4 a = __builtin_nontemporal_load(p + i), b = __builtin_nontemporal_load(p + i + stride);
            u32x4 c = __builtin_nontemporal_load(p + i + 2 * stride), d = __builtin_nontemporal_load(p + i + 3 * stride);
            acc ^= a ^ b ^ c ^ d;
        }
    } else {
        for (; i + 3 * stride < n16; i += 4 * stride) {
            u32x4 a = p[i], b = p[i + stride], c = p[i + 2 * stride], d = p[i + 3 * stride];
            acc ^= a ^ b ^ c ^ d;
        }
    }
    for (; i < n16; i += stride) {
        acc ^= p[i];
    }
    out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// One round of 8 x global_load_lds_dwordx4 (8 x 1 KiB) into LDS at dst; NT
// selects the non-temporal policy k_fold uses.
template <bool NT>
__device__ __forceinline__ void glds_round(uint32_t dst, const uint8_t* const (&s)[8])
{
    uint32_t k;
#define PROBE_DMA(CP)                                                                          \
    "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"                                    \
    "global_load_lds_dwordx4 %2, off" CP "\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"          \
    "global_load_lds_dwordx4 %3, off" CP "\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"          \
    "global_load_lds_dwordx4 %4, off" CP "\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"          \
    "global_load_lds_dwordx4 %5, off" CP "\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"          \
    "global_load_lds_dwordx4 %6, off" CP "\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"          \
    "global_load_lds_dwordx4 %7, off" CP "\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"          \
    "global_load_lds_dwordx4 %8, off" CP "\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"          \
    "global_load_lds_dwordx4 %9, off" CP "\n\t"                                                \
    "s_mov_b32 m0, %0\n\t"
    if (NT) {
        asm volatile(PROBE_DMA(" nt") : "=&s"(k) : "s"(dst), "v"(s[0]), "v"(s[1]), "v"(s[2]),
                     "v"(s[3]), "v"(s[4]), "v"(s[5]), "v"(s[6]), "v"(s[7]) : "memory", "scc");
    } else {
        asm volatile(PROBE_DMA("") : "=&s"(k) : "s"(dst), "v"(s[0]), "v"(s[1]), "v"(s[2]),
                     "v"(s[3]), "v"(s[4]), "v"(s[5]), "v"(s[6]), "v"(s[7]) : "memory", "scc");
    }
#undef PROBE_DMA
}

// Per-wave LDS-DMA ring with no compute, two 8 KiB slots per wave.
//   SEGMENTED = false: a wave's rounds are consecutive 8 KiB chunks of the
//     buffer, grid-strided over the waves;
//   SEGMENTED = true:  k_fold's headline shape -- a wave owns 64 segments of
//     seg_bytes and every round reads the next 128-byte line of each (8 lanes
//     per line, 8 segments per instruction), groups grid-strided.
template <bool NT, bool SEGMENTED>
__global__ __launch_bounds__(256, 1) void probe_read_glds(const uint8_t* __restrict__ base,
                                                           uint64_t nbytes, uint32_t seg_bytes,
                                                           uint32_t* out)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[65536];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wl = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)lds +
                        wave * 16384u;
    const uint64_t total_waves = (uint64_t)gridDim.x * 4;
    uint32_t slot = 0, acc = 0, inflight = 0;
    auto consume = [&]() {
        acc ^= *(const __attribute__((address_space(3))) uint32_t*)(uintptr_t)(
            wl + (slot ^ 1u) * 8192u + 4u * lane);
    };
    if (!SEGMENTED) {
        const uint64_t nrounds = nbytes / 8192u;
        for (uint64_t r = (uint64_t)blockIdx.x * 4 + wave; r < nrounds; r += total_waves) {
            const uint8_t* s0 = base + r * 8192u + 16u * lane;
            const uint8_t* const s[8] = {s0, s0 + 1024, s0 + 2048, s0 + 3072,
                                         s0 + 4096, s0 + 5120, s0 + 6144, s0 + 7168};
            glds_round<NT>(wl + slot * 8192u, s);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            consume();
            slot ^= 1u;
        }
    } else {
        const uint64_t gbytes = 64ull * seg_bytes;
        const uint64_t ngroups = nbytes / gbytes;
        const uint32_t lines = seg_bytes / 128u;
        for (uint64_t g = (uint64_t)blockIdx.x * 4 + wave; g < ngroups; g += total_waves) {
            const uint8_t* gb = base + g * gbytes + 16u * (lane & 7u);
            for (uint32_t r = 0; r < lines; ++r) {
                const uint8_t* s[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    s[i] = gb + (uint64_t)(8u * i + (lane >> 3)) * seg_bytes + 128u * r;
                }
                glds_round<NT>(wl + slot * 8192u, s);
                if (inflight) {
                    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                    consume();
                }
                inflight = 1;
                slot ^= 1u;
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

extern "C" int probe_launch(int which, const void* p, uint64_t nbytes, uint32_t* out, int grid,
                            uint32_t seg_bytes, void* stream)
{
    // which: 0 dwordx4, 1 dwordx4 nt, 2 LDS-DMA contiguous, 3 LDS-DMA contiguous nt,
    //        4 LDS-DMA segmented (k_fold shape), 5 LDS-DMA segmented nt
    hipStream_t s = (hipStream_t)stream;
    const uint8_t* b = (const uint8_t*)p;
    switch (which) {
    case 0:
    case 1:
        hipLaunchKernelGGL(probe_read_x4, dim3(grid), dim3(256), 0, s, (const u32x4*)p, nbytes / 16,
                           out, which);
        break;
    case 2: hipLaunchKernelGGL((probe_read_glds<false, false>), dim3(grid), dim3(256), 0, s, b, nbytes, seg_bytes, out); break;
    case 3: hipLaunchKernelGGL((probe_read_glds<true, false>), dim3(grid), dim3(256), 0, s, b, nbytes, seg_bytes, out); break;
    case 4: hipLaunchKernelGGL((probe_read_glds<false, true>), dim3(grid), dim3(256), 0, s, b, nbytes, seg_bytes, out); break;
    case 5: hipLaunchKernelGGL((probe_read_glds<true, true>), dim3(grid), dim3(256), 0, s, b, nbytes, seg_bytes, out); break;
    default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
