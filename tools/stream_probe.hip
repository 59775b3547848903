// stream_probe.hip -- read-only HBM streaming ceiling on this MI355X
// ("report a measured read-only streaming kernel ceiling on the
// same box as context").  Diagnostic only; not part of the product.
//   probe_read_x4:   global_load_dwordx4 grid-stride, XOR-reduced per thread
//   probe_read_glds: per-wave LDS-DMA ring (the k_fold staging pattern) with
//                    no compute: 8 x 1 KiB global_load_lds_dwordx4 per round
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

__global__ __launch_bounds__(256, 2) void probe_read_glds(const uint8_t* __restrict__ base,
                                                           uint64_t nbytes, uint32_t* out)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[65536];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wl = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)lds + wave * 16384u;
    const uint64_t per_round = 8192;  // one wave round
    const uint64_t nrounds = nbytes / per_round;
    const uint64_t total_waves = (uint64_t)gridDim.x * 4;
    uint32_t slot = 0, k = 0, acc = 0;
    for (uint64_t r = (uint64_t)blockIdx.x * 4 + wave; r < nrounds; r += total_waves) {
        const uint8_t* s0 = base + r * per_round + 16u * lane;
        const uint32_t dst = wl + slot * 8192u;
        asm volatile(
            "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
            "global_load_lds_dwordx4 %2, off\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
            "global_load_lds_dwordx4 %3, off\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
            "global_load_lds_dwordx4 %4, off\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
            "global_load_lds_dwordx4 %5, off\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
            "global_load_lds_dwordx4 %6, off\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
            "global_load_lds_dwordx4 %7, off\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
            "global_load_lds_dwordx4 %8, off\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
            "global_load_lds_dwordx4 %9, off\n\t"
            "s_mov_b32 m0, %0\n\t"
            : "=&s"(k) : "s"(dst), "v"(s0), "v"(s0 + 1024), "v"(s0 + 2048), "v"(s0 + 3072),
              "v"(s0 + 4096), "v"(s0 + 5120), "v"(s0 + 6144), "v"(s0 + 7168) : "memory", "scc");
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        acc ^= *(const __attribute__((address_space(3))) uint32_t*)(uintptr_t)(wl + (slot ^ 1u) * 8192u + 4u * lane);
        slot ^= 1u;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

extern "C" int probe_launch(int which, const void* p, uint64_t nbytes, uint32_t* out, int grid,
                            void* stream)
{
    hipStream_t s = (hipStream_t)stream;
    if (which == 0 || which == 1) {
        hipLaunchKernelGGL(probe_read_x4, dim3(grid), dim3(256), 0, s, (const u32x4*)p, nbytes / 16,
                           out, which);
    } else {
        hipLaunchKernelGGL(probe_read_glds, dim3(grid), dim3(256), 0, s, (const uint8_t*)p, nbytes,
                           out);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
