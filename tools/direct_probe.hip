// Direct-load probe (diagnostic, not product code): can one lane per short
// message, loading its own bytes straight into VGPRs (global_load_dwordx4
// nt, no LDS staging), stream a batch of 256-byte messages near the HBM
// roofline with k_fold-like per-message work?  The LDS-DMA staging of k_fold
// caps a CU at 8 waves x 2 slots x 8 KiB in flight; VGPRs hold 3x more.
//
//   probe <msg_bytes> <n_msgs> <word_work> <group_work> <mode>
//     word_work   VALU per data word (k_fold's fold: 6)
//     group_work  VALU per message after its data (k_fold's tail + combine:
//                 ~500 for a 2-line segment)
//     mode 0      one group in flight per wave
//     mode 1      the next group's loads issued before this group's work
// One JSON line per kernel variant (2 / 4 waves per SIMD by launch bounds).
// Build: hipcc --offload-arch=gfx950 -O3 tools/direct_probe.hip -o /tmp/direct_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int PIECES>
__device__ __forceinline__ void load_msg(const u32x4* p, u32x4 (&d)[PIECES])
{
#pragma unroll
    for (int i = 0; i < PIECES; ++i) {
        d[i] = __builtin_nontemporal_load(p + i);
    }
}

__device__ __forceinline__ uint32_t chain(uint32_t v, uint32_t w, int n)
{
    for (int k = 0; k < n; ++k) {
        v = __builtin_amdgcn_bitop3_b32(v, w, v >> 3, 0x96);
    }
    return v;
}

template <int PIECES, int WPS, int MODE>
__global__ __launch_bounds__(256, WPS) void k_probe(const uint8_t* base, uint32_t msg_bytes,
                                                    uint64_t n, int word_work, int group_work,
                                                    uint32_t* out)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    uint64_t g = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint64_t ngroups = (n + 63) / 64;
    u32x4 cur[PIECES], nxt[PIECES];
    if (g < ngroups) {
        const uint64_t m = min(g * 64 + lane, n - 1);
        load_msg<PIECES>((const u32x4*)(base + m * msg_bytes), cur);
    }
    for (; g < ngroups; g += waves) {
        const uint64_t m = g * 64 + lane;
        if (MODE == 1 && g + waves < ngroups) {
            const uint64_t m2 = min((g + waves) * 64 + lane, n - 1);
            load_msg<PIECES>((const u32x4*)(base + m2 * msg_bytes), nxt);
        }
        uint32_t v = (uint32_t)m;
#pragma unroll
        for (int i = 0; i < PIECES; ++i) {
            v = chain(v, cur[i].x, word_work);
            v = chain(v, cur[i].y, word_work);
            v = chain(v, cur[i].z, word_work);
            v = chain(v, cur[i].w, word_work);
        }
        v = chain(v, v * 7u, group_work);
        if (m < n) {
            out[m] = v;
        }
        if (MODE == 1) {
#pragma unroll
            for (int i = 0; i < PIECES; ++i) {
                cur[i] = nxt[i];
            }
        } else if (g + waves < ngroups) {
            const uint64_t m2 = min((g + waves) * 64 + lane, n - 1);
            load_msg<PIECES>((const u32x4*)(base + m2 * msg_bytes), cur);
        }
    }
}

template <int PIECES, int WPS, int MODE>
static void run(const uint8_t* d, uint32_t msg_bytes, uint64_t n, int ww, int gw, uint32_t* out,
                int cus)
{
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int grid = cus * WPS;  // 4 waves per block: WPS blocks per CU = WPS waves per SIMD
    for (int i = 0; i < 20; ++i) {
        hipLaunchKernelGGL((k_probe<PIECES, WPS, MODE>), dim3(grid), dim3(256), 0, 0, d, msg_bytes,
                           n, ww, gw, out);
    }
    (void)hipEventRecord(a, 0);
    const int reps = 50;
    for (int i = 0; i < reps; ++i) {
        hipLaunchKernelGGL((k_probe<PIECES, WPS, MODE>), dim3(grid), dim3(256), 0, 0, d, msg_bytes,
                           n, ww, gw, out);
    }
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    const double us = ms * 1e3 / reps;
    printf("{\"msg_bytes\": %u, \"n\": %llu, \"word_work\": %d, \"group_work\": %d, "
           "\"mode\": %d, \"waves_per_simd\": %d, \"us\": %.2f, \"TBps\": %.3f}\n",
           msg_bytes, (unsigned long long)n, ww, gw, MODE, WPS, us,
           (double)n * msg_bytes / us / 1e6);
}

int main(int argc, char** argv)
{
    const uint32_t msg = argc > 1 ? atoi(argv[1]) : 256;
    const uint64_t n = argc > 2 ? strtoull(argv[2], 0, 0) : (1u << 20);
    const int ww = argc > 3 ? atoi(argv[3]) : 6;
    const int gw = argc > 4 ? atoi(argv[4]) : 500;
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    uint8_t* d = nullptr;
    uint32_t* out = nullptr;
    if (hipMalloc(&d, n * msg + 4096) != hipSuccess || hipMalloc(&out, n * 4) != hipSuccess) {
        return 1;
    }
    (void)hipMemset(d, 0x5A, n * msg + 4096);
    if (msg != 256) {
        fprintf(stderr, "probe built for 256-byte messages\n");
        return 1;
    }
    run<16, 2, 0>(d, msg, n, ww, gw, out, cus);
    run<16, 4, 0>(d, msg, n, ww, gw, out, cus);
    run<16, 2, 1>(d, msg, n, ww, gw, out, cus);
    run<16, 3, 1>(d, msg, n, ww, gw, out, cus);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
