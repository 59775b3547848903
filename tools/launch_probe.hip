// Cost of a kernel whose blocks read one control word and exit, by block
// size: is an early-exit planner launch bound by wave launch?
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k_exit(const unsigned* ctrl, unsigned* sink)
{
    if (ctrl[0] == 0u) {
        return;
    }
    sink[blockIdx.x] = threadIdx.x;
}

int main()
{
    unsigned *ctrl, *sink;
    hipMalloc(&ctrl, 4);
    hipMalloc(&sink, 1 << 20);
    hipMemset(ctrl, 0, 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int threads[] = {64, 256, 512, 1024};
    for (int t : threads) {
        for (int blocks : {64, 256}) {
            for (int w = 0; w < 50; ++w) {
                hipLaunchKernelGGL(k_exit, dim3(blocks), dim3(t), 0, 0, ctrl, sink);
            }
            hipEventRecord(a, 0);
            const int reps = 2000;
            for (int r = 0; r < reps; ++r) {
                hipLaunchKernelGGL(k_exit, dim3(blocks), dim3(t), 0, 0, ctrl, sink);
            }
            hipEventRecord(b, 0);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            printf("{\"blocks\": %d, \"threads\": %d, \"us_per_launch\": %.3f}\n", blocks, t,
                   1000.0 * ms / reps);
        }
    }
    return 0;
}
