#!/bin/bash
# VGPR / SGPR / LDS / scratch of every kernel in crc32c_kernels.hip (gfx950),
# from the compiler's resource-usage remarks.  CPU only.
#   usage: tools/kernel_resources.sh [extra hipcc flags]
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 --offload-device-only -O3 -std=c++17 \
    -Iinclude -c blazingmq_amd/csrc/crc32c_kernels.hip -o /tmp/bmqcrc_res.o \
    -Rpass-analysis=kernel-resource-usage "$@" 2>&1 |
    grep -E "Function Name|VGPRs:|AGPRs|ScratchSize|Occupancy|LDS Size" |
    sed -e 's/.*remark: //' | paste - - - - - - | grep -E "k_fold|k_plan"
