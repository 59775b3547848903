#!/bin/bash
# round 5, GPU call 9: SQ counters of the one-segment kernel on small messages
# read from HBM (4 rotating copies): LDS-array cycles and bank conflicts
# against wave cycles, and the wave-cycle breakdown (two --pmc passes each,
# no trace domains besides the kernel trace)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r5/sq
mkdir -p $out
A="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
B="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
for w in "1048576 256" "2097152 128" "4194304 64"; do
  set -- $w
  for p in A B; do
    timeout -s KILL 90 rocprofv3 --pmc ${!p} --kernel-trace -d $out/${p}_$1_$2 -o run --output-format csv -- \
      python3 bench.py --config 1M_x_256B --msgs $1 --msg-bytes $2 --rotate 4 --steps 4 --warmup 1 \
      --no-cpu-baseline --settle-seconds 0 --no-kernel-timing > $out/${p}_$1_$2.log 2>&1 || exit $?
    echo "done $p $1 $2"
  done
done
