#!/bin/bash
# SQ counters of k_fold for any bench.py configuration: the two --pmc passes
# of tools/sq_small.sh (A: LDS cycles, conflicts, instruction counts; B: the
# wave-cycle breakdown), each its own run with the kernel trace only.
# usage (on the box): tools/sq_config.sh <out dir> <tag> <bench args...>
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=$1; tag=$2; shift 2
mkdir -p "$out"
A="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
B="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
for p in A B; do
  timeout -s KILL 120 rocprofv3 --pmc ${!p} --kernel-trace -d $out/${p}_$tag -o run --output-format csv -- \
    python3 bench.py "$@" --steps 4 --warmup 1 --no-cpu-baseline --settle-seconds 0 \
    --no-kernel-timing > $out/${p}_$tag.log 2>&1 || exit $?
  echo "done $p $tag"
done
