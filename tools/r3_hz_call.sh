#!/bin/bash
# One GPU call: Horner-chain A/B (tools/r3_ab_horner.sh), then the GPU suite
# on the chosen variant's library.  GPU box only.
#   usage: tools/r3_hz_call.sh <prefix> <variant>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export BMQCRC_GOLDEN_DIR=$PWD/tests/golden
bash tools/r3_ab_horner.sh "$1" > gpurun_out/$1_ab.log 2>&1 || { echo "A/B failed"; tail -5 gpurun_out/$1_ab.log; exit 1; }
grep -v "^==" gpurun_out/$1_ab.log | tail -30
cp blazingmq_amd/lib/variant_$2.so blazingmq_amd/lib/libbmqcrc.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/$1_gputests.log 2>&1; rc=$?
tail -3 gpurun_out/$1_gputests.log
exit $rc
