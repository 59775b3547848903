#!/bin/bash
# round 5, GPU call 29: k_plan_map's short-run slots by start marks and a
# max-scan (product, BMQCRC_SRUN_SCAN=1) against the binary search (variant
# srun0): parity + fuzz suites on the product, Zipf whole / 7/8-shard steps
# alternated, then traced planner times
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
VARIANTS="srun0" PARITY=1 TAG=call29ab ROUNDS=3 STEPS=40 CONFIGS="zipf_4M zipf_4M:7/8" \
  bash tools/r5_ab_multi.sh || exit $?
bash tools/plan_trace_ab.sh r5/call29pt "base srun0 base srun0"
