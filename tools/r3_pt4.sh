# Round-3: where k_plan_map spends its time (kernel traces): phase 1 alone
# (pd1), phase 1 + the grid-wide wait (pd2), the whole kernel (base), and the
# round-2 pair (r2), on Zipf 4M and its 1/8 shard.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/plan_trace_ab.sh pt4 "oldplan r2 pd1 base"
