# Round-3 A/B 7: one-line groups without a zeroed tap array (stail) and a
# raised wave priority around the next group's setup and loads (prio).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
REPS=2 bash tools/ab_args.sh ab7 "base stail prio" \
  "256:--config 1M_x_256B" "64:--config 1M_x_256B --msg-bytes 64" \
  "zipf:--config zipf_4M" "head:--config 64k_x_64KiB"
