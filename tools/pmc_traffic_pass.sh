#!/bin/bash
# FETCH_SIZE and WRITE_SIZE of every kernel of one bench.py run, each counter
# in its own rocprofv3 pass (kernel trace only), for traffic attribution.
#   usage (GPU box): tools/pmc_traffic_pass.sh <out dir> <bench args...>
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=$1; shift
mkdir -p "$out"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d $out/$c -o run --output-format csv -- \
    python3 bench.py "$@" --steps 5 --warmup 2 --no-cpu-baseline --settle-seconds 0 \
    --no-kernel-timing > $out/$c.log 2>&1 || exit $?
  echo "done $c"
done
