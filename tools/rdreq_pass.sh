#!/bin/bash
# TCC_EA0_RDREQ / TCC_EA0_RDREQ_32B per k_fold launch of one bench.py
# argument set (one rocprofv3 pass, kernel trace only): the request-size mix
# behind FETCH_SIZE, whose x2 correction is calibrated for 128-byte requests
# only (MI355X_MICROARCH.md, HBM).
#   usage (GPU box): tools/rdreq_pass.sh <out dir> <bench args...>
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=$1; shift
mkdir -p "$out"
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-trace \
    -d $out/rdreq -o run --output-format csv -- \
    python3 bench.py "$@" --steps 5 --warmup 2 --no-cpu-baseline --settle-seconds 0 \
    --no-kernel-timing > $out/rdreq.log 2>&1
