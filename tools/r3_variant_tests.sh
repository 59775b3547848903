#!/bin/bash
# Run GPU tests against a variant build swapped in for the product.
#   usage (on the box): tools/r3_variant_tests.sh <variant> <log> [pytest args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
v=$1; log=$2; shift 2
L=blazingmq_amd/lib
mkdir -p gpurun_out
cp $L/libbmqcrc.so /tmp/vt_base.so
cp $L/variant_$v.so $L/libbmqcrc.so
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu "$@" > $log 2>&1
rc=$?
cp /tmp/vt_base.so $L/libbmqcrc.so
tail -3 $log
exit $rc
