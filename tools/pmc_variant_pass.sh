#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (tools/pmc_traffic_pass.sh) of one bench.py
# argument set with a variant library swapped in, the product restored after.
#   usage (GPU box): tools/pmc_variant_pass.sh <out dir> <variant|base> <bench args...>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=$1; v=$2; shift 2
lib=blazingmq_amd/lib
cp $lib/libbmqcrc.so /tmp/pmc_variant_base.so
[ "$v" = base ] || cp $lib/variant_$v.so $lib/libbmqcrc.so
rc=0
bash tools/pmc_traffic_pass.sh "$out" "$@" || rc=$?
cp /tmp/pmc_variant_base.so $lib/libbmqcrc.so
exit $rc
