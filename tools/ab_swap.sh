#!/bin/bash
# Same-box A/B of two library builds: A = blazingmq_amd/lib/libbmqcrc.so,
# B = blazingmq_amd/lib/variant_<name>.so (tools/build_variant.sh), run
# alternately A B A B through tools/ab_configs.sh.  GPU box only.
#   usage: tools/ab_swap.sh <prefix> <name> config ...
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
prefix=$1; name=$2; shift 2
for rep in 1 2; do
    tools/ab_configs.sh "${prefix}_A$rep" base "$@"
    tools/ab_configs.sh "${prefix}_B$rep" "$name" "$@"
done
