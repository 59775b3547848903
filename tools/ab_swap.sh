#!/bin/bash
# Same-box A/B of two library builds: A = blazingmq_amd/lib/libbmqcrc.so,
# B = blazingmq_amd/lib/variant_<name>.so (tools/build_variant.sh), run
# alternately A B A B through tools/ab_configs.sh.  GPU box only.
#   usage: tools/ab_swap.sh <prefix> <name> "<tunes>" config ...
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
prefix=$1; name=$2; tunes=$3; shift 3
lib=blazingmq_amd/lib
cp $lib/libbmqcrc.so /tmp/ab_base.so
for rep in 1 2; do
    cp /tmp/ab_base.so $lib/libbmqcrc.so
    tools/ab_configs.sh "${prefix}_A$rep" "$tunes" "$@"
    cp $lib/variant_$name.so $lib/libbmqcrc.so
    tools/ab_configs.sh "${prefix}_B$rep" "$tunes" "$@"
done
cp /tmp/ab_base.so $lib/libbmqcrc.so
