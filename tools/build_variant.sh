#!/bin/bash
# Build libbmqcrc.so with extra -D flags (e.g. -DBMQCRC_TUNE_BITS=2, see
# csrc/bmqcrc_internal.h) into blazingmq_amd/lib/variant_<name>.so for a
# same-box A/B (tools/ab_swap.sh swaps it in for a second run).  The product
# build (libbmqcrc.so) is left untouched.
#   usage: tools/build_variant.sh <name> -DFOO=1 ...
set -e
cd "$(dirname "$0")/.."
name=$1; shift
python3 - "$name" "$@" <<'PY'
import sys
sys.path.insert(0, '.')
from blazingmq_amd import build
build.build_product(force=True, defines=sys.argv[2:], target_name="variant_%s.so" % sys.argv[1])
PY
ls -la blazingmq_amd/lib/
