#!/bin/bash
# Build libbmqcrc.so with extra -D flags into blazingmq_amd/lib/variant_<name>.so
# (same-box A/B: the GPU command swaps it in for a second run), then restore
# the normal build.  usage: tools/build_variant.sh <name> -DFOO=1 ...
set -e
cd "$(dirname "$0")/.."
name=$1; shift
f=blazingmq_amd/csrc/crc32c_kernels.hip
cp $f /tmp/variant_src.hip
{ for d in "$@"; do d=${d#-D}; echo "#define ${d%%=*} ${d#*=}"; done; cat /tmp/variant_src.hip; } > $f
python3 -c "import sys; sys.path.insert(0,'.'); from blazingmq_amd import build; build.build_product(force=True)" > /dev/null
cp blazingmq_amd/lib/libbmqcrc.so blazingmq_amd/lib/variant_$name.so
cp /tmp/variant_src.hip $f
python3 -c "import sys; sys.path.insert(0,'.'); from blazingmq_amd import build; build.build_product(force=True)" > /dev/null
ls -la blazingmq_amd/lib/
