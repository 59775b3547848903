#!/bin/bash
# round 5, GPU call 21: depth probe with adjacent / distant group pairs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r5/call21
mkdir -p $out
timeout -k 10 300 tools/bin/depth_probe > $out/depth_probe2.jsonl 2> $out/depth_probe2.err || exit $?
cat $out/depth_probe2.jsonl
