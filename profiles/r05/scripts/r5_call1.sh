#!/bin/bash
# round 5, GPU call 1: GPU suite (graph-capture fix, given-up timing bound),
# then the scalar CRC ladder and method A/B on the GPU box's host CPU
set -o pipefail
mkdir -p gpurun_out/r5
lscpu > gpurun_out/r5/lscpu.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/r5/gpu_suite_1.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --scalar > gpurun_out/r5/scalar_ladder.jsonl 2> gpurun_out/r5/scalar_ladder.err || exit $?
g++ -O2 -std=c++17 tools/scalar_ab.cpp -o gpurun_out/r5/scalar_ab || exit $?
timeout -k 10 120 gpurun_out/r5/scalar_ab check > gpurun_out/r5/scalar_ab_check.txt 2>&1 || exit $?
timeout -k 10 300 gpurun_out/r5/scalar_ab time > gpurun_out/r5/scalar_ab_time.jsonl 2>&1 || exit $?
timeout -k 10 120 gpurun_out/r5/scalar_ab time 10 64 80 96 112 128 144 160 176 192 224 256 320 384 512 > gpurun_out/r5/scalar_ab_sweep.jsonl 2>&1
