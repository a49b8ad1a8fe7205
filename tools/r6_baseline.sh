#!/bin/bash
# Round 6 baseline on the round-5 sources: the GPU suite with per-test durations, then the
# 8-rank column slab emulation (the W16 remainder pass of VERDICT r5 next #1).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6_base
timeout -k 10 880 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  --durations=40 -p no:cacheprovider > gpurun_out/r6_base/gpu_suite.txt 2>&1 || exit $?
timeout -k 10 240 python -u bench.py --layout col --emulate 8:0 --steps 10 --warmup 2 --cpu-iters 0 \
  > gpurun_out/r6_base/col8.json 2> gpurun_out/r6_base/col8.log || exit $?
