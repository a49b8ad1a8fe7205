#!/bin/bash
# Round 6: the new pipelined narrow / two-line rows GPU test.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v --timeout 200 \
  --timeout-method thread -p no:cacheprovider -k "narrow_and_two" > gpurun_out/narrow_test.txt 2>&1
