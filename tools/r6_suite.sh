#!/bin/bash
# Round 6: the whole GPU suite with per-test durations, then smoke.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6_suite
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider --durations=40 > gpurun_out/r6_suite/gpu_suite.txt 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6_suite/smoke.txt 2>&1 || exit $?
