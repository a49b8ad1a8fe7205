#!/bin/bash
# Round 6, first look: the new tests (direct rows, test-library hooks, timer), the 8-rank column
# slab emulation (W16 pass sized for 13 columns) and the headline bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6_a
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_probe.py "tests/test_gpu_split.py" \
  "tests/test_gpu_configs.py::test_products_col8_slab_three_row_passes" \
  "tests/test_gpu_configs.py::test_split_decision_is_collective" \
  "tests/test_gpu_configs.py::test_native_row_engine_poisoned_after_failed_agreement" \
  --durations=30 > $O/tests.txt 2>&1 || exit $?
timeout -k 10 240 python -u bench.py --layout col --emulate 8:0 --steps 10 --warmup 2 --cpu-iters 0 \
  > $O/col8.json 2> $O/col8.log || exit $?
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.log || exit $?
