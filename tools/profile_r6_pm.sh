#!/bin/bash
# Round 6: the remainder pass with piece-major LDS sums (bank conflicts of the W8 / W16 passes):
# parity of the split-row tests, then the 8-rank column slab (13-column sums and 16-column), a
# W8 case (F = 40 = 32 + 8) and the headline, and the LDS counters of the 13-column slab.
set -u
C="python bench.py --layout col --emulate 8:0 --steps 10 --warmup 2 --cpu-iters 0"
H="python bench.py --steps 10 --warmup 2 --cpu-iters 0"
P="timeout -s KILL 120 rocprofv3 -o run --output-format csv"
S2="SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_WAIT_INST_LDS"
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider"
tools/gpu_session.sh \
  "pm_tests::400::$T tests/test_gpu_split.py tests/test_gpu_split_rows.py tests/test_gpu_configs.py::test_products_col8_slab_three_row_passes" \
  "pm_c13::240::$C" "pm_c16::240::env APPNP_TUNING=1 APPNP_SB_COLS=16 $C" \
  "pm_f40::300::$H --features 40" "pm_head::300::$H" \
  "pm_sq_c13::150::$P --pmc $S2 -d gpurun_out/pmc6/pm_sq_c13 -- $C"
