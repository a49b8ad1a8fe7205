#!/bin/bash
# Round 6: piece-major LDS sums (shipped) against the round-5 row-major sums (variants/rm.so:
# -DAPPNP_REM_ROW_MAJOR) on the W8 (F = 40) and W16 (8-rank column slab, 16-column sums) passes,
# alternating.
set -u
C="python bench.py --layout col --emulate 8:0 --steps 10 --warmup 2 --cpu-iters 0"
H="python bench.py --steps 10 --warmup 2 --cpu-iters 0 --features 40"
V="env PPNP_AMD_LIB=variants/rm.so"
T="APPNP_TUNING=1 APPNP_SB_COLS=16"
tools/gpu_session.sh \
  "rm1_f40::300::$V $H" "pm_f40a::300::$H" "rm1_f40b::300::$V $H" "pm_f40b::300::$H" \
  "rm1_c16::240::$V $T $C" "pm_c16a::240::env $T $C" "rm1_c13::240::$V $C" "pm_c13a::240::$C"
