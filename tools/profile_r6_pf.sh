#!/bin/bash
# Round 6: the remainder pass with the next chunks' entries prefetched under the current
# gathers (variants/pf.so: -DAPPNP_REM_PREFETCH) against the shipped pass, on the 8-rank column
# slab (W16, sized for 13 and for 16 columns) and on the headline (W4 remainder of F = 100).
set -u
C="python bench.py --layout col --emulate 8:0 --steps 10 --warmup 2 --cpu-iters 0"
H="python bench.py --steps 10 --warmup 2 --cpu-iters 0"
V="env PPNP_AMD_LIB=variants/pf.so"
T="APPNP_TUNING=1 APPNP_SB_COLS=16"
tools/gpu_session.sh \
  "pf0_c13::240::$C" "pf1_c13::240::$V $C" \
  "pf0_c16::240::env $T $C" "pf1_c16::240::$V $T $C" \
  "pf0_head::300::$H" "pf1_head::300::$V $H" \
  "pf1_c13_b::240::$V $C" "pf0_c13_b::240::$C"
