#!/bin/bash
# Round 6: piece-major LDS sums with the row-major epilogue (pm2), 8-rank column slab (13 / 16
# columns), F = 40 (W8) and the headline, twice each in alternation.
set -u
C="python bench.py --layout col --emulate 8:0 --steps 10 --warmup 2 --cpu-iters 0"
H="python bench.py --steps 10 --warmup 2 --cpu-iters 0"
tools/gpu_session.sh \
  "pm2_c13::240::$C" "pm2_c16::240::env APPNP_TUNING=1 APPNP_SB_COLS=16 $C" \
  "pm2_f40::300::$H --features 40" "pm2_head::300::$H" \
  "pm2_c13b::240::$C" "pm2_c16b::240::env APPNP_TUNING=1 APPNP_SB_COLS=16 $C"
