#!/bin/bash
# Round 6, VERDICT r5 next #1: A/B of the 8-rank column slab's W16 pass (13 columns of F = 100;
# bench --layout col --emulate 8:0): sums packed to 52 B per row (3 row passes + 40,581 direct
# rows) against the round-5 layout (64 B, 4 passes), and the pieces between them; then the
# L2 hit / miss counters of the default.  Knobs: APPNP_TUNING=1 with APPNP_SB_COLS (size the pass
# for more columns), APPNP_SB_DIRECT (0: no direct rows), APPNP_REM_SYNC_W16 (barrier period).
set -u
B="python bench.py --layout col --emulate 8:0 --steps 10 --warmup 2 --cpu-iters 0"
T="env APPNP_TUNING=1"
P="timeout -s KILL 200 rocprofv3 -o run --output-format csv"
tools/gpu_session.sh \
  "w16_c13::240::$B" \
  "w16_c13_nodirect::240::$T APPNP_SB_DIRECT=0 $B" \
  "w16_c16::240::$T APPNP_SB_COLS=16 $B" \
  "w16_c16_direct4::240::$T APPNP_SB_COLS=16 APPNP_SB_DIRECT=4 $B" \
  "w16_c13_sync16::240::$T APPNP_REM_SYNC_W16=16 $B" \
  "w16_c13_sync64::240::$T APPNP_REM_SYNC_W16=64 $B" \
  "w16_c13_l2::240::$P --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc6/w16_c13/l2 -- $B" \
  "w16_c16_l2::240::APPNP_TUNING=1 APPNP_SB_COLS=16 $P --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc6/w16_c16/l2 -- $B"
