#!/bin/bash
# Round 6: entries in flight (APPNP_UW) on the 25-column slabs (one line per gather, 8 sub-groups
# per wave): the 2 x 4 rank (projected N = 8 winner) and the 4-rank column layout.
set -u
E="python bench.py --overlap --steps 10 --warmup 2 --cpu-iters 0"
C="python bench.py --steps 10 --warmup 2 --cpu-iters 0"
T="env APPNP_TUNING=1"
tools/gpu_session.sh \
  "k_r2c4_auto::240::$E --layout 2x4 --emulate 8:0" \
  "k_r2c4_uw4::240::$T APPNP_UW=4 $E --layout 2x4 --emulate 8:0" \
  "k_r2c4_uw8::240::$T APPNP_UW=8 $E --layout 2x4 --emulate 8:0" \
  "k_col4_auto::240::$C --layout col --emulate 4:0" \
  "k_col4_uw4::240::$T APPNP_UW=4 $C --layout col --emulate 4:0" \
  "k_col2l_auto::240::$C --layout col-lines --emulate 2:0" \
  "k_col2l_uw4::240::$T APPNP_UW=4 $C --layout col-lines --emulate 2:0"
