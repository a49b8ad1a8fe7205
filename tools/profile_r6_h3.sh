#!/bin/bash
# Round 6: entries in flight per sub-group (APPNP_UW, tuning override) on the pipelined
# shard-group launches, whose short rows (< 24 entries on average) get 1 by the rule.
set -u
E="python bench.py --overlap --steps 10 --warmup 2 --cpu-iters 0"
T="env APPNP_TUNING=1"
tools/gpu_session.sh \
  "h3_row8_uw1::240::$T APPNP_UW=1 $E --layout row --emulate 8:0" \
  "h3_row8_auto::240::$E --layout row --emulate 8:0" \
  "h3_row8_uw2::240::$T APPNP_UW=2 $E --layout row --emulate 8:0" \
  "h3_row8_uw4::240::$T APPNP_UW=4 $E --layout row --emulate 8:0" \
  "h3_r4c2_auto::240::$E --layout 4x2 --exchange group --emulate 8:0" \
  "h3_r4c2_uw2::240::$T APPNP_UW=2 $E --layout 4x2 --exchange group --emulate 8:0" \
  "h3_r4c2_uw4::240::$T APPNP_UW=4 $E --layout 4x2 --exchange group --emulate 8:0" \
  "h3_row8np_uw2::240::$T APPNP_UW=2 $E --layout row --emulate 8:0 --pipeline off"
