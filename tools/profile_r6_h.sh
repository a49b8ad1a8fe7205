#!/bin/bash
# Round 6: do the pipelined shard-group launches (short rows: 6-26 entries per row and launch)
# run faster on G-lane rows (narrow kernel) than a wavefront per row?  APPNP_WIDE=0 (tuning
# override) forces the narrow kernel on every SpMM launch of the emulated rank.
set -u
E="python bench.py --overlap --steps 10 --warmup 2 --cpu-iters 0"
N="env APPNP_TUNING=1 APPNP_WIDE=0"
tools/gpu_session.sh \
  "h_row8_pipe::240::$E --layout row --emulate 8:0" \
  "h_row8_pipe_narrow::240::$N $E --layout row --emulate 8:0" \
  "h_row8_nopipe_narrow::240::$N $E --layout row --emulate 8:0 --pipeline off" \
  "h_r4c2_pipe::240::$E --layout 4x2 --exchange group --emulate 8:0" \
  "h_r4c2_pipe_narrow::240::$N $E --layout 4x2 --exchange group --emulate 8:0" \
  "h_row4_pipe::240::$E --layout row --emulate 4:0" \
  "h_row4_pipe_narrow::240::$N $E --layout row --emulate 4:0"
