#!/bin/bash
# Round 6: the narrow kernel (G-lane rows, 64/G rows per wave) at G = 16 / 32 against a
# wavefront per row, forced on every SpMM launch (APPNP_TUNING=1 APPNP_WIDE=0) with
# variants/narrow32.so (launch_narrow extended to G = 16, 32): the pipelined shard-group
# launches have short rows (6-26 entries per row and launch).
set -u
E="python bench.py --overlap --steps 10 --warmup 2 --cpu-iters 0"
V="env PPNP_AMD_LIB=variants/narrow32.so"
N="env PPNP_AMD_LIB=variants/narrow32.so APPNP_TUNING=1 APPNP_WIDE=0"
tools/gpu_session.sh \
  "h2_row8_pipe_v::240::$V $E --layout row --emulate 8:0" \
  "h2_row8_pipe_narrow::240::$N $E --layout row --emulate 8:0" \
  "h2_row8_nopipe_narrow::240::$N $E --layout row --emulate 8:0 --pipeline off" \
  "h2_row8_nopipe_v::240::$V $E --layout row --emulate 8:0 --pipeline off" \
  "h2_r4c2_pipe_narrow::240::$N $E --layout 4x2 --exchange group --emulate 8:0" \
  "h2_r4c2_pipe_v::240::$V $E --layout 4x2 --exchange group --emulate 8:0" \
  "h2_row4_pipe_narrow::240::$N $E --layout row --emulate 4:0" \
  "h2_head_narrow::240::$N python bench.py --steps 10 --warmup 2 --cpu-iters 0"
