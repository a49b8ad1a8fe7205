#!/bin/bash
# Round 6: the remainder pass as two 16-wave workgroups per CU (32 waves, half the LDS and rows
# each; the same row passes) -- variants/wg2.so -- against one (the shipped library): headline
# (W4), F = 40 (W8), the 8-rank column slab (W16).
set -u
B="python bench.py --steps 10 --warmup 2 --cpu-iters 0"
V="env PPNP_AMD_LIB=variants/wg2.so"
tools/gpu_session.sh \
  "l_col8::240::$B --layout col --emulate 8:0" \
  "l_col8_wg2::240::$V $B --layout col --emulate 8:0" \
  "l_head::240::$B" \
  "l_head_wg2::240::$V $B" \
  "l_f40::240::$B --features 40" \
  "l_f40_wg2::240::$V $B --features 40" \
  "l_col8_wg2_b::240::$V $B --layout col --emulate 8:0" \
  "l_col8_b::240::$B --layout col --emulate 8:0"
