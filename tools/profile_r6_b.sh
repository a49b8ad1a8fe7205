#!/bin/bash
# Round 6: the pipelined row exchange on the GPU (multi-rank tests sharing the GPU over gloo),
# the compute cost of the pipelined 8-rank row layout per rank (--emulate 8:r, pipeline on/off),
# and the piece-major / row-major A/B of the remainder pass's LDS sums (variants/rm.so).
set -u
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
E="python bench.py --layout row --overlap --steps 10 --warmup 2 --cpu-iters 0"
C="python bench.py --layout col --emulate 8:0 --steps 10 --warmup 2 --cpu-iters 0"
H="python bench.py --steps 10 --warmup 2 --cpu-iters 0 --features 40"
V="env PPNP_AMD_LIB=variants/rm.so"
tools/gpu_session.sh \
  "b_tests::600::$T tests/test_gpu_configs.py -k 'arxiv_row_partition or native_row_engine_matches or native_row_engine_split_rows or row_partition_split_rows or rccl_callback'" \
  "b_row8_r0_pipe::240::$E --emulate 8:0" "b_row8_r0_nopipe::240::$E --emulate 8:0 --pipeline off" \
  "b_row8_r3_pipe::240::$E --emulate 8:3" "b_row8_r3_nopipe::240::$E --emulate 8:3 --pipeline off" \
  "b_row8_r7_pipe::240::$E --emulate 8:7" "b_row2_r0::240::$E --emulate 2:0" \
  "rm1_f40::300::$V $H" "pm_f40a::300::$H" "rm1_f40b::300::$V $H" "pm_f40b::300::$H" \
  "rm1_c16::240::$V env APPNP_TUNING=1 APPNP_SB_COLS=16 $C" "pm_c16a::240::env APPNP_TUNING=1 APPNP_SB_COLS=16 $C"
