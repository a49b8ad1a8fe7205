#!/bin/bash
# Round 6: the whole -m gpu suite with every test's duration (after sharing the
# products reference), then the epilogue-operand prefetch A/B: the partial / dH loaded when a
# row starts (this tree) against after its gathers (variants/nopv.so, the previous SpMM unit) on
# the row layouts' accumulate / finish launches, the adjoint and the headline.
set -u
T="python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider --durations=0"
E="python bench.py --layout row --overlap --steps 10 --warmup 2 --cpu-iters 0"
H="python bench.py --steps 10 --warmup 2 --cpu-iters 0"
V="env PPNP_AMD_LIB=variants/nopv.so"
tools/gpu_session.sh \
  "c_suite::900::$T" \
  "c_row8_r0_pipe::240::$E --emulate 8:0" "c_row8_r0_pipe_nopv::240::$V $E --emulate 8:0" \
  "c_row8_r0_nopipe::240::$E --emulate 8:0 --pipeline off" \
  "c_row8_r0_nopipe_nopv::240::$V $E --emulate 8:0 --pipeline off" \
  "c_row8_r3_pipe::240::$E --emulate 8:3" "c_row8_r3_pipe_nopv::240::$V $E --emulate 8:3" \
  "c_row2_r0::240::$E --emulate 2:0" "c_row2_r0_nopv::240::$V $E --emulate 2:0" \
  "c_bwd::240::python tools/bwd_time.py" "c_bwd_nopv::240::$V python tools/bwd_time.py" \
  "c_head::240::$H" "c_head_nopv::240::$V $H" "c_row8_r0_pipe_b::240::$E --emulate 8:0"
