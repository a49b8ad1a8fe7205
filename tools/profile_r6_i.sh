#!/bin/bash
# Round 6: two entries in flight on short rows that are ranges of long rows (launch_step):
# the 8-rank row layout pipelined (ranks 0 and 3) and not, the 4 x 2 pipelined rank, arxiv-synth
# and the headline on the new library; then the whole -m gpu suite.
set -u
E="python bench.py --overlap --steps 10 --warmup 2 --cpu-iters 0"
B="python bench.py --steps 10 --warmup 2 --cpu-iters 0"
tools/gpu_session.sh \
  "i_row8_pipe::240::$E --layout row --emulate 8:0" \
  "i_row8_pipe_r3::240::$E --layout row --emulate 8:3" \
  "i_row8_nopipe::240::$E --layout row --emulate 8:0 --pipeline off" \
  "i_r4c2_pipe::240::$E --layout 4x2 --exchange group --emulate 8:0" \
  "i_r4c2_relay::240::$E --layout 4x2 --emulate 8:0" \
  "i_row4_pipe::240::$E --layout row --emulate 4:0" \
  "i_arxiv::240::$B --workload arxiv-synth" \
  "i_head::240::$B" \
  "i_suite::900::python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider --durations=0"
