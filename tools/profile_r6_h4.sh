#!/bin/bash
# Round 6: entries in flight (APPNP_UW) on short-row launches of the bandwidth regime: arxiv-synth
# whole (14.8 entries a row; the rule gives 1), and the 8-rank row layout's local half again.
set -u
B="python bench.py --steps 10 --warmup 2 --cpu-iters 0"
T="env APPNP_TUNING=1"
tools/gpu_session.sh \
  "h4_arxiv_auto::240::$B --workload arxiv-synth" \
  "h4_arxiv_uw2::240::$T APPNP_UW=2 $B --workload arxiv-synth" \
  "h4_arxiv_auto_b::240::$B --workload arxiv-synth" \
  "h4_arxiv_uw2_b::240::$T APPNP_UW=2 $B --workload arxiv-synth" \
  "h4_powerlaw_auto::240::$B --workload products-powerlaw" \
  "h4_powerlaw_uw2::240::$T APPNP_UW=2 $B --workload products-powerlaw" \
  "h4_row8np_auto::240::$B --overlap --layout row --emulate 8:0 --pipeline off" \
  "h4_row8np_uw2::240::$T APPNP_UW=2 $B --overlap --layout row --emulate 8:0 --pipeline off"
