#!/bin/bash
export APPNP_TUNING=1  # round 6: the library reads tuning overrides only with APPNP_TUNING=1
# Round 5: entries in flight per sub-group of the main SpMM (APPNP_UW), read from
# roofline.kernel_ms (main = the SpMM launches of one untimed propagation).
set -u
B="python bench.py --cpu-iters 0 --steps 10"
tools/gpu_session.sh \
 "uw2::200::APPNP_UW=2 $B" \
 "uw4::200::APPNP_UW=4 $B" \
 "uw8::200::APPNP_UW=8 $B" \
 "uw1::200::APPNP_UW=1 $B" \
 "uw2b::200::APPNP_UW=2 $B"
