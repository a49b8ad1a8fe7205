#!/bin/bash
# Remainder pass (appnp_blocks.hip): pacing lead x source-block size on products-synth.
# Usage (GPU box): tools/sweep_rem.sh ; reads avg_launch_ms (per iteration) from each bench line.
B="python bench.py --steps 5 --warmup 2 --cpu-iters 0"
args=()
for sb in 16384 32768 65536; do
  for lead in 0 1 2 4; do
    args+=("rem_sb${sb}_lead${lead}::120::APPNP_SB_ROWS=$sb APPNP_REM_LEAD=$lead $B")
  done
done
tools/gpu_session.sh "${args[@]}"
