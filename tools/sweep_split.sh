#!/bin/bash
export APPNP_TUNING=1  # round 6: the library reads tuning overrides only with APPNP_TUNING=1
# Split rows (appnp_blocks.hip) on products-synth: per-iteration time with the path off
# (APPNP_SPLIT=0) and with the remainder pass's source block size (APPNP_SB_ROWS source rows
# per block) varied.
# Usage: tools/sweep_split.sh ["ENV=.. ENV=.." ...]
B="python bench.py --steps 5 --warmup 2 --cpu-iters 0"
for env in "${@:-APPNP_SPLIT=0|X=0|APPNP_SB_ROWS=98304|APPNP_SB_ROWS=163840|APPNP_SB_ROWS=196608}"; do
  IFS='|' read -r -a envs <<< "$env"
  for e in "${envs[@]}"; do
    out=$(env $e timeout -k 10 120 $B 2>/dev/null) || exit $?
    echo "[$e] $(echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('ms/iter %.4f' % r['avg_launch_ms'])")"
  done
done
