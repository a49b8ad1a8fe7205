#!/bin/bash
export APPNP_TUNING=1  # round 6: the library reads tuning overrides only with APPNP_TUNING=1
# Per-iteration time of products-synth against the feature width F (lines per gathered row).
# Usage: tools/sweep_features.sh [F ...]   (environment passed through, e.g. APPNP_SPLIT=0)
for f in ${@:-32 64 96 100 128}; do
  out=$(timeout -k 10 120 python bench.py --steps 5 --warmup 2 --cpu-iters 0 --features $f 2>/dev/null) || exit $?
  echo "F=$f $(echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms/iter %.4f' % d['roofline']['avg_launch_ms'])")"
done
