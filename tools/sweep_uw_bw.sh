#!/bin/bash
export APPNP_TUNING=1  # round 6: the library reads tuning overrides only with APPNP_TUNING=1
# Entries in flight per sub-group of the wide kernel (APPNP_UW) in the bandwidth regime.
# Usage: tools/sweep_uw_bw.sh "workload[:F[:dtype]]" ...
for spec in "${@:-products-synth arxiv-synth}"; do
  IFS=: read -r wl f dt <<< "$spec"
  extra=""
  [ -n "$f" ] && extra="$extra --features $f"
  [ -n "$dt" ] && extra="$extra --dtype $dt"
  for uw in 1 2 4; do
    out=$(APPNP_UW=$uw timeout -k 10 120 python bench.py --steps 5 --warmup 2 --cpu-iters 0 --workload $wl $extra 2>/dev/null) || exit $?
    echo "$spec UW=$uw $(echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms/iter %.4f' % d['roofline']['avg_launch_ms'])")"
  done
done
