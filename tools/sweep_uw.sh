#!/bin/bash
export APPNP_TUNING=1  # round 6: the library reads tuning overrides only with APPNP_TUNING=1
# Latency-regime shape overrides on the small workloads: entries in flight per sub-group of
# the wide kernel (APPNP_UW), wide/narrow (APPNP_WIDE), elements per lane (APPNP_VEC).
# Usage: tools/sweep_uw.sh "workload|ENV=.. ENV=..|..." ...
for spec in "${@:-pubmed-synth|X=0|APPNP_VEC=2|APPNP_VEC=4}"; do
  IFS='|' read -r -a parts <<< "$spec"
  wl=${parts[0]}
  for env in "${parts[@]:1}"; do
    out=$(env $env timeout -k 10 120 python bench.py --steps 20 --warmup 3 --cpu-iters 0 --workload $wl 2>/dev/null)
    rc=$?
    if [ $rc -ne 0 ]; then echo "$wl [$env] rc=$rc"; [ $rc -ge 124 ] && exit $rc; continue; fi
    echo "$wl [$env] $(echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('per-iter %.2f us' % (r['avg_launch_ms']*1e3))")"
  done
done
