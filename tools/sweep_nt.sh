#!/bin/bash
export APPNP_TUNING=1  # round 6: the library reads tuning overrides only with APPNP_TUNING=1
# Cache policy of the SpMM streams (StepArgs::nt, APPNP_NT bit mask: 1 col/val, 2 H, 4 Zout
# non-temporal) on the bench workloads.  Usage: tools/sweep_nt.sh [workload[:dtype]] ...
B="python bench.py --steps 5 --warmup 2 --cpu-iters 0"
for spec in "${@:-products-synth}"; do
  IFS=: read -r wl dt <<< "$spec"
  extra=""
  [ -n "$dt" ] && extra="--dtype $dt"
  for nt in 0 1 2 4 7 0; do
    out=$(APPNP_NT=$nt timeout -k 10 120 $B --workload $wl $extra 2>/dev/null) || exit $?
    echo "$spec nt=$nt $(echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('ms/iter %.4f lines/s %.1f G' % (r['avg_launch_ms'], r['gather_line_rate']['achieved_G_lines_s']))")"
  done
done
