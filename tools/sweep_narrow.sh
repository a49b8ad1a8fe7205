#!/bin/bash
export APPNP_TUNING=1  # round 6: the library reads tuning overrides only with APPNP_TUNING=1
# narrow (G-lane group per row) vs wide (wavefront per row) kernels on the per-rank slabs of
# column layouts (emulated ranks): APPNP_WIDE_ALL=1 forces the wide kernel
B="python bench.py --steps 5 --warmup 2 --cpu-iters 0"
for spec in "${@:-products-synth:col:4:0}"; do
  IFS=: read -r wl lay P r <<< "$spec"
  for env in "X=0" "APPNP_WIDE_ALL=1"; do
    out=$(env $env timeout -k 10 120 $B --workload $wl --layout $lay --emulate $P:$r 2>/dev/null) || exit $?
    echo "$spec $env $(echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('ms/iter %.4f lines/s %.1f G' % (r['avg_launch_ms'], r['gather_line_rate']['achieved_G_lines_s']))")"
  done
done
