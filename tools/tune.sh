#!/bin/bash
export APPNP_TUNING=1  # round 6: the library reads tuning overrides only with APPNP_TUNING=1
# grid-size sweep of the SpMM launch on products-synth (APPNP_MAX_BLOCKS)
for b in 1024 2048 4096 8192 32768 1000000; do
  echo "max_blocks=$b"
  APPNP_MAX_BLOCKS=$b timeout -k 10 120 python bench.py --steps 5 --warmup 2 --cpu-iters 0 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('  ms/iter %.3f  lines/s %.1f G' % (r['avg_launch_ms'], r['gather_line_rate']['achieved_G_lines_s']))" || exit $?
done
