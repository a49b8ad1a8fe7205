#!/bin/bash
# per-iteration time of the latency-regime workloads (small graphs, one launch per iteration)
B="python bench.py --steps 20 --warmup 3 --cpu-iters 0"
for wl in ${@:-cora-ml-real citeseer-real pubmed-synth ms-academic-synth cora-ml}; do
  out=$(timeout -k 10 120 $B --workload $wl 2>/dev/null) || exit $?
  echo "$wl $(echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('per-iter %.2f us  ms/step %.4f' % (r['avg_launch_ms']*1e3, d['ms_per_step']))")"
done
