#!/bin/bash
# Round 4, final tree: the driver's bench command under rocprofv3 (kernel stats of exactly the
# command whose line is judged), the other BASELINE workloads, and the timing-state study: six
# separate bench processes, each printing its iteration time beside the line-rate probe taken
# right before its timed region (roofline.box_line_rate).  Logs under gpurun_out/.
set -u
B="python bench.py --steps 10 --warmup 2 --cpu-iters 0"
specs=("driver_cmd_prof::400::rocprofv3 --kernel-trace --stats -d gpurun_out/driver_prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5")
for i in 1 2 3 4 5 6; do specs+=("state_$i::200::$B"); done
for w in pubmed-synth ms-academic-synth arxiv-synth cora-ml-real; do
  specs+=("w_$w::200::python bench.py --steps 20 --warmup 3 --cpu-iters 0 --workload $w")
done
tools/gpu_session.sh "${specs[@]}"
