#!/bin/bash
# A/B of remainder-pass variants on products-synth, one rocprofv3 kernel-stats run per variant.
# Usage: tools/rem_ab.sh "<tag>=<env assignments>" ...
#   e.g. tools/rem_ab.sh "stripe1=APPNP_REM_STRIPE=1" "stripe0=APPNP_REM_STRIPE=0"
# Results: gpurun_out/remab/<tag>/run_kernel_stats.csv
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B="python bench.py --steps 3 --warmup 1 --cpu-iters 0 ${BENCH_ARGS:-}"
specs=()
for v in "$@"; do
  t="${v%%=*}"; e="${v#*=}"
  specs+=("$t::240::$e rocprofv3 --kernel-trace --stats -d gpurun_out/remab/$t -o run --output-format csv -- $B")
done
tools/gpu_session.sh "${specs[@]}"
