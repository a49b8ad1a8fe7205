set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for e in ${EXPS:-0 1 2 3}; do
  if [ $e = 0 ]; then unset PPNP_AMD_LIB; else export PPNP_AMD_LIB=$GRAFT_REPO_ROOT/tools/bin/libexp$e.so; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/remexp/e$e -o run --output-format csv -- python bench.py --steps 3 --warmup 1 ${CPUARG---cpu-iters 0} > gpurun_out/remexp/e$e.log 2>&1 || { echo "exp $e failed rc=$?"; exit 1; }
  find gpurun_out/remexp/e$e -name "*kernel_trace*" -delete; find gpurun_out/remexp/e$e -name "*.db" -delete
  echo "exp $e done"
done
