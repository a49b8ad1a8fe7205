#!/bin/bash
# Round 5: the north_star's 8-rank products-synth row partition on the one GPU (tests/dist_worker.py
# against rank 0's float64 oracle; tests/dist_capi_worker.py, the library's own loop, against the
# single-GPU propagation), each rank's result line kept.  gpurun: bash tools/run_8rank.sh
set -o pipefail
out=gpurun_out/r5_8rank
mkdir -p $out
port() { python -c 'import socket; s=socket.socket(); s.bind(("127.0.0.1",0)); print(s.getsockname()[1])'; }
export PPNP_DIST_BACKEND=gloo PYTHONPATH=$PWD OMP_NUM_THREADS=2
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=8 --master-addr=127.0.0.1 \
  --master-port=$(port) tests/dist_worker.py --layout row --workload products-synth --oracle-torch --oracle-rank0 \
  --expect-split 4 --overlap > $out/python_row8.txt 2>&1 &&
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=8 --master-addr=127.0.0.1 \
  --master-port=$(port) tests/dist_capi_worker.py --workload products-synth --split --overlap \
  > $out/native_row8.txt 2>&1
