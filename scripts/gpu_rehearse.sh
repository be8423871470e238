#!/bin/bash
# Multi-rank rehearsal of bench.py on ONE GPU (gloo backend for the clock
# reduction and the C4 all-gather): the driver's N = 2 / 8 launch, with a
# small per-rank batch so 8 ranks fit one card.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PDPLQR_BENCH_BACKEND=gloo
for R in 2 8; do
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $R --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus $R --steps 3 --warmup 1 --batch 256 --c4-N 65536 > gpurun_out/rehearse_$R.log 2>&1 || { echo "R=$R failed"; tail -20 gpurun_out/rehearse_$R.log; exit 1; }
  grep '^{' gpurun_out/rehearse_$R.log | tail -1 | cut -c1-300
done
