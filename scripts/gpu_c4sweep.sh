#!/bin/bash
# C4 segment-length sweeps: the 1-GPU horizon (N = 65536, 24/8) and one
# 8-way slice (N = 8192), against the cost model's automatic choice (0)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python scripts/sweep_seglen.py 24 8 65536 0 8 16 24 32 48 64 96 > gpurun_out/sweep_c4_full.log 2>&1 || { tail -5 gpurun_out/sweep_c4_full.log; exit 1; }
timeout -k 10 300 python scripts/sweep_seglen.py 24 8 8192 0 2 4 6 8 12 16 24 32 > gpurun_out/sweep_c4_slice.log 2>&1 || { tail -5 gpurun_out/sweep_c4_slice.log; exit 1; }
timeout -k 10 300 python scripts/sweep_seglen.py 12 4 1024 0 2 4 8 16 32 64 > gpurun_out/sweep_c2.log 2>&1 || { tail -5 gpurun_out/sweep_c2.log; exit 1; }
cat gpurun_out/sweep_c4_full.log gpurun_out/sweep_c4_slice.log gpurun_out/sweep_c2.log | grep '^{'
