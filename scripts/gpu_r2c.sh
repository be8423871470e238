#!/bin/bash
# round-2 session: value-form backward parity + LDS layout A/B + bench with the ADMM line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_serial.py tests/test_gpu_admm.py > gpurun_out/pytest_r2c.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_r2c.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="base nopad" bash scripts/ab_variants.sh || exit 5
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench.log; exit 4; }
tail -1 gpurun_out/bench.log
