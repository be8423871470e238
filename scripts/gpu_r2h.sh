#!/bin/bash
# KKT register-tile model setup: parity, then the C5 kernel trace and the bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kkt.py tests/test_gpu_admm.py tests/test_gpu_configs.py::test_c5_conic_kkt_full_size > gpurun_out/pytest_r2h.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_r2h.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/pytest_r2h.log | head -20; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python3 scripts/prof_c5.py > gpurun_out/prof_c5.log 2>&1 || { echo prof_c5 failed; tail -20 gpurun_out/prof_c5.log; exit 5; }
grep '^{' gpurun_out/prof_c5.log | tail -1 | cut -c1-300
