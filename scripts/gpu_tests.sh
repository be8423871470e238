#!/bin/bash
# GPU test run only (no bench): pytest -m gpu with per-test timeouts.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|Error|passed|failed" gpurun_out/pytest_gpu.log | tail -15
exit $rc
