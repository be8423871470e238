#!/bin/bash
# Serial solver for 32 < n + m <= 64 (kernels_big.hip): the new parity tests,
# then the serial / ADMM suites that share the touched dispatch code.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2r
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_big.py -x -v --timeout 120 --timeout-method thread > $O/big.log 2>&1
rc=$?; echo "big rc=$rc"; tail -25 $O/big.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_serial.py tests/test_gpu_admm.py -x -q --timeout 200 --timeout-method thread > $O/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 $O/suite.log
exit $rc
