set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u scripts/diag_status.py > gpurun_out/diag_status_fixed.json 2> gpurun_out/diag_status_fixed.err && head -c 1200 gpurun_out/diag_status_fixed.json && echo &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_serial.py > gpurun_out/pytest_r2a.log 2>&1; rc=$?; tail -30 gpurun_out/pytest_r2a.log; exit $rc
