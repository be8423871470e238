set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_serial.py > gpurun_out/pytest_r2b.log 2>&1; rc=$?; tail -30 gpurun_out/pytest_r2b.log; exit $rc
