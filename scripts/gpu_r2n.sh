#!/bin/bash
# Radix-4 segment scan (k_seg_scan4, T = 1): parity of every parallel path,
# then C2 (N = 1024 single problem) same-box A/B against radix 2
# (PDPLQR_NO_SCAN4=1), interleaved, plus a kernel trace of each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2n
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parallel.py tests/test_gpu_psd.py tests/test_gpu_horizon.py tests/test_gpu_configs.py tests/test_gpu_combine.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for v in r4 r2 r4 r2 r4 r2; do
  if [ $v = r2 ]; then export PDPLQR_NO_SCAN4=1; else unset PDPLQR_NO_SCAN4; fi
  timeout -k 10 120 python scripts/prof_c2.py > $O/c2_$v.log 2>&1 || { echo "c2 $v failed"; tail -3 $O/c2_$v.log; exit 5; }
  python3 -c "import json; d=json.loads(open('$O/c2_$v.log').read().strip().splitlines()[-1]); print('$v', round(d['parallel']['ms_per_solve'], 4), d['parallel']['status_ok'])"
done
unset PDPLQR_NO_SCAN4
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tr4 -o run -- python3 scripts/prof_c2.py > $O/tr4.log 2>&1 || exit 6
echo traced
