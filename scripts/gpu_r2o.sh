#!/bin/bash
# Bank-spread E reads in the streamed nofact kernels: parity (serial nofact,
# ADMM), then interleaved A/B against the previous kernels_nofact.hip
# (build/variants/libpdplqr_nfold.so): headline factor-reuse and C5 ADMM.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_serial.py tests/test_gpu_admm.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for v in new old new old; do
  if [ $v = old ]; then export PDPLQR_LIB=$PWD/pdp-lqr_amd/build/variants/libpdplqr_nfold.so; else unset PDPLQR_LIB; fi
  timeout -k 10 200 python scripts/prof_nofact.py > $O/nf_$v.log 2>&1 || { echo "nofact $v failed"; tail -3 $O/nf_$v.log; exit 5; }
  timeout -k 10 200 python scripts/prof_c5.py > $O/c5_$v.log 2>&1 || { echo "c5 $v failed"; tail -3 $O/c5_$v.log; exit 5; }
  python3 - $O $v <<'PY'
import json, sys
o, v = sys.argv[1], sys.argv[2]
nf = json.loads([l for l in open(f'{o}/nf_{v}.log') if l.startswith('{')][-1])
c5 = json.loads([l for l in open(f'{o}/c5_{v}.log') if l.startswith('{')][-1])
print(v, 'nofact', round(nf['kernels_ms']['backward_without_factorization'], 3), 'iter', round(nf['ms_per_iteration'], 3),
      'admm_ric', round(c5['admm_riccati']['ms_per_iteration'], 4), nf['oracle_rel_err'])
PY
done
