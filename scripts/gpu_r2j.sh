#!/bin/bash
# Blocked-Cholesky 4x4 step on MFMA (PDPLQR_T4_MFMA): parity of every path that
# uses chol_blk4 / chol_blk4_aug, then an interleaved same-box A/B of the bench
# secondaries against the broadcast form (build/variants/libpdplqr_t4off.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_kkt.py tests/test_gpu_combine.py tests/test_gpu_parallel.py \
  tests/test_gpu_horizon.py tests/test_gpu_admm.py tests/test_gpu_psd.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
i=0
for v in new base new base; do
  i=$((i+1))
  if [ $v = base ]; then export PDPLQR_LIB=$PWD/pdp-lqr_amd/build/variants/libpdplqr_t4off.so; else unset PDPLQR_LIB; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > $O/ab_${v}_$i.json 2> $O/ab_${v}_$i.err || { echo "bench $v rc=$?"; tail -5 $O/ab_${v}_$i.err; exit 5; }
  python3 - $O/ab_${v}_$i.json $v <<'EOF'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
s = d['secondary']; c5 = s['C5_conic_kkt']
print(sys.argv[2], 'C5 kkt', round(c5['kkt']['ms_per_solve'], 3), 'admm_kkt/it', round(c5['admm_kkt']['ms_per_iteration'], 3),
      'C4', round(s['C4_horizon_sharded']['ms_per_solve'], 4), 'C2', round(s['C2_single_N1024_parallel']['parallel']['ms_per_solve'], 4),
      'hdl bwd', round(d['kernels_ms']['backward'], 3), 'ok', d['status_ok'], c5['kkt']['status_ok'], c5['kkt']['oracle_rel_err'],
      s['C4_horizon_sharded']['oracle_rel_err'])
EOF
done
