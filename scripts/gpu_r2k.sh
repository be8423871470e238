#!/bin/bash
# MFMA VGPR form (-mllvm -amdgpu-mfma-vgpr-form): GPU suite on the variant, then
# an interleaved same-box A/B against the default build (vgpr = the variant, dflt = the default build),
# and the headline backward with its u-block panel on MFMA (st4, PDPLQR_SCHUR_T4=1).
# 
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2k
mkdir -p $O
export TMPDIR=/tmp
PDPLQR_LIB=$PWD/pdp-lqr_amd/build/variants/libpdplqr_vgprform.so timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
PDPLQR_LIB=$PWD/pdp-lqr_amd/build/variants/libpdplqr_schurt4.so timeout -k 10 400 python -u -m pytest tests/test_gpu_serial.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_st4.log 2>&1
rc=$?; echo "pytest st4 rc=$rc"; tail -2 $O/pytest_st4.log
[ $rc -eq 0 ] || exit $rc
i=0
for v in dflt vgpr st4 dflt vgpr st4; do
  i=$((i+1))
  case $v in
    vgpr) export PDPLQR_LIB=$PWD/pdp-lqr_amd/build/variants/libpdplqr_vgprform.so ;;
    st4) export PDPLQR_LIB=$PWD/pdp-lqr_amd/build/variants/libpdplqr_schurt4.so ;;
    *) unset PDPLQR_LIB ;;
  esac
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > $O/ab_${v}_$i.json 2> $O/ab_${v}_$i.err || { echo "bench $v rc=$?"; tail -5 $O/ab_${v}_$i.err; exit 5; }
  python3 - $O/ab_${v}_$i.json $v <<'EOF'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
s = d['secondary']; c5 = s['C5_conic_kkt']
print(sys.argv[2], 'C5 kkt', round(c5['kkt']['ms_per_solve'], 3), 'admm_kkt/it', round(c5['admm_kkt']['ms_per_iteration'], 3),
      'C4', round(s['C4_horizon_sharded']['ms_per_solve'], 4), 'C2', round(s['C2_single_N1024_parallel']['parallel']['ms_per_solve'], 4),
      'hdl bwd', round(d['kernels_ms']['backward'], 3), 'fwd', round(d['kernels_ms']['forward'], 3), 'C3', round(s['C3_batched_N256']['ms_per_solve'], 3), 'ok', d['status_ok'], c5['kkt']['status_ok'], c5['kkt']['oracle_rel_err'],
      s['C4_horizon_sharded']['oracle_rel_err'])
EOF
done
