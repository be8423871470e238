#!/bin/bash
# LDS-DMA ring depth 6 (build/variants/libpdplqr_depth6.so) for k_nofact_dma,
# k_nofact_admm_dma and k_rollout_dma against the default 4: parity of the
# streamed kernels on the variant, then interleaved same-box bench A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2m
mkdir -p $O
export TMPDIR=/tmp
V=$PWD/pdp-lqr_amd/build/variants/libpdplqr_depth6.so
PDPLQR_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_serial.py tests/test_gpu_admm.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
i=0
for v in d4 d6 d4 d6; do
  i=$((i+1))
  if [ $v = d6 ]; then export PDPLQR_LIB=$V; else unset PDPLQR_LIB; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > $O/ab_${v}_$i.json 2> $O/ab_${v}_$i.err || { echo "bench $v rc=$?"; tail -5 $O/ab_${v}_$i.err; exit 5; }
  python3 - $O/ab_${v}_$i.json $v <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
s = d['secondary']; c5 = s['C5_conic_kkt']; fr = s['factor_reuse']
print(sys.argv[2], 'hdl bwd/fwd', round(d['kernels_ms']['backward'], 3), round(d['kernels_ms']['forward'], 3),
      'nofact/fwd', round(fr['kernels_ms']['backward_without_factorization'], 3), round(fr['kernels_ms']['forward'], 3),
      'C5 ric', round(c5['riccati']['ms_per_solve'], 3), 'admm_ric/it', round(c5['admm_riccati']['ms_per_iteration'], 3),
      'C3', round(s['C3_batched_N256']['ms_per_solve'], 3), 'ok', d['status_ok'], fr['oracle_rel_err'], c5['riccati']['oracle_rel_err'])
PY
done
