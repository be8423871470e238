#!/bin/bash
# Two-wave fused ADMM / nofact kernel (k_nofact_admm_dma2): ADMM parity, then an
# interleaved same-box A/B of the C5 ADMM iterations against the one-wave kernel
# (PDPLQR_ADMM_ONE_WAVE=1, same library).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_admm.py tests/test_gpu_serial.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
i=0
for v in new base new base; do
  i=$((i+1))
  if [ $v = base ]; then export PDPLQR_ADMM_ONE_WAVE=1; else unset PDPLQR_ADMM_ONE_WAVE; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > $O/ab_${v}_$i.json 2> $O/ab_${v}_$i.err || { echo "bench $v rc=$?"; tail -5 $O/ab_${v}_$i.err; exit 5; }
  python3 - $O/ab_${v}_$i.json $v <<'EOF'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
c5 = d['secondary']['C5_conic_kkt']
print(sys.argv[2], 'admm_riccati/it', round(c5['admm_riccati']['ms_per_iteration'], 4), 'admm_kkt/it',
      round(c5['admm_kkt']['ms_per_iteration'], 4), {k: v for k, v in c5['admm_riccati'].items() if k != 'ms_per_iteration'})
EOF
done
