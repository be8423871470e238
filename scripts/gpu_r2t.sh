#!/bin/bash
# Gain record computed from one T^T product per lane (y = W row or lu'):
# serial parity, then an interleaved same-box A/B against the previous gain
# kernel (build/variants/libpdplqr_gain0.so) and the L-form record.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_serial.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
i=0
for v in new old L new old L new old L; do
  i=$((i+1))
  unset PDPLQR_REC_L PDPLQR_LIB
  if [ $v = L ]; then export PDPLQR_REC_L=1; fi
  if [ $v = old ]; then export PDPLQR_LIB=$PWD/pdp-lqr_amd/build/variants/libpdplqr_gain0.so; fi
  timeout -k 10 200 python bench.py --no-cpu --no-secondary > $O/ab_${v}_$i.json 2> $O/ab_${v}_$i.err || { echo "bench $v rc=$?"; tail -5 $O/ab_${v}_$i.err; exit 5; }
  python3 - $O/ab_${v}_$i.json $v <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
pc = d['roofline'].get('pattern_ceiling', {})
print(sys.argv[2], 'ms/step', round(d['ms_per_step'], 4), 'bwd', round(d['kernels_ms']['backward'], 4),
      'fwd', round(d['kernels_ms']['forward'], 4), 'status_ok', d['status_ok'],
      'pattern bwd/fwd', round(pc.get('backward_ms', 0), 3), round(pc.get('forward_ms', 0), 3))
PY
done
