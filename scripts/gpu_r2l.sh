#!/bin/bash
# Packed triangular KKT tiles + raw-load prefetch in the twisted solve: KKT /
# ADMM parity, then per-kernel C5 traces of the new build and of the previous
# kkt.hip (build/variants/libpdplqr_kktold.so), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kkt.py tests/test_gpu_admm.py tests/test_gpu_configs.py tests/test_bench_contract.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
i=0
for v in new old new old; do
  i=$((i+1))
  if [ $v = old ]; then export PDPLQR_LIB=$PWD/pdp-lqr_amd/build/variants/libpdplqr_kktold.so; else unset PDPLQR_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$i -o run -- python3 scripts/prof_c5.py > $O/c5_${v}_$i.log 2>&1 || { echo "prof $v rc=$?"; tail -5 $O/c5_${v}_$i.log; exit 5; }
  python3 - $O/p$i $v <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
out = []
for r in csv.DictReader(open(f)):
    if 'kkt' in r['Name']:
        out.append((r['Name'].split('(')[0].replace('pdplqr::', ''), float(r['AverageNs']) / 1e3))
print(sys.argv[2], ' '.join(f'{n}={t:.0f}' for n, t in sorted(out)))
PY
done
