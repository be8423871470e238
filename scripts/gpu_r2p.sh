#!/bin/bash
# ADMM update with hoisted row loads (k_admm_update<16, ., ., 4>): ADMM parity,
# then interleaved A/B of the C5 ADMM lines against the previous admm.hip
# (build/variants/libpdplqr_admmold.so) with a kernel trace of each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_admm.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
i=0
for v in new old new old; do
  i=$((i+1))
  if [ $v = old ]; then export PDPLQR_LIB=$PWD/pdp-lqr_amd/build/variants/libpdplqr_admmold.so; else unset PDPLQR_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$i -o run -- python3 scripts/prof_c5.py > $O/c5_${v}_$i.log 2>&1 || { echo "prof $v rc=$?"; exit 5; }
  python3 - $O/p$i $O/c5_${v}_$i.log $v <<'PY'
import csv, glob, json, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
k = {r['Name'].split('(')[0].replace('void pdplqr::', '').replace('pdplqr::', ''): round(float(r['AverageNs']) / 1e3)
     for r in csv.DictReader(open(f)) if 'admm' in r['Name']}
d = json.loads([l for l in open(sys.argv[2]) if l.startswith('{')][-1])
print(sys.argv[3], 'admm_kkt', round(d['admm_kkt']['ms_per_iteration'], 3), 'admm_ric', round(d['admm_riccati']['ms_per_iteration'], 3), k)
PY
done
