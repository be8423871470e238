#!/bin/bash
# C5 + ADMM kernel trace, LDS-conflict PMC of the value-form backward (padded vs unpadded)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python3 scripts/prof_c5.py > gpurun_out/prof_c5.log 2>&1 || { echo prof_c5 failed; tail -20 gpurun_out/prof_c5.log; exit 5; }
tail -1 gpurun_out/prof_c5.log
for v in base nopad; do
  if [ "$v" = base ]; then unset PDPLQR_LIB; else export PDPLQR_LIB=$PWD/pdp-lqr_amd/build/variants/libpdplqr_$v.so; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAVES --output-format csv -d gpurun_out/pmc/lds_$v -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-secondary > gpurun_out/pmc/lds_$v.log 2>&1 || { echo "pmc $v failed"; tail -5 gpurun_out/pmc/lds_$v.log; exit 6; }
done
echo pmc ok
