#!/bin/bash
# A/B of variant libraries on the bench workload (no secondary configs):
#   VARIANTS="base nt" bash scripts/ab_variants.sh
# "base" = the in-tree libpdplqr.so, any other name X = pdp-lqr_amd/build/variants/libpdplqr_X.so.
# Interleaved runs (ABAB...) so clock drift hits every variant alike.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2 3; do
  for v in ${VARIANTS:-base nt}; do
    if [ "$v" = base ]; then unset PDPLQR_LIB; else export PDPLQR_LIB=$PWD/pdp-lqr_amd/build/variants/libpdplqr_$v.so; fi
    timeout -k 10 150 python bench.py --steps 10 --warmup 3 --no-cpu --no-secondary > gpurun_out/abv_$v.json 2>gpurun_out/abv_$v.err || { echo "$v failed"; tail -5 gpurun_out/abv_$v.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/abv_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e6,1), {k: round(x,3) for k,x in d['kernels_ms'].items()})"
  done
done
