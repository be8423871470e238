# A/B of variant libraries on one box: bash scripts/ab_multi.sh name1 name2 ...
# name "new" = the in-tree library, else pdp-lqr_amd/build/variants/libpdplqr_<name>.so
set -e
mkdir -p gpurun_out
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = new ]; then unset PDPLQR_LIB; else export PDPLQR_LIB=$PWD/pdp-lqr_amd/build/variants/libpdplqr_$v.so; fi
    timeout -k 10 150 python bench.py --steps 10 --warmup 3 --no-cpu --no-secondary > gpurun_out/ab_$v.json 2>gpurun_out/ab_$v.err
    python -c "import json; d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[0]); print('$v', round(d['value']/1e6,1), d['kernels_ms'])"
  done
done
