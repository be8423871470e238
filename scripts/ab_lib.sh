set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_gain.log 2>&1
tail -3 gpurun_out/pt_gain.log
for v in base new base new; do
  if [ $v = base ]; then export PDPLQR_LIB=$PWD/pdp-lqr_amd/build/variants/libpdplqr_base.so; else unset PDPLQR_LIB; fi
  timeout -k 10 150 python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/ab_$v.json 2>gpurun_out/ab_$v.err
  echo $v; python -c "import json,sys; d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[0]); print(d['value'], d['ms_per_step'], d.get('kernels', d.get('phases')))"
done
