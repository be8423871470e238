set -u
# Parity tests of the parallel paths, then C4 timings (N = 65536 and the 8-rank slice 8192) of the
# in-tree library against pdp-lqr_amd/build/variants/libpdplqr_old.so, interleaved.
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_combine.py tests/test_gpu_parallel.py tests/test_gpu_horizon.py > gpurun_out/blk.log 2>&1; rc=$?; tail -3 gpurun_out/blk.log; [ $rc -eq 0 ] || exit $rc
for v in new old new old; do
  if [ $v = old ]; then export PDPLQR_LIB=$PWD/pdp-lqr_amd/build/variants/libpdplqr_old.so; else unset PDPLQR_LIB; fi
  echo "$v $(timeout -k 10 120 python scripts/prof_c4.py 65536 8192 2>/dev/null | python3 -c 'import json,sys; print([round(json.loads(l)["ms_per_solve"],3) for l in sys.stdin if l.startswith("{")])')" || exit 1
done
