mkdir -p gpurun_out
for v in base sym1 sym2; do
  if [ "$v" = base ]; then unset PDPLQR_LIB; else export PDPLQR_LIB=$PWD/pdp-lqr_amd/build/variants/libpdplqr_$v.so; fi
  echo "== $v"
  timeout -k 10 240 python -u scripts/diag_status.py > gpurun_out/diag_status_$v.json 2> gpurun_out/diag_status_$v.err || { echo "$v failed rc=$?"; tail -20 gpurun_out/diag_status_$v.err; exit 1; }
  head -c 1500 gpurun_out/diag_status_$v.json; echo
done
