#!/bin/bash
# rocprofv3 PMC passes (one counter group per pass; never combined with trace domains)
# for the bench workload; summarised into profiles/<tag>_pmc.json by scripts/pmc_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --no-cpu ${BENCH_ARGS:-}"
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" "SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 bench.py $ARGS > gpurun_out/pmc/p$i.log 2>&1 || { echo "pmc pass $i ($ctr) failed rc=$?"; tail -5 gpurun_out/pmc/p$i.log; }
done
python3 scripts/pmc_summary.py gpurun_out/pmc "${TAG:-N1024_n12_m4_b4096_kf0}" > gpurun_out/pmc/summary.json && cat gpurun_out/pmc/summary.json
