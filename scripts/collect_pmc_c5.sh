#!/bin/bash
# C5 (conic N = 512, nc = 4, batch 1024): rocprofv3 kernel trace + PMC passes
# (one counter group per pass, never combined with trace domains) of
# scripts/prof_c5.py; summarised per kernel by scripts/pmc_summary.py with the
# KKT factor as the dominant kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/pmc_c5
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 scripts/prof_c5.py > $O/trace.log 2>&1 || { echo "trace failed rc=$?"; tail -5 $O/trace.log; exit 4; }
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" "SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d $O/p$i -o run -- python3 scripts/prof_c5.py > $O/p$i.log 2>&1 || { echo "pmc pass $i ($ctr) failed rc=$?"; tail -5 $O/p$i.log; exit 5; }
done
python3 scripts/pmc_summary.py $O N512_n12_m4_nc4_b1024 k_kkt_factor > $O/summary.json && head -c 600 $O/summary.json
