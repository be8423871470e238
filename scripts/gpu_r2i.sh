#!/bin/bash
# Factor-reuse (backward_without_factorization) pass at the headline config:
# kernel trace + PMC passes of k_nofact_dma, then the full bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2i
mkdir -p $O/pmc
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/prof_nofact.py > $O/nofact.log 2>&1 || { echo "nofact rc=$?"; tail -5 $O/nofact.log; exit 2; }
tail -1 $O/nofact.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 scripts/prof_nofact.py > $O/prof.log 2>&1 || { echo "prof rc=$?"; tail -5 $O/prof.log; exit 3; }
echo "prof ok"
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d $O/pmc/p$i -o run -- python3 scripts/prof_nofact.py > $O/pmc/p$i.log 2>&1 || { echo "pmc pass $i ($ctr) rc=$?"; tail -5 $O/pmc/p$i.log; exit 4; }
done
python3 scripts/pmc_summary.py $O/pmc nofact_N1024_n12_m4_b4096 k_nofact_dma > $O/nofact_pmc.json && grep -A3 bytes_per_launch $O/nofact_pmc.json
timeout -k 10 420 python bench.py --steps 10 --warmup 2 > $O/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench.log; exit 5; }
tail -c 600 $O/bench.log
