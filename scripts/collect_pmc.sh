#!/bin/bash
# rocprofv3 PMC passes of one workload (one counter group per pass, never
# combined with trace domains; MI355X_MICROARCH.md slot limits), summarised per
# kernel by scripts/pmc_summary.py into $OUT/summary.json.
#   TAG=<workload tag> DOM=<dominant kernel substring> OUT=gpurun_out/<dir> \
#     scripts/collect_pmc.sh python3 <script> [args...]
# default: the headline bench workload.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/pmc}
TAG=${TAG:-N1024_n12_m4_b4096_kf0}
DOM=${DOM:-k_riccati_bwd}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ $# -eq 0 ]; then set -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-secondary; fi
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" "SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/p$i" -o run -- "$@" > "$OUT/p$i.log" 2>&1 || { echo "pmc pass $i ($ctr) failed rc=$?"; tail -5 "$OUT/p$i.log"; exit 5; }
done
python3 scripts/pmc_summary.py "$OUT" "$TAG" "$DOM" > "$OUT/summary.json" && head -c 400 "$OUT/summary.json"
