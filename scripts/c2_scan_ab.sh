#!/bin/bash
# C2 (one N = 1024 12/4 problem, PARALLEL solver): suffix-scan round forms A/B on one box.
# default: k_seg_scan4 (two Hillis-Steele rounds per launch); PDPLQR_NO_SCAN4=1 PDPLQR_SCAN_SK=1: Sklansky
# rounds; PDPLQR_NO_SCAN4=1: radix-2 Hillis-Steele.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/c2ab; mkdir -p $O
for v in "" "PDPLQR_NO_SCAN4=1 PDPLQR_SCAN_SK=1" "PDPLQR_NO_SCAN4=1" ""; do
  echo "[$v] $(env $v timeout -k 10 120 python -u scripts/sweep_seglen.py 12 4 1024 0 | grep -o '"ms": [0-9.]*' | head -1)" >> $O/c2.log
done
