set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3sweep; mkdir -p $O
for L in 0 10 12 14 20 24; do
  echo "L=$L $(PDPLQR_SEGMENT_LEN=$L timeout -k 10 120 python -u scripts/prof_shards.py 65536 8 | grep -o '"max_rank_ms": [0-9.]*')" >> $O/shards.log
done
timeout -k 10 200 python -u scripts/sweep_seglen.py 24 8 65536 0 48 65 80 96 >> $O/c4_1wave.log
PDPLQR_MW_ALWAYS=1 timeout -k 10 200 python -u scripts/sweep_seglen.py 24 8 65536 0 48 65 96 130 >> $O/c4_mw.log
