"""Sum rocprofv3 --pmc counter values per kernel (and count dispatches):
python scripts/pmc_kernels.py <dir-with-counter_collection.csv> [kernel-substring]"""
import collections
import csv
import glob
import sys

files = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
sub = sys.argv[2] if len(sys.argv) > 2 else ""
acc = collections.defaultdict(float)
disp = collections.defaultdict(set)
for f in files:
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if sub not in k:
            continue
        acc[(k[:60], r["Counter_Name"])] += float(r["Counter_Value"])
        disp[k[:60]].add(r["Dispatch_Id"])
for (k, cn), v in sorted(acc.items()):
    print(f"{k:60s} {cn:28s} {v:16.0f}  per-dispatch {v / max(1, len(disp[k])):14.0f}")
