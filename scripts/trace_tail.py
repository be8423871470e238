"""Print the kernel timeline of the last solve in a rocprofv3 kernel trace:
python scripts/trace_tail.py <run_kernel_trace.csv> [count]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
cnt = int(sys.argv[2]) if len(sys.argv) > 2 else 30
last = rows[-cnt:]
t0 = int(last[0]["Start_Timestamp"])
for r in last:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1000:9.1f} {(e - s) / 1000:8.1f}  {r['Kernel_Name'][:60]}")
