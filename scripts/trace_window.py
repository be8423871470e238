"""Kernel timeline (start offset, duration, gap to the previous kernel) of a
rocprofv3 kernel trace, from the N-th last launch of a kernel whose name
contains PATTERN: python scripts/trace_window.py run_kernel_trace.csv PATTERN [count] [nth_last]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
pat = sys.argv[2]
cnt = int(sys.argv[3]) if len(sys.argv) > 3 else 30
nth = int(sys.argv[4]) if len(sys.argv) > 4 else 1
hits = [i for i, r in enumerate(rows) if pat in r["Kernel_Name"]]
i0 = hits[-nth]
win = rows[i0:i0 + cnt]
t0 = int(win[0]["Start_Timestamp"])
prev = None
busy = 0
for r in win:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1000 if prev is not None else 0.0
    busy += e - s
    print(f"{(s - t0) / 1000:9.1f} dur {(e - s) / 1000:8.1f} gap {gap:6.1f}  {r['Kernel_Name'][:80]}")
    prev = e
print(f"span {(prev - t0) / 1000:.1f} us, kernels busy {busy / 1000:.1f} us")
