"""Summarise rocprofv3 --pmc passes (scripts/collect_pmc.sh) per kernel.

HBM bytes per launch = FETCH_SIZE * 1024 * 2 + WRITE_SIZE * 1024 for the
dominant kernel: MI355X_MICROARCH.md section HBM -- on gfx950 FETCH_SIZE
(= TCC_EA0_RDREQ x 64 B) reports half the bytes of a wide coalesced read, so
it is doubled; WRITE_SIZE is exact.  The raw counters are kept alongside so
the correction can be re-derived (RDREQ_32B shows the request size mix).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    root, tag = sys.argv[1], sys.argv[2]
    dom = sys.argv[3] if len(sys.argv) > 3 else "k_riccati_bwd"  # dominant-kernel substring
    per = defaultdict(lambda: defaultdict(list))
    rows = []
    for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    # the bench also runs secondary configs through the same kernels (smaller
    # grids): per kernel, only the dispatches of its largest grid (the bench
    # workload) are averaged
    gmax = defaultdict(int)
    for row in rows:
        gmax[row.get("Kernel_Name", "?")] = max(gmax[row.get("Kernel_Name", "?")], int(row.get("Grid_Size", 0)))
    for row in rows:
        k = row.get("Kernel_Name", "?")
        if int(row.get("Grid_Size", 0)) == gmax[k]:
            per[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {"workload": tag, "kernels": {}}
    # PMC_SOLVES: the profiled run made that many solves of the workload and
    # nothing else through these kernels -- bench.pmc_traffic then counts each
    # kernel dispatches / solves times per solve (C4: the scan rounds)
    if os.environ.get("PMC_SOLVES"):
        out["solves"] = int(os.environ["PMC_SOLVES"])
    for k, d in per.items():
        short = k.split("(")[0].replace("void ", "")
        if "pdplqr" not in short:
            continue
        out["kernels"][short] = {c: sum(v) / len(v) for c, v in d.items()}
        # dispatches of the kernel at that grid: each counter is collected by
        # one pass of scripts/collect_pmc.sh, which sees every dispatch
        out["kernels"][short]["dispatches"] = max(len(v) for v in d.values())
    # dominant kernel of the bench step: the value-form backward when present
    names = sorted(out["kernels"], key=lambda k: ("bwd_schur" not in k, dom not in k))
    bwd = [out["kernels"][k] for k in names if dom in k]
    if bwd:
        out["dominant_kernel"] = [k for k in names if dom in k][0]
    if bwd and "FETCH_SIZE" in bwd[0] and "WRITE_SIZE" in bwd[0]:
        b = bwd[0]
        out["bytes_per_launch"] = b["FETCH_SIZE"] * 1024 * 2 + b["WRITE_SIZE"] * 1024
        out["correction"] = "FETCH_SIZE x2 (gfx950 wide-read undercount), WRITE_SIZE x1; units KB"
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
