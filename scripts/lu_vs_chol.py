"""Condensed combine forms on the latency-bound horizon paths (diagnostic):
C2 (one N = 1024, 12/4 problem) and one rank of the 8-rank C4 split
(N = 8192 slice, 24/8) with CondensedSystemSolverType CHOLESKY and LU, the
solver on the caller's stream, median of reps; prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pdp-lqr_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from pdplqr import BatchedLQRSolver  # noqa: E402


def time_solve(n, m, N, condensed, reps=20):
    dev = torch.device("cuda", 0)
    E, c, H, h, x0 = bench.gen_batch_device(n, m, N, 1, seed=77, device=dev)
    ws0 = torch.zeros(1, N * (n + m) + n, dtype=torch.float64, device=dev)
    out = torch.empty_like(ws0)
    bs = BatchedLQRSolver(n, m, N, 1, solver="parallel", num_segments=8, keep_factors=True, condensed=condensed,
                          device=0)
    bs.set_model(E, c, H, h)
    bs.update_problem_data(ws0, sigma=1e-6)
    bs.synchronize()
    side = torch.cuda.Stream(device=dev)
    bs.handle.set_stream(side.cuda_stream)
    ts = []
    with torch.cuda.stream(side):
        for i in range(reps + 3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(side)
            bs.backward()
            bs.forward(x0, out)
            e1.record(side)
            torch.cuda.synchronize()
            if i >= 3:
                ts.append(e0.elapsed_time(e1))
    ok = bool(np.all(bs.status() == 0))
    bs.close()
    return round(float(np.median(ts)), 4), ok, out.cpu().numpy()


def main():
    torch.cuda.set_device(0)
    res = {}
    for tag, (n, m, N) in {"C2_12x4_N1024": (12, 4, 1024), "C4slice_24x8_N8192": (24, 8, 8192)}.items():
        r = {}
        outs = {}
        for cond in ("CHOLESKY", "LU"):
            ms, ok, o = time_solve(n, m, N, cond)
            r[cond] = {"ms": ms, "ok": ok}
            outs[cond] = o
        r["rel_diff"] = float(np.linalg.norm(outs["LU"] - outs["CHOLESKY"]) / np.linalg.norm(outs["CHOLESKY"]))
        res[tag] = r
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
