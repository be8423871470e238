"""Batched serial solve (update + backward + forward) past n + m = 64
(kernels_xl.hip, the size-generic path): ms per solve and per stage.
usage: python scripts/prof_xl.py [reps=3]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pdp-lqr_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from pdplqr import BatchedLQRSolver  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    for n, m, N, batch, keep in [(50, 15, 64, 256, False), (96, 32, 32, 256, False), (96, 32, 32, 256, True),
                                 (160, 40, 16, 64, False)]:
        s = n + m
        E, c, H, h, x0 = bench.gen_batch_device(n, m, N, batch, seed=17, device=dev)
        ws0 = torch.zeros(batch, N * s + n, dtype=torch.float64, device=dev)
        out = torch.empty_like(ws0)
        bs = BatchedLQRSolver(n, m, N, batch, keep_factors=keep, device=0)
        bs.set_model(E, c, H, h)
        st = torch.cuda.Stream(device=dev)
        bs.handle.set_stream(st.cuda_stream)
        ts = []
        with torch.cuda.stream(st):
            for i in range(reps + 1):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                bs.update_problem_data(ws0, sigma=1e-6)
                e0.record(st)
                bs.backward()
                bs.forward(x0, out)
                e1.record(st)
                torch.cuda.synchronize()
                if i:
                    ts.append(e0.elapsed_time(e1))
        ms = float(np.median(ts))
        st_nz = int(np.count_nonzero(bs.status()))
        nonfinite = int((~torch.isfinite(out)).sum().item())
        ok = st_nz == 0 and nonfinite == 0
        print(json.dumps({"n": n, "m": m, "N": N, "batch": batch, "keep_factors": keep, "ms_per_solve": round(ms, 3),
                          "us_per_stage": round(ms * 1e3 / N, 2), "ok": ok, "status_nonzero": st_nz,
                          "nonfinite": nonfinite, "first_bad": [int(v) for v in np.unique(bs.status())[:4]]}),
              flush=True)
        bs.close()


if __name__ == "__main__":
    main()
