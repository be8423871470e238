"""Batched serial solve (backward + forward, N = 256, batch 1024) of wide
shapes: the 3 x 3 register-tile instances (wide3_dispatch) and, for contrast,
shapes that keep the block-wide LDS kernels.  Prints one JSON line per shape:
ms per solve and the fraction of 8 TB/s on SURVEY 8(d)'s per-stage bytes
8 (n s + n + s^2 + s) + 8 s.
usage: python scripts/prof_wide.py [reps=5]"""
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
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    N, batch = 256, 1024
    for n, m in [(24, 16), (32, 8), (20, 16), (40, 8), (44, 4), (32, 16), (30, 10), (50, 10)]:
        s = n + m
        E, c, H, h, x0 = bench.gen_batch_device(n, m, N, batch, seed=91, device=dev)
        ws0 = torch.zeros(batch, N * s + n, dtype=torch.float64, device=dev)
        out = torch.empty_like(ws0)
        bs = BatchedLQRSolver(n, m, N, batch, device=0)
        bs.set_model(E, c, H, h)
        bs.update_problem_data(ws0, sigma=1e-6)
        st = torch.cuda.Stream(device=dev)
        bs.handle.set_stream(st.cuda_stream)
        ts = []
        with torch.cuda.stream(st):
            for i in range(reps + 1):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                bs.backward()
                bs.forward(x0, out)
                e1.record(st)
                torch.cuda.synchronize()
                if i:
                    ts.append(e0.elapsed_time(e1))
        ms = float(np.median(ts))
        byts = 8 * (n * s + n + s * s + s) + 8 * s
        ok = bool(np.all(bs.status() == 0)) and bool(torch.isfinite(out).all().item())
        print(json.dumps({"n": n, "m": m, "N": N, "batch": batch, "ms_per_solve": round(ms, 4),
                          "frac_of_8TBs": round(byts * N * batch / (ms * 1e-3) / 8e12, 4), "ok": ok}), flush=True)
        bs.close()


if __name__ == "__main__":
    main()
