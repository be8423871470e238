"""Sweep the device segment length of the PARALLEL solver for one problem
(default: C2, N = 1024, 12/4) and print ms per backward + forward for each,
next to the automatic choice (segment_len = 0).
python scripts/sweep_seglen.py [n m N L1 L2 ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pdp-lqr_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from pdplqr import BatchedLQRSolver  # noqa: E402


def main():
    a = [int(x) for x in sys.argv[1:]]
    n, m, N = (a[:3] if len(a) >= 3 else [12, 4, 1024])
    Ls = a[3:] or [0, 1, 2, 4, 8, 16, 32, 64]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    E, c, H, h, x0 = bench.gen_batch_device(n, m, N, 1, seed=77, device=dev)
    ws0 = torch.zeros(1, N * (n + m) + n, dtype=torch.float64, device=dev)
    out = torch.empty_like(ws0)
    for L in Ls:
        bs = BatchedLQRSolver(n, m, N, 1, solver="parallel", num_segments=8, keep_factors=True, device=0,
                              segment_len=L)
        bs.set_model(E, c, H, h)
        bs.update_problem_data(ws0, sigma=1e-6)

        def step():
            bs.backward()
            bs.forward(x0, out)

        t = bench._timed(step, 10, 3, dev, None)
        print(json.dumps({"n": n, "m": m, "N": N, "segment_len": L, "ms": round(t * 1e3, 4)}), flush=True)
        bs.close()


if __name__ == "__main__":
    main()
