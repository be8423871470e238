"""Repeatability check of the size-generic serial path (kernels_xl.hip): the
same solve repeated on one handle must give identical bits and a clean status."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pdp-lqr_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from pdplqr import BatchedLQRSolver  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
for (n, m, N, batch, keep) in [(50, 15, 64, 256, False), (96, 32, 32, 256, False), (96, 32, 32, 256, True), (96, 32, 32, 256, True), (96, 32, 32, 256, False)]:
    s = n + m
    E, c, H, h, x0 = bench.gen_batch_device(n, m, N, batch, seed=17, device=dev)
    ws0 = torch.zeros(batch, N * s + n, dtype=torch.float64, device=dev)
    bs = BatchedLQRSolver(n, m, N, batch, keep_factors=keep, device=0)
    bs.set_model(E, c, H, h)
    side = torch.cuda.Stream(device=dev)
    bs.handle.set_stream(side.cuda_stream)
    ref, bad = None, []
    with torch.cuda.stream(side):
        for it in range(12):
            out = torch.full_like(ws0, float("nan"))
            bs.update_problem_data(ws0, sigma=1e-6)
            bs.backward()
            bs.forward(x0, out)
            torch.cuda.synchronize()
            st = bs.status()
            o = out.cpu().numpy()
            if ref is None:
                ref = o
            if np.count_nonzero(st) or not np.isfinite(o).all() or not np.array_equal(o, ref):
                bad.append((it, int(np.count_nonzero(st)), int((~np.isfinite(o)).sum()),
                            float(np.nanmax(np.abs(o - ref)))))
    print(n, m, N, batch, keep, "bad iterations:", bad, flush=True)
    bs.close()
