"""C5 ADMM outer loop only (N = 512, 12/4, nc = 4, batch 1024, |u| <= 0.5,
rho = 1, cold start), for rocprofv3 kernel traces of one iteration's kernels.
usage: python scripts/prof_admm.py [serial|kkt] [iterations=30]"""
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


def main():
    solver = sys.argv[1] if len(sys.argv) > 1 else "kkt"
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    n, m, N, batch, nc = 12, 4, 512, 1024, 4
    s = n + m
    E, c, H, h, x0 = bench.gen_batch_device(n, m, N, batch, seed=555, device=dev)  # bench_conic's data
    ncs = np.array([nc] * N + [0], dtype=np.int32)
    Dk = torch.zeros(nc, s, dtype=torch.float64, device=dev)
    Dk[:, :m] = torch.eye(m, dtype=torch.float64, device=dev)
    D = Dk.t().contiguous().reshape(-1).repeat(batch, N)
    ny = nc * N
    lb = torch.full((batch, ny), -0.5, dtype=torch.float64, device=dev)
    ub = torch.full((batch, ny), 0.5, dtype=torch.float64, device=dev)
    rho = torch.full((batch, ny), 1.0, dtype=torch.float64, device=dev)
    w = torch.zeros(batch, N * s + n, dtype=torch.float64, device=dev)
    y = torch.zeros(batch, ny, dtype=torch.float64, device=dev)
    z = torch.zeros_like(y)
    bs = BatchedLQRSolver(n, m, N, batch, solver=solver, ncs=ncs, keep_factors=(solver == "serial"), device=0)
    bs.set_model(E, c, H, h, D)
    out = {}
    for rep in range(3):
        w.zero_()
        y.zero_()
        z.zero_()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        bs.admm_solve(x0, lb, ub, rho, w, y, z, max_iter=iters, check_every=iters, eps_abs=0.0, eps_rel=0.0)
        torch.cuda.synchronize()
        out[f"rep{rep}_ms_per_iteration"] = (time.perf_counter() - t0) * 1e3 / iters
    out.update(solver=solver, iterations=iters)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
