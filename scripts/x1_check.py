"""Step-by-step run of the one-wave-per-SIMD (X1) kernel instances with a
synchronize and a progress line after every call (diagnostic: a hang names its
call).  usage: python scripts/x1_check.py BATCH N SOLVERS (comma list of serial, kkt, plain)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pdp-lqr_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from pdplqr import BatchedLQRSolver  # noqa: E402


def say(*a):
    print(f"[{time.time() - T0:7.2f}s]", *a, flush=True)


T0 = time.time()


def main():
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    solvers = sys.argv[3].split(",") if len(sys.argv) > 3 else ["serial", "kkt"]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    n, m, nc, s = 12, 4, 4, 16
    E, c, H, h, x0 = bench.gen_batch_device(n, m, N, batch, seed=555, device=dev)
    ncs = np.array([nc] * N + [0], dtype=np.int32)
    Dk = torch.zeros(nc, s, dtype=torch.float64, device=dev)
    Dk[:, :m] = torch.eye(m, dtype=torch.float64, device=dev)
    D = Dk.t().contiguous().reshape(-1).repeat(batch, N)
    g = torch.Generator(device=dev)
    g.manual_seed(556)
    ny = nc * N
    ws = torch.randn(batch, N * s + n, dtype=torch.float64, device=dev, generator=g)
    ys = torch.randn(batch, ny, dtype=torch.float64, device=dev, generator=g)
    zs = torch.randn(batch, ny, dtype=torch.float64, device=dev, generator=g)
    rho = torch.full((batch, ny), 0.1, dtype=torch.float64, device=dev)
    irho = 1.0 / rho
    out = torch.empty(batch, N * s + n, dtype=torch.float64, device=dev)
    say("data ready", batch, N)
    for solver in solvers:
        if solver == "plain":
            bs = BatchedLQRSolver(n, m, N, batch, device=0)
            bs.set_model(E, c, H, h)
            bs.update_problem_data(ws, sigma=1e-6)
        else:
            bs = BatchedLQRSolver(n, m, N, batch, solver=solver, ncs=ncs, device=0)
            bs.set_model(E, c, H, h, D)
            bs.update_problem_data(ws, ys, zs, irho, sigma=1e-6)
        bs.synchronize()
        say(solver, "update ok")
        if solver == "plain":
            bs.backward()
        else:
            bs.backward(irho if solver == "kkt" else rho)
        bs.synchronize()
        say(solver, "backward ok")
        bs.forward(x0, out)
        bs.synchronize()
        say(solver, "forward ok", float(out.abs().max()))
        bs.close()


if __name__ == "__main__":
    main()
