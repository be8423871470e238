"""C5 KKT / Riccati backward time after different preceding work (diagnostic):
  repeat   backward + forward back to back
  update   update_problem_data, then backward + forward (the protocol)
  stream   a 512 MB device copy (another kernel's traffic), then backward + forward
  idle     the device idle for 2 ms, then backward + forward
  update_copy / update_idle   update_problem_data, then the copy / the idle time
Backward kernel time from events on the solver's stream, median of 5."""
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


def head():
    """The same probe at the headline config (N = 1024, batch 4096, no constraints)."""
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    n, m, N, B = 12, 4, 1024, 4096
    E, c, H, h, x0 = bench.gen_batch_device(n, m, N, B, seed=1234, device=dev)
    ws0 = torch.zeros(B, N * (n + m) + n, dtype=torch.float64, device=dev)
    out = torch.empty_like(ws0)
    big_a = torch.ones(64 << 20, dtype=torch.float64, device=dev)
    big_b = torch.empty_like(big_a)
    bs = BatchedLQRSolver(n, m, N, B, device=0)
    bs.set_model(E, c, H, h)
    bs.update_problem_data(ws0, sigma=1e-6)
    bs.synchronize()
    side = torch.cuda.Stream(device=dev)
    bs.handle.set_stream(side.cuda_stream)
    res = {}
    with torch.cuda.stream(side):
        for mode in ("repeat", "update", "stream", "update_copy", "repeat"):
            ts = []
            for _ in range(5):
                if mode in ("update", "update_copy"):
                    bs.update_problem_data(ws0, sigma=1e-6)
                if mode in ("stream", "update_copy"):
                    big_b.copy_(big_a)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(side)
                bs.backward()
                e1.record(side)
                bs.forward(x0, out)
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            res[mode + ("2" if mode in res else "")] = round(float(np.median(ts)), 4)
    print(json.dumps({"head": res}), flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "head":
        return head()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    n, m, nc, N, batch = 12, 4, 4, 512, 1024
    s = n + m
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
    big_a = torch.ones(64 << 20, dtype=torch.float64, device=dev)
    big_b = torch.empty_like(big_a)
    res = {}
    for solver in ("kkt", "serial"):
        bs = BatchedLQRSolver(n, m, N, batch, solver=solver, ncs=ncs, device=0)
        bs.set_model(E, c, H, h, D)
        bs.update_problem_data(ws, ys, zs, irho, sigma=1e-6)
        bs.synchronize()
        torch.cuda.synchronize()
        side = torch.cuda.Stream(device=dev)
        bs.handle.set_stream(side.cuda_stream)
        r = irho if solver == "kkt" else rho
        out_s = {}
        with torch.cuda.stream(side):
            for mode in ("repeat", "update", "stream", "idle", "update_copy", "update_idle", "repeat"):
                ts = []
                for _ in range(5):
                    if mode == "update":
                        bs.update_problem_data(ws, ys, zs, irho, sigma=1e-6)
                    elif mode == "stream":
                        big_b.copy_(big_a)
                    elif mode == "idle":
                        torch.cuda.synchronize()
                        time.sleep(0.002)
                    elif mode == "update_copy":
                        bs.update_problem_data(ws, ys, zs, irho, sigma=1e-6)
                        big_b.copy_(big_a)
                    elif mode == "update_idle":
                        bs.update_problem_data(ws, ys, zs, irho, sigma=1e-6)
                        torch.cuda.synchronize()
                        time.sleep(0.002)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(side)
                    bs.backward(r)
                    e1.record(side)
                    bs.forward(x0, out)
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1))
                out_s[mode + ("2" if mode in out_s else "")] = round(float(np.median(ts)), 4)
        res[solver] = out_s
        bs.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
