"""C5 Riccati (N = 512, 12/4, nc = 4 u-box rows, batch 1024) on the PARALLEL
kernels (several segments per problem so several waves share
a SIMD) against the serial path, protocol-timed as bench.py's C5 line
(update_problem_data untimed before every timed backward + forward).
usage: python scripts/c5_parallel_probe.py"""
import json
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


def run(solver, **kw):
    bs = BatchedLQRSolver(n, m, N, batch, solver=solver, ncs=ncs, **kw)
    bs.set_model(E, c, H, h, D)
    out = torch.empty(batch, N * s + n, dtype=torch.float64, device=dev)
    side = torch.cuda.Stream()
    bs.synchronize()
    bs.handle.set_stream(side.cuda_stream)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(7)]
    with torch.cuda.stream(side):
        for e0, e1 in evs:
            bs.update_problem_data(ws, ys, zs, irho, sigma=1e-6)
            e0.record(side)
            bs.backward(rho)
            bs.forward(x0, out)
            e1.record(side)
    torch.cuda.synchronize()
    t = float(np.median([e0.elapsed_time(e1) for e0, e1 in evs[2:]]))
    st = int(np.max(bs.status()))
    bs.close()
    return t, out, st


t0, ref, st0 = run("serial")
print(json.dumps({"solver": "serial", "ms": t0, "status": st0}), flush=True)
for ns, sl in ((2, 0), (4, 0), (8, 0), (4, 64), (8, 32), (16, 32), (2, 128), (4, 128)):
    try:
        t, out, st = run("parallel", num_segments=ns, segment_len=sl)
        err = float((torch.linalg.norm(out - ref) / torch.linalg.norm(ref)).item())
        print(json.dumps({"solver": "parallel", "num_segments": ns, "segment_len": sl, "ms": t, "status": st,
                          "rel_err_vs_serial": err}), flush=True)
    except Exception as e:  # noqa: BLE001
        print(json.dumps({"solver": "parallel", "num_segments": ns, "segment_len": sl, "error": str(e)}), flush=True)
