"""Same-box A/B of the C5 solve (backward + forward, N = 512, 12/4, nc = 4,
batch 1024; solvers kkt / serial) and of the headline batch (solver "head":
N = 1024, 12/4, batch 4096, backward and forward timed apart) across library
variants.

usage: python scripts/ab_kkt.py [--rounds R] [--solvers kkt+serial+head] LIB [LIB ...]
  LIB: a path to a libpdplqr variant, or "default" (the in-tree library).
Each (round, LIB) runs in a child process (the library is loaded once per
process); prints one line per run and a median summary per LIB.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(solvers, N=512, batch=1024, steps=20, warmup=3):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "pdp-lqr_amd")]
    import numpy as np
    import torch

    import bench
    from pdplqr import BatchedLQRSolver

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    n, m, nc = 12, 4, 4
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
    res = {}
    if "head" in solvers:
        del E, c, H, h, D
        torch.cuda.empty_cache()
        Nh, bh = 1024, 4096
        Eh, ch, Hh, hh, xh = bench.gen_batch_device(n, m, Nh, bh, seed=1234, device=dev)
        bs = BatchedLQRSolver(n, m, Nh, bh, solver="serial")
        bs.set_model(Eh, ch, Hh, hh)
        bs.update_problem_data(torch.zeros(bh, Nh * s + n, dtype=torch.float64, device=dev), sigma=1e-6)
        oh = torch.empty(bh, Nh * s + n, dtype=torch.float64, device=dev)
        bs.backward()
        tb = bench._timed(lambda: bs.backward(), 2 * steps, warmup, dev, None)
        tf = bench._timed(lambda: bs.forward(xh, oh), 2 * steps, warmup, dev, None)
        ok = bool(np.all(bs.status() == 0))
        res["head_bwd"] = {"ms_per_solve": tb * 1e3, "status_ok": ok}
        res["head_fwd"] = {"ms_per_solve": tf * 1e3, "status_ok": ok}
        bs.close()
        solvers = [x for x in solvers if x != "head"]
        if solvers:
            raise SystemExit("head runs alone")
    for solver in solvers:
        bs = BatchedLQRSolver(n, m, N, batch, solver=solver, ncs=ncs)
        bs.set_model(E, c, H, h, D)
        bs.update_problem_data(ws, ys, zs, irho, sigma=1e-6)
        r = irho if solver == "kkt" else rho

        def step():
            bs.backward(r)
            bs.forward(x0, out)

        t = bench._timed(step, steps, warmup, dev, None)
        res[solver] = {"ms_per_solve": t * 1e3, "status_ok": bool(np.all(bs.status() == 0))}
        bs.close()
    print(json.dumps(res), flush=True)


def main():
    args = sys.argv[1:]
    if args and args[0] == "--child":
        child(tuple(args[1:]))
        return
    rounds = 2
    if args and args[0] == "--rounds":
        rounds = int(args[1])
        args = args[2:]
    solvers = ["kkt"]
    if args and args[0] == "--solvers":
        solvers = args[1].split("+")  # (scripts/gpu_run.sh splits its step arguments at commas)
        args = args[2:]
    res = {a: [] for a in args}
    for _ in range(rounds):
        for lib in args:
            env = dict(os.environ)
            if lib != "default":
                env["PDPLQR_LIB"] = lib
            out = subprocess.run([sys.executable, "-u", __file__, "--child"] + solvers, env=env, capture_output=True,
                                 text=True, timeout=300)
            line = [x for x in out.stdout.splitlines() if x.startswith("{")]
            if out.returncode or not line:
                print(lib, "FAILED", out.returncode, out.stderr[-2000:], flush=True)
                sys.exit(1)
            d = json.loads(line[-1])
            res[lib].append(d)
            print(os.path.basename(lib), json.dumps(d), flush=True)
    for lib, rs in res.items():
        for s in (rs[0].keys() if rs else ()):
            v = sorted(r[s]["ms_per_solve"] for r in rs)
            print(f"SUMMARY {os.path.basename(lib)} {s} median {v[len(v) // 2]:.4f} ms  all {v}", flush=True)


if __name__ == "__main__":
    main()
