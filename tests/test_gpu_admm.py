"""ADMM outer loop on the GPU (pdplqr_admm_solve, csrc/admm.hip) against the
oracle's restatement (oracle.admm_solve), which tests/test_oracle_admm.py pins
to an independent KKT certificate.

* fixed iteration counts (eps = 0): every solver kind, warm starts, several
  problems per batch -- the whole iterate (w, y, z) within 1e-9 relative of
  the oracle (1e-8 on the KKT path, as tests/test_gpu_kkt.py);
* converged runs: the same per-problem iteration counts and convergence flags
  as the oracle, frozen problems keep their answer while others iterate;
* config C5 at its size (N = 512, 12/4, nc = 4, batch 1024): finite, status
  clean, sampled problems vs the oracle;
* device (torch) buffers give the same bits as host buffers; the model-level
  API (LQRSolver.admm_solve over Node.e_lb / e_ub) matches the oracle.
All calls go through the C ABI (libpdplqr.so).
"""
import numpy as np
import pytest

from conftest import rel_err
from oracle.oracle import admm_solve as oracle_admm
from pdplqr.model import pack_model, pack_stage_vectors
from pdplqr.problems import quadrotor_model, random_model

pytestmark = pytest.mark.gpu

TOL = 1e-9
TOL_KKT = 1e-8


@pytest.fixture(scope="module", autouse=True)
def _device():
    from pdplqr import device_count

    assert device_count() > 0, "no HIP device visible: GPU tests must run on an MI355X"


def _batch(models, x0s, seed=0, warm=True):
    """Stack packed models into the boundary's batch-major arrays; random warm
    starts (w, y, z) when `warm`."""
    pms = [pack_model(m) for m in models]
    ncs = [int(x) for x in pms[0].ncs]
    g = np.random.default_rng(seed)
    A = {k: np.ascontiguousarray(np.stack([getattr(p, k) for p in pms])) for k in "E c H h D".split()}
    lb = np.stack([np.clip(pack_stage_vectors([nd.e_lb for nd in m.nodes], ncs), -1e20, 1e20) for m in models])
    ub = np.stack([np.clip(pack_stage_vectors([nd.e_ub for nd in m.nodes], ncs), -1e20, 1e20) for m in models])
    B, W, Y = len(models), pms[0].h.size, int(sum(ncs))
    ws = 0.1 * g.standard_normal((B, W)) if warm else np.zeros((B, W))
    ys = 0.1 * g.standard_normal((B, Y)) if warm else np.zeros((B, Y))
    zs = 0.1 * g.standard_normal((B, Y)) if warm else np.zeros((B, Y))
    return pms, ncs, A, np.ascontiguousarray(lb), np.ascontiguousarray(ub), np.ascontiguousarray(np.stack(x0s)), ws, ys, zs


def _ubox_models(B, n=6, m=3, N=40, nc=3, bound=0.3, seed0=100):
    models, x0s = [], []
    for b in range(B):
        mod, x0 = random_model(n, m, N, seed=seed0 + b, nc=nc, D_kind="ubox")
        for nd in mod.nodes:
            if nd.n_con:
                nd.e_lb[:] = -bound
                nd.e_ub[:] = bound
        models.append(mod)
        x0s.append(x0)
    return models, x0s


def _run_gpu(solver, pms, ncs, A, lb, ub, x0, ws, ys, zs, rho, keep=True, **st):
    from pdplqr import BatchedLQRSolver

    p = pms[0]
    kw = {}
    if solver.startswith("parallel"):
        kw = {"num_segments": 4, "condensed": solver.split("-")[1]}
    bs = BatchedLQRSolver(p.n, p.m, p.N, len(pms), solver=solver.split("-")[0], keep_factors=keep, ncs=ncs, **kw)
    bs.set_model(A["E"], A["c"], A["H"], A["h"], A["D"])
    w, y, z = ws.copy(), ys.copy(), zs.copy()
    info = bs.admm_solve(x0, lb, ub, rho, w, y, z, **st)
    assert np.count_nonzero(bs.status()) == 0
    bs.close()
    return w, y, z, info


SOLVERS = [("serial", True), ("serial", False), ("parallel-LU", True), ("parallel-CHOLESKY", True)]


@pytest.mark.parametrize("solver,keep", SOLVERS)
def test_fixed_iterations_match_oracle(solver, keep):
    models, x0s = _ubox_models(5)
    pms, ncs, A, lb, ub, x0, ws, ys, zs = _batch(models, x0s, seed=1)
    rho = np.full(lb.shape, 10.0)
    w, y, z, info = _run_gpu(solver, pms, ncs, A, lb, ub, x0, ws, ys, zs, rho, keep, max_iter=40, eps_abs=0.0,
                             eps_rel=0.0)
    assert info["iterations"] == 40 and np.all(info["iters"] == 40) and not info["converged"].any()
    okw = {"num_segments": 4, "condensed": solver.split("-")[1]} if solver.startswith("parallel") else {}
    for b in range(len(pms)):
        ow, oy, oz, oi = oracle_admm(pms[b], x0[b], lb[b], ub[b], rho[b], ws[b], ys[b], zs[b],
                                     solver=solver.split("-")[0], max_iter=40, eps_abs=0.0, eps_rel=0.0, **okw)
        assert rel_err(w[b], ow) < TOL and rel_err(y[b], oy) < TOL and rel_err(z[b], oz) < TOL, b
        assert abs(info["prim_res"][b] - oi["prim_res"]) <= 1e-9 * max(oi["prim_res"], 1e-300) + 1e-15


def test_kkt_solver_fixed_iterations():
    """QDLDLSolver x-updates (P = 16 path: 12/4, nc = 4 box on u)."""
    models, x0s = _ubox_models(3, n=12, m=4, N=48, nc=4, bound=0.5, seed0=300)
    pms, ncs, A, lb, ub, x0, ws, ys, zs = _batch(models, x0s, seed=2)
    rho = np.full(lb.shape, 10.0)
    w, y, z, info = _run_gpu("kkt", pms, ncs, A, lb, ub, x0, ws, ys, zs, rho, False, max_iter=30, eps_abs=0.0,
                             eps_rel=0.0)
    for b in range(len(pms)):
        ow, oy, oz, _ = oracle_admm(pms[b], x0[b], lb[b], ub[b], rho[b], ws[b], ys[b], zs[b], solver="kkt",
                                    max_iter=30, eps_abs=0.0, eps_rel=0.0)
        assert rel_err(w[b], ow) < TOL_KKT and rel_err(y[b], oy) < TOL_KKT and rel_err(z[b], oz) < TOL_KKT, b


def test_kkt_linear_pass_equals_refactor(monkeypatch):
    """12/4 KKT x-updates after the first: the right-hand-side pass on the
    factor cache (k_kkt_ric_nofact) against re-running the whole Riccati-
    ordered backward every iteration (PDPLQR_KKT_NO_LINEAR=1) -- the same
    matrix, so the same iterates to rounding -- and both against the oracle
    (a box on u at every stage, nc = 4)."""
    models, x0s = _ubox_models(3, n=12, m=4, N=37, nc=4, bound=0.4, seed0=310)
    pms, ncs, A, lb, ub, x0, ws, ys, zs = _batch(models, x0s, seed=3)
    rho = np.full(lb.shape, 5.0)
    st = dict(max_iter=25, eps_abs=0.0, eps_rel=0.0)
    w1, y1, z1, _ = _run_gpu("kkt", pms, ncs, A, lb, ub, x0, ws, ys, zs, rho, False, **st)
    monkeypatch.setenv("PDPLQR_KKT_NO_LINEAR", "1")
    w2, y2, z2, _ = _run_gpu("kkt", pms, ncs, A, lb, ub, x0, ws, ys, zs, rho, False, **st)
    monkeypatch.delenv("PDPLQR_KKT_NO_LINEAR")
    assert rel_err(w1, w2) < 1e-11 and rel_err(y1, y2) < 1e-11 and rel_err(z1, z2) < 1e-11
    for b in range(len(pms)):
        ow, oy, oz, _ = oracle_admm(pms[b], x0[b], lb[b], ub[b], rho[b], ws[b], ys[b], zs[b], solver="kkt", **st)
        assert rel_err(w1[b], ow) < TOL_KKT and rel_err(y1[b], oy) < TOL_KKT and rel_err(z1[b], oz) < TOL_KKT, b


@pytest.mark.parametrize("check_every", [1, 25])
def test_converged_runs_freeze_per_problem(check_every):
    """Quadrotor with 4 start heights: each problem converges at its own
    iteration, identical to a single-problem oracle run, and stays frozen."""
    models, x0s = [], []
    for hgt in (-1.0, 0.0, 0.5, -2.0):
        mod, x0 = quadrotor_model(30, nc_on=True)
        x0 = x0.copy()
        x0[2] = hgt
        models.append(mod)
        x0s.append(x0)
    pms, ncs, A, lb, ub, x0, ws, ys, zs = _batch(models, x0s, warm=False)
    rho = np.full(lb.shape, 0.1)
    st = dict(max_iter=4000, check_every=check_every, eps_abs=1e-6, eps_rel=1e-6)
    w, y, z, info = _run_gpu("serial", pms, ncs, A, lb, ub, x0, ws, ys, zs, rho, True, **st)
    assert info["converged"].all()
    assert len(set(info["iters"].tolist())) > 1, "vacuous: all problems converged together"
    for b in range(len(pms)):
        ow, oy, oz, oi = oracle_admm(pms[b], x0[b], lb[b], ub[b], rho[b], solver="serial", **st)
        assert oi["converged"] and info["iters"][b] == oi["iters"], (b, info["iters"][b], oi["iters"])
        assert rel_err(w[b], ow) < 1e-9 and rel_err(y[b], oy) < 1e-9, b


def test_c5_full_size_admm():
    """Config C5 at its size: N = 512, 12/4, nc = 4 (D = [I 0], |u| <= 0.5),
    batch 1024, rho = 1, 20 fixed iterations; sampled problems vs the oracle."""
    import torch

    from bench import gen_batch_device
    from pdplqr import BatchedLQRSolver
    from pdplqr.model import PackedModel

    n, m, nc, N, B = 12, 4, 4, 512, 1024
    s = n + m
    dev = torch.device("cuda", 0)
    E, c, H, h, x0 = gen_batch_device(n, m, N, B, seed=555, device=dev)
    ncs = np.array([nc] * N + [0], dtype=np.int32)
    Dk = torch.zeros(nc, s, dtype=torch.float64, device=dev)
    Dk[:, :m] = torch.eye(m, dtype=torch.float64, device=dev)
    D = Dk.t().contiguous().reshape(-1).repeat(B, N)
    ny = nc * N
    lb = torch.full((B, ny), -0.5, dtype=torch.float64, device=dev)
    ub = torch.full((B, ny), 0.5, dtype=torch.float64, device=dev)
    rho = torch.full((B, ny), 1.0, dtype=torch.float64, device=dev)
    ws = torch.zeros(B, N * s + n, dtype=torch.float64, device=dev)
    ys = torch.zeros(B, ny, dtype=torch.float64, device=dev)
    zs = torch.zeros(B, ny, dtype=torch.float64, device=dev)
    bs = BatchedLQRSolver(n, m, N, B, solver="serial", keep_factors=True, ncs=ncs)
    bs.set_model(E, c, H, h, D)
    info = bs.admm_solve(x0, lb, ub, rho, ws, ys, zs, max_iter=20, eps_abs=0.0, eps_rel=0.0)
    bs.synchronize()
    assert np.count_nonzero(bs.status()) == 0
    assert bool(torch.isfinite(ws).all()) and bool(torch.isfinite(ys).all())
    assert float(zs.abs().max()) <= 0.5
    bs.close()
    Dh = D.cpu().numpy()
    arr = [t.cpu().numpy() for t in (E, c, H, h, x0, ws, ys, zs)]
    for b in sorted({0, 1, B - 1} | set(np.random.default_rng(9).choice(B, 3, replace=False).tolist())):
        pm = PackedModel(n, m, N, ncs, arr[0][b], arr[1][b], arr[2][b], arr[3][b], Dh[b])
        ow, oy, oz, _ = oracle_admm(pm, arr[4][b], np.full(ny, -0.5), np.full(ny, 0.5), np.full(ny, 1.0),
                                    max_iter=20, eps_abs=0.0, eps_rel=0.0)
        assert rel_err(arr[5][b], ow) < TOL and rel_err(arr[6][b], oy) < TOL and rel_err(arr[7][b], oz) < TOL, b


def test_device_buffers_equal_host_buffers():
    import torch

    models, x0s = _ubox_models(4)
    pms, ncs, A, lb, ub, x0, ws, ys, zs = _batch(models, x0s, seed=3)
    rho = np.full(lb.shape, 10.0)
    st = dict(max_iter=60, check_every=10, eps_abs=1e-7, eps_rel=1e-7)
    hw, hy, hz, hi = _run_gpu("serial", pms, ncs, A, lb, ub, x0, ws, ys, zs, rho, True, **st)
    dev = torch.device("cuda", 0)
    T = {k: torch.from_numpy(v).to(dev) for k, v in A.items()}
    t = [torch.from_numpy(a).to(dev) for a in (lb, ub, x0, ws, ys, zs, rho)]
    from pdplqr import BatchedLQRSolver

    p = pms[0]
    bs = BatchedLQRSolver(p.n, p.m, p.N, len(pms), keep_factors=True, ncs=ncs)
    bs.set_model(T["E"], T["c"], T["H"], T["h"], T["D"])
    di = bs.admm_solve(t[2], t[0], t[1], t[6], t[3], t[4], t[5], **st)
    torch.cuda.synchronize()
    assert np.array_equal(t[3].cpu().numpy(), hw) and np.array_equal(t[4].cpu().numpy(), hy)
    assert np.array_equal(t[5].cpu().numpy(), hz) and np.array_equal(di["iters"], hi["iters"])
    bs.close()


def test_model_level_api_quadrotor():
    """LQRSolver(model).admm_solve over the nodes' e_lb / e_ub, warm start from
    initialize_vectors (lqr_example.cpp:12-46), against the oracle."""
    from pdplqr import LQRParallelSolver, LQRSolver, QDLDLSolver, initialize_vectors

    model, x0 = quadrotor_model(30, nc_on=True)
    x0 = x0.copy()
    x0[2] = -1.0
    pm = pack_model(model)
    ncs = [int(x) for x in pm.ncs]
    lb = np.clip(pack_stage_vectors([nd.e_lb for nd in model.nodes], ncs), -1e20, 1e20)
    ub = np.clip(pack_stage_vectors([nd.e_ub for nd in model.nodes], ncs), -1e20, 1e20)
    st = dict(max_iter=3000, check_every=25, eps_abs=1e-6, eps_rel=1e-6)
    for kind, solver in (("serial", LQRSolver(model)), ("parallel", LQRParallelSolver(model, 4))):
        ws, ys, zs, rho_vecs, _ = initialize_vectors(model, 0.1)
        info = solver.admm_solve(x0, ws, ys, zs, rho_vecs, **st)
        okw = {"num_segments": 4} if kind == "parallel" else {}
        ow, oy, oz, oi = oracle_admm(pm, x0, lb, ub, np.full(lb.size, 0.1), solver=kind, **st, **okw)
        assert info["converged"] and info["iters"] == oi["iters"], (kind, info, oi)
        w = np.concatenate(ws)
        assert rel_err(w, ow) < 1e-9 and rel_err(np.concatenate(ys), oy) < 1e-9, kind
    q = QDLDLSolver(model)
    ws, ys, zs, rho_vecs, _ = initialize_vectors(model, 0.1)
    info = q.admm_solve(x0, ws, ys, zs, rho_vecs, **st)
    ow, oy, oz, oi = oracle_admm(pm, x0, lb, ub, np.full(lb.size, 0.1), solver="kkt", **st)
    assert info["converged"] == oi["converged"]
    assert rel_err(np.concatenate(ws), ow) < 1e-7


@pytest.mark.parametrize("solver", ["serial", "parallel-LU", "kkt"])
def test_adaptive_rho_matches_oracle(solver):
    """OSQP's adaptive rho on the device: from rho = 0.1 (which stalls on these
    problems) every problem rescales on its own schedule and converges; the
    per-problem iteration counts, final rho and iterate equal the oracle's."""
    if solver == "kkt":
        models, x0s = _ubox_models(3, n=12, m=4, N=48, nc=4, bound=0.5, seed0=400)
    else:
        models, x0s = _ubox_models(4)
    pms, ncs, A, lb, ub, x0, ws, ys, zs = _batch(models, x0s, warm=False)
    rho = np.full(lb.shape, 0.1)
    st = dict(max_iter=3000, check_every=25, eps_abs=1e-7, eps_rel=1e-7)
    w, y, z, info = _run_gpu(solver, pms, ncs, A, lb, ub, x0, ws, ys, zs, rho, True, **st)
    okw = {"num_segments": 4, "condensed": "LU"} if solver.startswith("parallel") else {}
    tol = TOL_KKT if solver == "kkt" else 1e-9
    for b in range(len(pms)):
        ow, oy, oz, oi = oracle_admm(pms[b], x0[b], lb[b], ub[b], rho[b], solver=solver.split("-")[0], **st, **okw)
        assert oi["converged"] and oi["rho_updates"] >= 1, oi
        assert bool(info["converged"][b]) and info["iters"][b] == oi["iters"], (b, info["iters"][b], oi["iters"])
        # rho is a product of residual ratios: residuals are differences of
        # iterates near convergence (eps 1e-7), so they carry the path's rounding
        # amplified.  KKT: the GPU's explicit H^-1 / block LDL^T against the
        # oracle's sparse LDL^T leave ~1e-6 on rho (measured 1.0e-6) -- 1e-5
        assert rel_err(info["rho"][b], oi["rho"]) < (1e-5 if solver == "kkt" else 1e-9), b
        assert rel_err(w[b], ow) < tol and rel_err(y[b], oy) < tol, b


@pytest.mark.parametrize("solver", ["serial", "kkt"])
@pytest.mark.parametrize("check_every,adaptive", [(1, False), (5, True), (25, True)])
def test_fused_update_equals_unfused(check_every, adaptive, solver):
    """At 12/4 with 4 rows per stage (C5's layout) the serial solver runs the
    ADMM update inside the streamed backward (k_nofact_admm_dma), the KKT
    solver inside its rollout (k_kkt_ric_fwd<3, true, ...>).  Same per-problem
    iteration counts, convergence flags and rho as the separate update pass
    (PDPLQR_NO_ADMM_FUSE), iterates to 1e-8, and the oracle."""
    import os

    n, m, nc, N, B = 12, 4, 4, 60, 6
    models, x0s = [], []
    for b in range(B):
        mod, x0 = random_model(n, m, N, seed=700 + b, nc=nc, D_kind="ubox")
        for k, nd in enumerate(mod.nodes):
            if nd.n_con:
                nd.e_lb[:] = -0.4 - 0.1 * b
                nd.e_ub[:] = 0.4 + 0.1 * b
        models.append(mod)
        x0s.append(x0)
    # terminal stage without constraints (the fused layout): rebuild the models
    from pdplqr.model import LQRModel

    fixed = []
    for mod in models:
        nm = LQRModel(n, m, N)
        for k, nd in enumerate(mod.nodes):
            nm.add_node(n, m, nc if k < N else 0, k, k == N)
            t = nm.nodes[k]
            t.H[:] = nd.H
            t.h[:] = nd.h
            if k < N:
                t.E[:] = nd.E
                t.c[:] = nd.c
                t.D_con[:] = nd.D_con
                t.e_lb[:] = nd.e_lb
                t.e_ub[:] = nd.e_ub
        fixed.append(nm)
    pms, ncs, A, lb, ub, x0, ws, ys, zs = _batch(fixed, x0s, seed=9)
    rho = np.full(lb.shape, 0.3)
    st = dict(max_iter=400, check_every=check_every, eps_abs=1e-6, eps_rel=1e-6, adaptive_rho=adaptive)
    res = {}
    for mode in ("fused", "separate"):
        if mode == "separate":
            os.environ["PDPLQR_NO_ADMM_FUSE"] = "1"
        try:
            res[mode] = _run_gpu(solver, pms, ncs, A, lb, ub, x0, ws, ys, zs, rho, solver == "serial", **st)
        finally:
            os.environ.pop("PDPLQR_NO_ADMM_FUSE", None)
    (wf, yf, zf, fi), (wsep, ysep, zsep, si) = res["fused"], res["separate"]
    assert np.array_equal(fi["iters"], si["iters"]) and np.array_equal(fi["converged"], si["converged"])
    assert fi["converged"].any() or not adaptive  # fixed rho = 0.3 needs more than 400 iterations here
    for a, b_ in ((wf, wsep), (yf, ysep), (zf, zsep), (fi["rho"], si["rho"])):
        d = np.linalg.norm(a - b_, axis=1) / np.maximum(np.linalg.norm(b_, axis=1), 1e-300)
        # rounding of the fused h~ sum (permlane tree vs k_penalty's sequential
        # sum) carried through up to 400 contractive iterations and rho changes
        assert float(d.max()) < 1e-8, float(d.max())
    tol = 1e-9 if solver == "serial" else TOL_KKT
    for b in (0, B - 1):
        ow, oy, oz, oi = oracle_admm(pms[b], x0[b], lb[b], ub[b], rho[b], ws[b], ys[b], zs[b], solver=solver, **st)
        assert oi["iters"] == fi["iters"][b]
        assert rel_err(wf[b], ow) < tol and rel_err(yf[b], oy) < tol, b


def test_invalid_bounds_and_rho_are_rejected():
    """e_lb > e_ub on a row, or rho <= 0, is an ERR_INVALID before any solve
    (OSQP's validation); the C-ABI message names it."""
    from pdplqr import PdplqrError

    models, x0s = _ubox_models(2)
    pms, ncs, A, lb, ub, x0, ws, ys, zs = _batch(models, x0s)
    rho = np.full(lb.shape, 1.0)
    bad = lb.copy()
    bad[1, 5] = ub[1, 5] + 1.0
    with pytest.raises(PdplqrError) as e:
        _run_gpu("serial", pms, ncs, A, bad, ub, x0, ws, ys, zs, rho, True, max_iter=5)
    assert "e_lb > e_ub" in str(e.value)
    r2 = rho.copy()
    r2[0, 0] = 0.0
    with pytest.raises(PdplqrError):
        _run_gpu("serial", pms, ncs, A, lb, ub, x0, ws, ys, zs, r2, True, max_iter=5)
    w, y, z, info = _run_gpu("serial", pms, ncs, A, lb, ub, x0, ws, ys, zs, rho, True, max_iter=5)
    assert info["iterations"] == 5


def test_adaptive_rho_no_active_row_keeps_rho():
    """No row active at any check (bounds +-1e6): |D^T y| = 0, the rescale is
    skipped on the device as in the oracle, and rho stays at its start value."""
    models, x0s = _ubox_models(3, bound=1e6)
    pms, ncs, A, lb, ub, x0, ws, ys, zs = _batch(models, x0s, warm=False)
    rho = np.full(lb.shape, 0.1)
    st = dict(max_iter=100, check_every=5, eps_abs=1e-12, eps_rel=1e-12)
    w, y, z, info = _run_gpu("serial", pms, ncs, A, lb, ub, x0, ws, ys, zs, rho, True, **st)
    for b in range(len(pms)):
        ow, oy, oz, oi = oracle_admm(pms[b], x0[b], lb[b], ub[b], rho[b], solver="serial", **st)
        assert oi["rho_updates"] == 0
        assert np.all(info["rho"][b] == 0.1), info["rho"][b]
        assert rel_err(w[b], ow) < 1e-9


def _xbox_models(B, N=32, xb=0.1, ub_=0.5, seed0=900):
    """12/4, four rows per stage: a box on u_0, u_1 and on the states x_0, x_1
    (stage 0's state rows unbounded: x_0 is fixed); terminal rows box x_0..x_3.
    Active state rows at a large rho put ~rho straight into P, which drives
    rho_dyn ||P|| of the KKT path's lambda elimination out of the Neumann range."""
    n, m = 12, 4
    models, x0s = [], []
    for b in range(B):
        mod, x0 = random_model(n, m, N, seed=seed0 + b, nc=4, D_kind="ubox")
        for k, nd in enumerate(mod.nodes):
            nd.D_con[:] = 0.0
            if k < N:
                nd.D_con[0, 0] = nd.D_con[1, 1] = 1.0
                nd.D_con[2, m] = nd.D_con[3, m + 1] = 1.0
                nd.e_lb[:2], nd.e_ub[:2] = -ub_, ub_
                xr = 1e6 if k == 0 else xb
                nd.e_lb[2:], nd.e_ub[2:] = -xr, xr
            else:
                for r in range(4):
                    nd.D_con[r, r] = 1.0
                nd.e_lb[:], nd.e_ub[:] = -xb, xb
        models.append(mod)
        x0s.append(x0)
    return models, x0s


def test_kkt_state_box_large_rho_fixed_iterations():
    """ADMM-KKT with active state boxes at rho = 3e5 (rho_dyn ||P|| ~ 0.4: the
    exact Moreau envelope on every stage), fixed iterations, iterates vs the
    oracle's QDLDL at 1e-8."""
    models, x0s = _xbox_models(3)
    pms, ncs, A, lb, ub, x0, ws, ys, zs = _batch(models, x0s, seed=4)
    rho = np.full(lb.shape, 3e5)
    st = dict(max_iter=60, eps_abs=0.0, eps_rel=0.0, adaptive_rho=False)
    w, y, z, info = _run_gpu("kkt", pms, ncs, A, lb, ub, x0, ws, ys, zs, rho, False, **st)
    for b in range(len(pms)):
        ow, oy, oz, _ = oracle_admm(pms[b], x0[b], lb[b], ub[b], rho[b], ws[b], ys[b], zs[b], solver="kkt", **st)
        assert rel_err(w[b], ow) < TOL_KKT and rel_err(y[b], oy) < TOL_KKT and rel_err(z[b], oz) < TOL_KKT, b


def test_kkt_state_box_adaptive_rho_reaches_large_rho():
    """Adaptive rho from 1e4 on state-boxed problems: problem 0 rescales up to
    rho ~ 3e5 before it converges (oracle: 6 rescales, 1000 iterations).  Same
    iteration counts and convergence as the oracle.  rho is a product of six
    residual ratios taken at ~1e-6 residuals, so it carries the two paths'
    rounding amplified (measured 1.05e-5 relative): 1e-4; the iterates then
    agree to the termination tolerance's scale (1e-6 relative)."""
    models, x0s = _xbox_models(2)
    pms, ncs, A, lb, ub, x0, ws, ys, zs = _batch(models, x0s, warm=False)
    rho = np.full(lb.shape, 1e4)
    st = dict(max_iter=3000, check_every=5, eps_abs=1e-6, eps_rel=1e-6)
    w, y, z, info = _run_gpu("kkt", pms, ncs, A, lb, ub, x0, ws, ys, zs, rho, True, **st)
    reached = 0.0
    for b in range(len(pms)):
        ow, oy, oz, oi = oracle_admm(pms[b], x0[b], lb[b], ub[b], rho[b], solver="kkt", **st)
        assert oi["converged"] and bool(info["converged"][b])
        assert info["iters"][b] == oi["iters"], (b, info["iters"][b], oi["iters"])
        assert rel_err(info["rho"][b], oi["rho"]) < 1e-4, b
        assert rel_err(w[b], ow) < 1e-6 and rel_err(y[b], oy) < 1e-6, (b, rel_err(w[b], ow), rel_err(y[b], oy))
        reached = max(reached, float(np.max(oi["rho"])))
    assert reached >= 1e5, reached
