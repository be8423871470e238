"""GPU parity of the serial solver for stage sizes 64 < n + m <= 256
(csrc/kernels_xl.hip: one 256-thread block per problem, the stage matrices in
a per-problem global-memory workspace, the reference's factor form
lqr_kernel.hpp:80-212 restated literally) against the size-generic CPU oracle.

Covers backward with and without kept factors, forward, the value function,
backward_without_factorization, rho-penalised stages, the status of an
indefinite stage, and the ADMM loop over the serial solver (k_admm_update_xl).  Tolerance 1e-9 relative, as the
other serial parity tests.  The KKT solver (QDLDLSolver, k_kkt_ric_bwd_xl /
k_kkt_ric_fwd_xl) against OracleKKT's QDLDL at 1e-8, as the other KKT tests,
on both sides of the Neumann / exact P~ switch, and its ADMM loop.  The
PARALLEL solver (kernels_xl_par.hip: stage kernels past n + m = 64, element
kernels past n = 64) against OracleParallel and OracleSerial at 1e-9, both
condensed forms, backward_without_factorization and horizon shards."""
import numpy as np
import pytest

from conftest import rel_err
from oracle.oracle import OracleSerial
from pdplqr.model import PackedModel
from pdplqr.problems import random_batch_arrays

pytestmark = pytest.mark.gpu
TOL = 1e-9

# (n, m, N, batch): s = 65 (smallest), 70, 100 (m > n), 128, 160
SHAPES = [(50, 15, 6, 2), (40, 30, 5, 2), (36, 64, 4, 2), (100, 28, 3, 2), (120, 40, 2, 1)]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    from pdplqr import device_count

    assert device_count() > 0, "no HIP device visible"


def _problem(n, m, N, batch, nc, seed):
    E, c, H, h, x0 = random_batch_arrays(n, m, N, batch, seed)
    s = n + m
    g = np.random.default_rng(seed + 1)
    ncs = np.full(N + 1, nc, dtype=np.int32)
    dims = [s] * N + [n]
    D = np.concatenate([g.standard_normal((batch, nc * dk)) for dk in dims], axis=1) if nc else np.zeros((batch, 0))
    ny = int(ncs.sum())
    ws = 0.1 * g.standard_normal((batch, N * s + n))
    ys, zs = g.standard_normal((batch, ny)), g.standard_normal((batch, ny))
    irho = 0.05 + g.random((batch, ny))
    return dict(E=E, c=c, H=H, h=h, x0=x0, ncs=ncs, D=D, ws=ws, ys=ys, zs=zs, irho=irho, nc=nc)


def _oracle(p, b, n, m, N, ws=None, nofact_ws=None):
    nc = p["nc"]
    pm = PackedModel(n, m, N, p["ncs"], p["E"][b], p["c"][b], p["H"][b], p["h"][b], p["D"][b] if nc else np.zeros(0))
    o = OracleSerial(pm)
    args = lambda w: (w, p["ys"][b] if nc else None, p["zs"][b] if nc else None, p["irho"][b] if nc else None, 1e-6)
    o.update_problem_data(*args(p["ws"][b] if ws is None else ws))
    o.backward((1.0 / p["irho"][b]) if nc else None)
    if nofact_ws is not None:
        o.update_problem_data(*args(nofact_ws))
        o.backward_without_factorization((1.0 / p["irho"][b]) if nc else None)
    return o, o.forward(p["x0"][b])


@pytest.mark.parametrize("n,m,N,batch", SHAPES)
@pytest.mark.parametrize("keep", [False, True])
@pytest.mark.parametrize("nc", [0, 3])
def test_xl_serial_matches_oracle(n, m, N, batch, keep, nc):
    from pdplqr import BatchedLQRSolver

    p = _problem(n, m, N, batch, nc, 11 * n + m + nc)
    bs = BatchedLQRSolver(n, m, N, batch, solver="serial", keep_factors=keep, ncs=p["ncs"])
    bs.set_model(p["E"], p["c"], p["H"], p["h"], p["D"] if nc else None)
    rho = (1.0 / p["irho"]) if nc else None
    bs.update_problem_data(p["ws"], p["ys"] if nc else None, p["zs"] if nc else None, p["irho"] if nc else None,
                           sigma=1e-6)
    bs.backward(rho)
    out = np.zeros_like(p["ws"])
    bs.forward(p["x0"], out)
    assert np.all(bs.status() == 0)
    for b in range(batch):
        o, ref = _oracle(p, b, n, m, N)
        assert rel_err(out[b], ref) < TOL, b
        if keep:
            for k in (0, N):
                P, pv = bs.value_function(b, k)
                Po, po = o.value_function(k)
                assert rel_err(P, Po) < TOL and rel_err(pv, po) < 1e-8, (b, k)
    if keep:  # lqr_solver.hpp:65-70: new linear data on the kept factors
        ws1 = p["ws"] + 0.2 * np.random.default_rng(n).standard_normal(p["ws"].shape)
        bs.update_problem_data(ws1, p["ys"] if nc else None, p["zs"] if nc else None, p["irho"] if nc else None,
                               sigma=1e-6)
        bs.backward_without_factorization(rho)
        out1 = np.zeros_like(out)
        bs.forward(p["x0"], out1)
        for b in range(batch):
            _, ref1 = _oracle(p, b, n, m, N, nofact_ws=ws1[b])
            assert rel_err(out1[b], ref1) < TOL, b
    bs.close()


@pytest.mark.parametrize("keep", [False, True])
def test_xl_indefinite_stage_sets_status(keep):
    """An indefinite stage matrix: the factorisation of that stage fails (a
    control pivot), as k_riccati_bwd_big's full factor does."""
    from pdplqr import BatchedLQRSolver

    n, m, N, batch = 50, 20, 6, 2
    E, c, H, h, x0 = random_batch_arrays(n, m, N, batch, 5)
    s = n + m
    H = H.copy()
    H[1, 3 * s * s:4 * s * s] = -np.eye(s).reshape(-1)  # stage 3 of problem 1
    bs = BatchedLQRSolver(n, m, N, batch, keep_factors=keep)
    bs.set_model(E, c, H, h)
    bs.update_problem_data(np.zeros((batch, N * s + n)), sigma=0.0)
    bs.backward()
    st = bs.status()
    assert st[0] == 0 and st[1] == 3 + 1
    bs.close()


KKT_SHAPES = [(50, 15, 6, 2), (36, 64, 4, 2), (100, 28, 3, 2)]


@pytest.mark.parametrize("n,m,N,batch", KKT_SHAPES)
@pytest.mark.parametrize("nc", [0, 3])
@pytest.mark.parametrize("rho_dyn", [1e-6, 0.3])
def test_xl_kkt_matches_oracle(n, m, N, batch, nc, rho_dyn):
    """QDLDLSolver past n + m = 64: rho_dyn 1e-6 keeps rho_dyn ||P||_F inside
    the Neumann range, 0.3 puts every stage past it (the Cholesky of
    I + rho_dyn P with both triangular solves)."""
    from oracle.oracle import OracleKKT
    from pdplqr import BatchedLQRSolver

    p = _problem(n, m, N, batch, nc, 7 * n + m + nc)
    bs = BatchedLQRSolver(n, m, N, batch, solver="kkt", ncs=p["ncs"], rho_dyn=rho_dyn)
    bs.set_model(p["E"], p["c"], p["H"], p["h"], p["D"] if nc else None)
    bs.update_problem_data(p["ws"], p["ys"] if nc else None, p["zs"] if nc else None, p["irho"] if nc else None,
                           sigma=1e-6)
    bs.backward(p["irho"] if nc else None)
    out = np.zeros_like(p["ws"])
    bs.forward(p["x0"], out)
    assert np.all(bs.status() == 0)
    for b in range(batch):
        pm = PackedModel(n, m, N, p["ncs"], p["E"][b], p["c"][b], p["H"][b], p["h"][b],
                         p["D"][b] if nc else np.zeros(0))
        o = OracleKKT(pm, rho_dyn=rho_dyn)
        o.update_problem_data(p["ws"][b], p["ys"][b], p["zs"][b], p["irho"][b], 1e-6)
        o.backward(p["irho"][b])
        assert rel_err(out[b], o.forward(p["x0"][b])) < 1e-8, b
    bs.close()


def test_xl_kkt_x0_accumulates():
    """update_rhs_initial_stage accumulates -S0 x0 on every forward
    (kkt.hpp:207-222): two forwards after one update solve with x0 + x0' and
    report the second call's x0 in ws[0]; the oracle does the same."""
    from oracle.oracle import OracleKKT
    from pdplqr import BatchedLQRSolver

    n, m, N, batch = 60, 20, 4, 2
    p = _problem(n, m, N, batch, 0, 3)
    bs = BatchedLQRSolver(n, m, N, batch, solver="kkt")
    bs.set_model(p["E"], p["c"], p["H"], p["h"])
    bs.update_problem_data(p["ws"], sigma=1e-6)
    bs.backward()
    x1 = 0.5 * p["x0"]
    out0, out1 = np.zeros_like(p["ws"]), np.zeros_like(p["ws"])
    bs.forward(p["x0"], out0)
    bs.forward(x1, out1)
    for b in range(batch):
        pm = PackedModel(n, m, N, p["ncs"], p["E"][b], p["c"][b], p["H"][b], p["h"][b], np.zeros(0))
        o = OracleKKT(pm)
        o.update_problem_data(p["ws"][b], None, None, None, 1e-6)
        o.backward(None)
        r0 = o.forward(p["x0"][b])
        r1 = o.forward(x1[b])
        assert rel_err(out0[b], r0) < 1e-8 and rel_err(out1[b], r1) < 1e-8, b
    bs.close()


@pytest.mark.parametrize("keep", [True, False])
def test_xl_admm_matches_oracle(keep):
    """The ADMM loop over the serial solver at n + m = 70 (k_admm_update_xl:
    a wave per stage, several entries a lane) against the oracle's loop."""
    from oracle.oracle import admm_solve as oracle_admm
    from pdplqr import BatchedLQRSolver
    from pdplqr.model import pack_model, pack_stage_vectors
    from pdplqr.problems import random_model

    models, x0s = [], []
    for b in range(2):
        mod, x0 = random_model(50, 20, 6, seed=950 + b, nc=5, D_kind="ubox")
        for nd in mod.nodes:
            if nd.n_con:
                nd.e_lb[:] = -0.3
                nd.e_ub[:] = 0.3
        models.append(mod)
        x0s.append(x0)
    pms = [pack_model(m) for m in models]
    ncs = [int(x) for x in pms[0].ncs]
    A = {k: np.ascontiguousarray(np.stack([getattr(p, k) for p in pms])) for k in "E c H h D".split()}
    lb = np.stack([np.clip(pack_stage_vectors([nd.e_lb for nd in m.nodes], ncs), -1e20, 1e20) for m in models])
    ub = np.stack([np.clip(pack_stage_vectors([nd.e_ub for nd in m.nodes], ncs), -1e20, 1e20) for m in models])
    x0 = np.ascontiguousarray(np.stack(x0s))
    g = np.random.default_rng(6)
    W, Y = pms[0].h.size, int(sum(ncs))
    ws, ys, zs = 0.1 * g.standard_normal((2, W)), 0.1 * g.standard_normal((2, Y)), 0.1 * g.standard_normal((2, Y))
    rho = np.full(lb.shape, 10.0)
    p = pms[0]
    bs = BatchedLQRSolver(p.n, p.m, p.N, 2, keep_factors=keep, ncs=ncs)
    bs.set_model(A["E"], A["c"], A["H"], A["h"], A["D"])
    w, y, z = ws.copy(), ys.copy(), zs.copy()
    info = bs.admm_solve(x0, np.ascontiguousarray(lb), np.ascontiguousarray(ub), rho, w, y, z, max_iter=15,
                         eps_abs=0.0, eps_rel=0.0)
    assert info["iterations"] == 15 and np.count_nonzero(bs.status()) == 0
    bs.close()
    for b in range(2):
        ow, oy, oz, _ = oracle_admm(pms[b], x0[b], lb[b], ub[b], rho[b], ws[b], ys[b], zs[b], solver="serial",
                                    max_iter=15, eps_abs=0.0, eps_rel=0.0)
        assert rel_err(w[b], ow) < TOL and rel_err(y[b], oy) < TOL and rel_err(z[b], oz) < TOL, b


def test_xl_kkt_admm_matches_oracle():
    """The ADMM loop over the KKT solver at n + m = 70 (the whole backward every
    iteration: no linear-only pass past 12/4) against the oracle's loop."""
    from oracle.oracle import admm_solve as oracle_admm
    from pdplqr import BatchedLQRSolver
    from pdplqr.model import pack_model, pack_stage_vectors
    from pdplqr.problems import random_model

    models, x0s = [], []
    for b in range(2):
        mod, x0 = random_model(50, 20, 5, seed=970 + b, nc=5, D_kind="ubox")
        for nd in mod.nodes:
            if nd.n_con:
                nd.e_lb[:] = -0.3
                nd.e_ub[:] = 0.3
        models.append(mod)
        x0s.append(x0)
    pms = [pack_model(m) for m in models]
    ncs = [int(x) for x in pms[0].ncs]
    A = {k: np.ascontiguousarray(np.stack([getattr(p, k) for p in pms])) for k in "E c H h D".split()}
    lb = np.stack([np.clip(pack_stage_vectors([nd.e_lb for nd in m.nodes], ncs), -1e20, 1e20) for m in models])
    ub = np.stack([np.clip(pack_stage_vectors([nd.e_ub for nd in m.nodes], ncs), -1e20, 1e20) for m in models])
    x0 = np.ascontiguousarray(np.stack(x0s))
    g = np.random.default_rng(8)
    W, Y = pms[0].h.size, int(sum(ncs))
    ws, ys, zs = 0.1 * g.standard_normal((2, W)), 0.1 * g.standard_normal((2, Y)), 0.1 * g.standard_normal((2, Y))
    rho = np.full(lb.shape, 10.0)
    p = pms[0]
    bs = BatchedLQRSolver(p.n, p.m, p.N, 2, solver="kkt", ncs=ncs)
    bs.set_model(A["E"], A["c"], A["H"], A["h"], A["D"])
    w, y, z = ws.copy(), ys.copy(), zs.copy()
    info = bs.admm_solve(x0, np.ascontiguousarray(lb), np.ascontiguousarray(ub), rho, w, y, z, max_iter=12,
                         eps_abs=0.0, eps_rel=0.0)
    assert info["iterations"] == 12 and np.count_nonzero(bs.status()) == 0
    bs.close()
    for b in range(2):
        ow, oy, oz, _ = oracle_admm(pms[b], x0[b], lb[b], ub[b], rho[b], ws[b], ys[b], zs[b], solver="kkt",
                                    max_iter=12, eps_abs=0.0, eps_rel=0.0)
        assert rel_err(w[b], ow) < 1e-8 and rel_err(y[b], oy) < 1e-8 and rel_err(z[b], oz) < 1e-8, b


def test_set_stream_orders_the_model_upload():
    """pdplqr_set_stream: work queued on the old stream (set_model's upload and
    repack) precedes the first launch on the new one.  Before the ordering, a
    solve switched to a fresh stream right after set_model could read a model
    still in flight (seen as spurious failed stages at n + m = 128)."""
    import torch

    from pdplqr import BatchedLQRSolver

    n, m, N, batch = 96, 32, 8, 64
    s = n + m
    E, c, H, h, x0 = random_batch_arrays(n, m, N, batch, 31)
    dev = torch.device("cuda", 0)
    T = {k: torch.from_numpy(v).to(dev) for k, v in dict(E=E, c=c, H=H, h=h, x0=x0).items()}
    ws0 = torch.zeros(batch, N * s + n, dtype=torch.float64, device=dev)
    outs = []
    for switch in (False, True):
        bs = BatchedLQRSolver(n, m, N, batch, keep_factors=True)
        bs.set_model(T["E"], T["c"], T["H"], T["h"])
        st = torch.cuda.Stream(device=dev)
        if switch:
            bs.handle.set_stream(st.cuda_stream)
        out = torch.full_like(ws0, float("nan"))
        with torch.cuda.stream(st):
            bs.update_problem_data(ws0, sigma=1e-6)
            bs.backward()
            bs.forward(T["x0"], out)
        torch.cuda.synchronize()
        assert np.count_nonzero(bs.status()) == 0, switch
        outs.append(out.cpu().numpy())
        bs.close()
    assert np.isfinite(outs[1]).all() and np.array_equal(outs[0], outs[1])


# (n, m, N, batch): element kernels on tiles (n = 20), LDS (n = 50) and the XL
# workspace (n = 80, 100); stage kernels XL throughout
PAR_SHAPES = [(20, 60, 16, 2), (50, 15, 16, 2), (80, 20, 12, 2), (100, 28, 10, 1)]


@pytest.mark.parametrize("n,m,N,batch", PAR_SHAPES)
@pytest.mark.parametrize("condensed", ["CHOLESKY", "LU"])
@pytest.mark.parametrize("ns,seglen", [(3, 0), (2, 2)])
@pytest.mark.parametrize("nc", [0, 3])
def test_xl_parallel_matches_oracle(n, m, N, batch, condensed, ns, seglen, nc):
    from oracle.oracle import OracleParallel
    from pdplqr import BatchedLQRSolver

    p = _problem(n, m, N, batch, nc, 5 * n + m + nc + ns)
    bs = BatchedLQRSolver(n, m, N, batch, solver="parallel", num_segments=ns, keep_factors=True, condensed=condensed,
                          segment_len=seglen, ncs=p["ncs"])
    bs.set_model(p["E"], p["c"], p["H"], p["h"], p["D"] if nc else None)
    rho = (1.0 / p["irho"]) if nc else None
    bs.update_problem_data(p["ws"], p["ys"] if nc else None, p["zs"] if nc else None, p["irho"] if nc else None,
                           sigma=1e-6)
    bs.backward(rho)
    out = np.zeros_like(p["ws"])
    bs.forward(p["x0"], out)
    assert np.all(bs.status() == 0)
    for b in range(batch):
        _, ref = _oracle(p, b, n, m, N)
        assert rel_err(out[b], ref) < TOL, b
        pm = PackedModel(n, m, N, p["ncs"], p["E"][b], p["c"][b], p["H"][b], p["h"][b],
                         p["D"][b] if nc else np.zeros(0))
        o = OracleParallel(pm, ns, True, condensed)
        o.update_problem_data(p["ws"][b], p["ys"][b] if nc else None, p["zs"][b] if nc else None,
                              p["irho"][b] if nc else None, 1e-6)
        o.backward(rho[b] if nc else None)
        assert rel_err(out[b], o.forward(p["x0"][b])) < TOL, b
    # backward_without_factorization (lqr_solver_parallel.hpp:148-154): new linear data
    ws1 = p["ws"] + 0.2 * np.random.default_rng(n).standard_normal(p["ws"].shape)
    bs.update_problem_data(ws1, p["ys"] if nc else None, p["zs"] if nc else None, p["irho"] if nc else None,
                           sigma=1e-6)
    bs.backward_without_factorization(rho)
    out1 = np.zeros_like(out)
    bs.forward(p["x0"], out1)
    for b in range(batch):
        _, ref1 = _oracle(p, b, n, m, N, ws=ws1[b])
        assert rel_err(out1[b], ref1) < TOL, b
    bs.close()


@pytest.mark.parametrize("n,m,N,batch,R,seglen", [(70, 20, 24, 2, 3, 3), (40, 30, 20, 1, 4, 2)])
def test_xl_horizon_shards_match_oracle(n, m, N, batch, R, seglen):
    """Horizon shards (pdplqr_shard_backward / shard_forward) past n + m = 64:
    virtual ranks in one process against the serial oracle (the rank fold by
    the scan form, k_rank_maps_xl for n > 64)."""
    from test_gpu_horizon import _run_virtual

    got, ref = _run_virtual(n, m, N, batch, R, seglen)
    for b in range(batch):
        assert rel_err(got[b], ref[b]) < TOL, b


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_xl_multidev_matches_oracle(devices):
    """A num_devices split past n + m = 64 (n = 70: the rank maps on the XL
    element kernels): factorising backward, then backward_without_factorization
    on new linear data, against the serial oracle."""
    from pdplqr import BatchedLQRSolver

    n, m, N, batch, nc = 70, 20, 18, 2, 3
    p = _problem(n, m, N, batch, nc, 41)
    rho = 1.0 / p["irho"]
    bs = BatchedLQRSolver(n, m, N, batch, solver="parallel", num_segments=2, keep_factors=True, ncs=p["ncs"],
                          devices=devices)
    bs.set_model(p["E"], p["c"], p["H"], p["h"], p["D"])
    bs.update_problem_data(p["ws"], p["ys"], p["zs"], p["irho"], sigma=1e-6)
    bs.backward(rho)
    out = np.zeros_like(p["ws"])
    bs.forward(p["x0"], out)
    assert np.all(bs.status() == 0)
    for b in range(batch):
        assert rel_err(out[b], _oracle(p, b, n, m, N)[1]) < TOL, b
    ws1 = p["ws"] + 0.2 * np.random.default_rng(3).standard_normal(p["ws"].shape)
    bs.update_problem_data(ws1, p["ys"], p["zs"], p["irho"], sigma=1e-6)
    bs.backward_without_factorization(rho)
    out1 = np.zeros_like(out)
    bs.forward(p["x0"], out1)
    for b in range(batch):
        assert rel_err(out1[b], _oracle(p, b, n, m, N, ws=ws1[b])[1]) < TOL, b
    bs.close()


def test_xl_parallel_admm_matches_oracle():
    """The ADMM loop over the PARALLEL solver at n + m = 70 (segment kernels on
    the XL workspace, backward_without_factorization from iteration 2 on)
    against the oracle's loop over its parallel restatement."""
    from oracle.oracle import admm_solve as oracle_admm
    from pdplqr import BatchedLQRSolver
    from pdplqr.model import pack_model, pack_stage_vectors
    from pdplqr.problems import random_model

    models, x0s = [], []
    for b in range(2):
        mod, x0 = random_model(50, 20, 12, seed=990 + b, nc=5, D_kind="ubox")
        for nd in mod.nodes:
            if nd.n_con:
                nd.e_lb[:] = -0.3
                nd.e_ub[:] = 0.3
        models.append(mod)
        x0s.append(x0)
    pms = [pack_model(m) for m in models]
    ncs = [int(x) for x in pms[0].ncs]
    A = {k: np.ascontiguousarray(np.stack([getattr(p, k) for p in pms])) for k in "E c H h D".split()}
    lb = np.stack([np.clip(pack_stage_vectors([nd.e_lb for nd in m.nodes], ncs), -1e20, 1e20) for m in models])
    ub = np.stack([np.clip(pack_stage_vectors([nd.e_ub for nd in m.nodes], ncs), -1e20, 1e20) for m in models])
    x0 = np.ascontiguousarray(np.stack(x0s))
    g = np.random.default_rng(12)
    W, Y = pms[0].h.size, int(sum(ncs))
    ws, ys, zs = 0.1 * g.standard_normal((2, W)), 0.1 * g.standard_normal((2, Y)), 0.1 * g.standard_normal((2, Y))
    rho = np.full(lb.shape, 10.0)
    p = pms[0]
    bs = BatchedLQRSolver(p.n, p.m, p.N, 2, solver="parallel", num_segments=3, condensed="CHOLESKY",
                          keep_factors=True, ncs=ncs)
    bs.set_model(A["E"], A["c"], A["H"], A["h"], A["D"])
    w, y, z = ws.copy(), ys.copy(), zs.copy()
    info = bs.admm_solve(x0, np.ascontiguousarray(lb), np.ascontiguousarray(ub), rho, w, y, z, max_iter=12,
                         eps_abs=0.0, eps_rel=0.0)
    assert info["iterations"] == 12 and np.count_nonzero(bs.status()) == 0
    bs.close()
    for b in range(2):
        ow, oy, oz, _ = oracle_admm(pms[b], x0[b], lb[b], ub[b], rho[b], ws[b], ys[b], zs[b], solver="parallel",
                                    num_segments=3, condensed="CHOLESKY", max_iter=12, eps_abs=0.0, eps_rel=0.0)
        assert rel_err(w[b], ow) < TOL and rel_err(y[b], oy) < TOL and rel_err(z[b], oz) < TOL, b


@pytest.mark.parametrize("keep", [False, True])
def test_xl_state_pivot_stop_follows_eigen_blocked(keep):
    """Eigen's LLT::compute factors orders >= 32 in blocks
    (llt_inplace::blocked: 8 columns below order 128), so a state pivot that
    stops it inside a later block leaves the Schur complement of the finished
    blocks in the later columns -- not their input values.  State 20 of a
    50 / 15 problem is dead: the terminal factor (order 50) stops at 20 (block
    16..23), every stage factor (order 65) at 35 (block 32..39).  The XL
    kernels (xl_llt) against the oracle's restated blocked LLT (1e-9), status
    clean (a zero state pivot is not flagged, as the reference ignores it)."""
    from pdplqr import BatchedLQRSolver
    from psd_models import decoupled_dead_state

    n, m, N, batch, k = 50, 15, 5, 2, 20
    s = n + m
    E, c, H, h, x0 = decoupled_dead_state(n, m, N, batch, 77, k)
    bs = BatchedLQRSolver(n, m, N, batch, keep_factors=keep)
    bs.set_model(E, c, H, h)
    ws = 0.1 * np.random.default_rng(78).standard_normal((batch, N * s + n))
    bs.update_problem_data(ws, sigma=0.0)
    bs.backward()
    out = np.zeros((batch, N * s + n))
    bs.forward(x0, out)
    assert np.all(bs.status() == 0)
    assert np.all(np.isfinite(out))
    for b in range(batch):
        o = OracleSerial(PackedModel(n, m, N, np.zeros(N + 1, dtype=np.int32), E[b], c[b], H[b], h[b], np.zeros(0)))
        o.update_problem_data(ws[b], None, None, None, 0.0)
        o.backward(None)
        assert rel_err(out[b], o.forward(x0[b])) < TOL, b
    bs.close()
