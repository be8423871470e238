"""GPU parity of the serial solver for stage sizes 32 < n + m <= 64
(csrc/kernels_big.hip: one 256-thread block per problem, LDS-resident stage
matrices) against the CPU oracle, which is size-generic like the reference's
dynamic-Eigen kernels (lqr_kernel.hpp:104-147).

Covers backward with and without kept factors, forward, the value function,
backward_without_factorization, constrained stages (rho penalty), the status
flag of an indefinite stage, the ADMM loop over the serial solver, and the
shape limits of the three solvers.  Tolerance
1e-9 relative (fp64, different summation order), as tests/test_gpu_serial.py.
All calls go through the C ABI (libpdplqr.so).
"""
import numpy as np
import pytest

from conftest import rel_err, u_parts
from oracle.oracle import OracleSerial
from oracle.oracle import admm_solve as oracle_admm
from pdplqr.model import PackedModel, pack_model, pack_stage_vectors
from pdplqr.problems import random_batch_arrays, random_model

pytestmark = pytest.mark.gpu

TOL = 1e-9

# (24, 16): the one-wave 3 x 3 register-tile backward (k_riccati_bwd_fast<3, 24, 16>)
SHAPES = [(30, 10, 12, 3), (40, 24, 6, 2), (33, 1, 9, 2), (1, 40, 5, 2), (20, 13, 15, 3), (48, 16, 4, 2),
          (24, 16, 21, 3), (24, 16, 2, 2)]


@pytest.fixture(scope="module", autouse=True)
def _device():
    from pdplqr import device_count

    assert device_count() > 0, "no HIP device visible: GPU tests must run on an MI355X"


def _oracle(n, m, N, E, c, H, h, ws0, x0, ws1=None):
    pm = PackedModel(n, m, N, np.zeros(N + 1, dtype=np.int32), E, c, H, h, np.zeros(0))
    o = OracleSerial(pm)
    o.update_problem_data(ws0, None, None, None, 1e-6)
    o.backward(None)
    if ws1 is not None:
        o.update_problem_data(ws1, None, None, None, 1e-6)
        o.backward_without_factorization(None)
    return o, o.forward(x0)


@pytest.mark.parametrize("keep", [True, False])
@pytest.mark.parametrize("n,m,N,batch", SHAPES)
def test_big_serial_matches_oracle(n, m, N, batch, keep):
    from pdplqr import BatchedLQRSolver

    E, c, H, h, x0 = random_batch_arrays(n, m, N, batch, 700 + n + m)
    s = n + m
    ws0 = 0.1 * np.random.default_rng(n).standard_normal((batch, N * s + n))
    bs = BatchedLQRSolver(n, m, N, batch, keep_factors=keep)
    bs.set_model(E, c, H, h)
    bs.update_problem_data(ws0, sigma=1e-6)
    bs.backward()
    out = np.zeros_like(ws0)
    bs.forward(x0, out)
    assert np.all(bs.status() == 0)
    for b in range(batch):
        o, ref = _oracle(n, m, N, E[b], c[b], H[b], h[b], ws0[b], x0[b])
        assert rel_err(out[b], ref) < TOL, b
        assert rel_err(u_parts(out[b], n, m, N), u_parts(ref, n, m, N)) < 1e-6
        if keep:
            for k in (0, N // 2, N):
                P, p = bs.value_function(b, k)
                Po, po = o.value_function(k)
                assert rel_err(P, Po) < TOL and rel_err(p, po) < 1e-8, (b, k)
    if keep:  # lqr_solver.hpp:65-70 with new linear data
        ws1 = ws0 + 0.2 * np.random.default_rng(n + 1).standard_normal(ws0.shape)
        bs.update_problem_data(ws1, sigma=1e-6)
        bs.backward_without_factorization()
        out1 = np.zeros_like(ws0)
        bs.forward(x0, out1)
        for b in range(batch):
            _, ref1 = _oracle(n, m, N, E[b], c[b], H[b], h[b], ws0[b], x0[b], ws1[b])
            assert rel_err(out1[b], ref1) < TOL, b
    bs.close()


def test_big_constrained_model_matches_oracle():
    """rho-penalised stages (k_penalty) feeding the big backward, model-level API."""
    from pdplqr import LQRSolver
    from pdplqr.problems import random_admm_vectors

    model, x0 = random_model(28, 9, 14, seed=5, nc=6)
    pm = pack_model(model)
    ws, ys, zs, rho, irho = random_admm_vectors(model, seed=2)
    sol = LQRSolver(model)
    sol.update_problem_data(ws, ys, zs, irho, 1e-6)
    sol.backward(rho)
    out = [w.copy() for w in ws]
    sol.forward(x0, out)
    assert sol.status() == 0
    flat = lambda v: np.concatenate([np.asarray(a, dtype=np.float64).ravel() for a in v])
    o = OracleSerial(pm)
    o.update_problem_data(flat(ws), flat(ys), flat(zs), flat(irho), 1e-6)
    o.backward(flat(rho))
    assert rel_err(np.concatenate(out), o.forward(x0)) < TOL


@pytest.mark.parametrize("n,m", [(30, 6), (24, 16)])
@pytest.mark.parametrize("keep", [True, False])
def test_big_non_spd_sets_status_flag(keep, n, m):
    """(24, 16): k_riccati_bwd_fast<3> (keep) and the value-form k_riccati_bwd_vf3."""
    from pdplqr import BatchedLQRSolver

    N, batch = 10, 3
    E, c, H, h, x0 = random_batch_arrays(n, m, N, batch, 3)
    s = n + m
    H = H.copy()
    H[1, 7 * s * s:8 * s * s] = -np.eye(s).reshape(-1)  # stage 7 of problem 1 indefinite
    bs = BatchedLQRSolver(n, m, N, batch, keep_factors=keep)
    bs.set_model(E, c, H, h)
    bs.update_problem_data(np.zeros((batch, N * s + n)), sigma=0.0)
    bs.backward()
    st = bs.status()
    assert st[0] == 0 and st[2] == 0
    if keep:  # the full factorisation (k_riccati_bwd_big) fails at the indefinite stage itself
        assert st[1] == 7 + 1
    else:
        # the value form (kernels_wide.hip, no factor cache) eliminates only the
        # u pivots: it flags where a control pivot or a value diagonal goes bad,
        # which the indefinite stage 7 reaches at an earlier stage (DESIGN.md
        # section 2, status semantics of the value-form kernels)
        assert 1 <= st[1] <= 7 + 1
    bs.close()


def test_big_admm_serial_matches_oracle():
    from pdplqr import BatchedLQRSolver

    models, x0s = [], []
    for b in range(2):
        mod, x0 = random_model(26, 8, 12, seed=900 + b, nc=5, D_kind="ubox")
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
    g = np.random.default_rng(4)
    W, Y = pms[0].h.size, int(sum(ncs))
    ws, ys, zs = 0.1 * g.standard_normal((2, W)), 0.1 * g.standard_normal((2, Y)), 0.1 * g.standard_normal((2, Y))
    rho = np.full(lb.shape, 10.0)
    p = pms[0]
    bs = BatchedLQRSolver(p.n, p.m, p.N, 2, keep_factors=True, ncs=ncs)
    bs.set_model(A["E"], A["c"], A["H"], A["h"], A["D"])
    w, y, z = ws.copy(), ys.copy(), zs.copy()
    info = bs.admm_solve(x0, np.ascontiguousarray(lb), np.ascontiguousarray(ub), rho, w, y, z, max_iter=25,
                         eps_abs=0.0, eps_rel=0.0)
    assert info["iterations"] == 25 and np.count_nonzero(bs.status()) == 0
    bs.close()
    for b in range(2):
        ow, oy, oz, _ = oracle_admm(pms[b], x0[b], lb[b], ub[b], rho[b], ws[b], ys[b], zs[b], solver="serial",
                                    max_iter=25, eps_abs=0.0, eps_rel=0.0)
        assert rel_err(w[b], ow) < TOL and rel_err(y[b], oy) < TOL and rel_err(z[b], oz) < TOL, b


def test_big_shape_limits():
    """32 < n + m <= 64 runs on every solver (kernels_big.hip, kernels_wide.hip;
    tests/test_gpu_wide.py); 64 < n + m <= 256 as well (kernels_xl.hip,
    kernels_xl_par.hip, tests/test_gpu_xl.py); past that every solver refuses."""
    from pdplqr import BatchedLQRSolver, PdplqrError

    for solver in ("serial", "parallel", "kkt"):
        BatchedLQRSolver(30, 10, 8, 1, solver=solver, num_segments=2).close()
        with pytest.raises(PdplqrError):
            BatchedLQRSolver(200, 57, 4, 1, solver=solver, num_segments=2)
        BatchedLQRSolver(50, 15, 4, 1, solver=solver, num_segments=2).close()
