"""The oracle's ADMM outer loop (oracle.admm_solve) pinned by an independent
optimality certificate (CPU).

The ADMM loop is not in the reference (README.md:8), so no reference output
exists for it ("parity unpinned" w.r.t. reference outputs).  Its converged
answer is instead checked against the first-order conditions of the conic LQ
    min sum 1/2 w^T H w + h^T w  s.t. dynamics, x0 fixed, e_lb <= D w <= e_ub
computed by tests/dense_ref.py (dense LAPACK KKT, not a restatement):
  * feasibility: D w within [e_lb, e_ub] up to the tolerance;
  * stationarity: w equals the equality-constrained optimum with linear term
    h + D^T y (the dense KKT solve, sigma = 0, no penalty);
  * complementarity: y_i > 0 only on an active upper bound, y_i < 0 only on an
    active lower bound;
and some constraint is active in every case (else the test would be vacuous).
"""
import numpy as np
import pytest

from conftest import rel_err
from dense_ref import riccati_optimum
from oracle.oracle import admm_solve
from pdplqr.model import PackedModel, initialize_vectors, pack_model, pack_stage_vectors
from pdplqr.problems import quadrotor_model, random_model


def _case(name):
    if name == "quadrotor":
        model, x0 = quadrotor_model(30, nc_on=True)
        x0 = x0.copy()
        x0[2] = -1.0  # start 2 m below the reference height: the thrust bound activates
    else:
        model, x0 = random_model(6, 3, 40, seed=7, nc=3, D_kind="ubox")
        for nd in model.nodes:
            if nd.n_con:
                nd.e_lb[:] = -0.3
                nd.e_ub[:] = 0.3
    pm = pack_model(model)
    ncs = [int(x) for x in pm.ncs]
    lb = pack_stage_vectors([nd.e_lb for nd in model.nodes], ncs)
    ub = pack_stage_vectors([nd.e_ub for nd in model.nodes], ncs)
    return model, pm, x0, np.clip(lb, -1e20, 1e20), np.clip(ub, -1e20, 1e20)


RHO = {"quadrotor": 0.1, "ubox": 10.0}  # fixed rho; 0.1 stalls at 1e-5 on the unstable random dynamics


def _certificate(pm, x0, w, y, lb, ub, tol):
    n, m, N = pm.n, pm.m, pm.N
    s = n + m
    ncs = [int(x) for x in pm.ncs]
    # D w per stage
    dw, doff, yoff = np.zeros(len(y)), 0, 0
    Dt_y = np.zeros(N * s + n)
    for k in range(N + 1):
        nc, dim = ncs[k], (s if k < N else n)
        if nc:
            Dk = pm.D[doff:doff + nc * dim].reshape(nc, dim, order="F")
            dw[yoff:yoff + nc] = Dk @ w[k * s:k * s + dim]
            Dt_y[k * s:k * s + dim] = Dk.T @ y[yoff:yoff + nc]
        doff += nc * dim
        yoff += nc
    assert np.all(dw >= lb - tol) and np.all(dw <= ub + tol), "infeasible"
    active = (np.abs(y) > 1e-6)
    assert active.any(), "no active constraint: vacuous case"
    assert np.all(np.abs(dw[y > 1e-6] - ub[y > 1e-6]) < 10 * tol), "y > 0 on an inactive upper bound"
    assert np.all(np.abs(dw[y < -1e-6] - lb[y < -1e-6]) < 10 * tol), "y < 0 on an inactive lower bound"
    pm2 = PackedModel(n, m, N, np.zeros(N + 1, dtype=np.int32), pm.E, pm.c, pm.H, pm.h + Dt_y, np.zeros(0))
    z0 = np.zeros(0)
    w_kkt = riccati_optimum(pm2, x0, np.zeros(N * s + n), z0, z0, z0, z0, 0.0)
    return rel_err(w, w_kkt)


@pytest.mark.parametrize("solver", ["serial", "parallel", "kkt"])
@pytest.mark.parametrize("name", ["quadrotor", "ubox"])
def test_admm_converges_to_kkt_point(name, solver):
    model, pm, x0, lb, ub = _case(name)
    ny = int(np.sum(pm.ncs))
    rho = np.full(ny, RHO[name])
    kw = {"num_segments": 4} if solver == "parallel" else {}
    w, y, z, info = admm_solve(pm, x0, lb, ub, rho, solver=solver, max_iter=20000, check_every=25, eps_abs=1e-8,
                               eps_rel=1e-8, **kw)
    assert info["converged"], info
    # the KKT-path answer carries the frozen rho_dyn = sigma = 1e-6 regularisation
    # of qdldl_solver.hpp:38-41 -- a 1e-6-level perturbation of the problem
    err = _certificate(pm, x0, w, y, lb, ub, 1e-6)
    assert err < (1e-3 if solver == "kkt" else 1e-6), err


def test_admm_solvers_agree_iteration_by_iteration():
    """Serial and parallel x-updates are the same LQ solve: 60 fixed
    iterations (eps = 0) agree to rounding."""
    model, pm, x0, lb, ub = _case("ubox")
    ny = int(np.sum(pm.ncs))
    rho = np.full(ny, RHO["ubox"])
    a = admm_solve(pm, x0, lb, ub, rho, solver="serial", max_iter=60, eps_abs=0, eps_rel=0)
    b = admm_solve(pm, x0, lb, ub, rho, solver="parallel", max_iter=60, eps_abs=0, eps_rel=0, num_segments=3)
    assert a[3]["iters"] == b[3]["iters"] == 60
    for u, v in zip(a[:3], b[:3]):
        assert rel_err(u, v) < 1e-10


def test_admm_without_constraints_is_one_solve():
    model, x0 = random_model(4, 2, 20, seed=3)
    pm = pack_model(model)
    w, y, z, info = admm_solve(pm, x0, np.zeros(0), np.zeros(0), np.zeros(0))
    assert info["iters"] == 1 and info["converged"]
    ws, ys, zs, _, irho = initialize_vectors(model, 0.1)
    from oracle.oracle import OracleSerial

    o = OracleSerial(pm)
    o.update_problem_data(np.zeros(pm.N * (pm.n + pm.m) + pm.n), None, None, None, 1e-6)
    o.backward(None)
    assert rel_err(w, o.forward(x0)) < 1e-15


def test_adaptive_rho_recovers_a_poor_rho():
    """rho = 0.1 stalls on the unstable ubox case (see RHO); OSQP's adaptive
    rho rule moves it and the run converges to the KKT point."""
    model, pm, x0, lb, ub = _case("ubox")
    rho = np.full(int(np.sum(pm.ncs)), 0.1)
    st = dict(max_iter=3000, check_every=25, eps_abs=1e-8, eps_rel=1e-8)
    _, _, _, fixed = admm_solve(pm, x0, lb, ub, rho, adaptive_rho=False, **st)
    w, y, z, info = admm_solve(pm, x0, lb, ub, rho, adaptive_rho=True, **st)
    assert not fixed["converged"]
    assert info["converged"] and info["rho_updates"] >= 1 and info["rho"][0] > 0.5, info
    assert _certificate(pm, x0, w, y, lb, ub, 1e-6) < 1e-6


def test_adaptive_rho_keeps_rho_when_no_row_is_active():
    """Bounds so loose that no row is ever active: y stays exactly 0 and
    |D^T y| = 0, where OSQP's estimate (normalised by |D^T y| alone) would
    collapse to ~1e-14 and pin rho at its 1e-6 clamp.  The rule
    skips the rescale while |D^T y| <= eps_abs, so rho is untouched."""
    model, pm, x0, lb, ub = _case("ubox")
    ny = int(np.sum(pm.ncs))
    lb, ub = np.full(ny, -1e6), np.full(ny, 1e6)
    rho = np.full(ny, 0.1)
    w, y, z, info = admm_solve(pm, x0, lb, ub, rho, max_iter=100, check_every=5, eps_abs=1e-12, eps_rel=1e-12)
    assert np.all(y == 0.0)
    assert info["rho_updates"] == 0 and np.all(info["rho"] == 0.1), info
