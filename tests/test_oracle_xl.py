"""The oracle's restatements past n + m = 64 (test infrastructure for
tests/test_gpu_xl.py): OracleSerial, OracleParallel (both condensed forms) and
OracleKKT against the independent dense solves of tests/dense_ref.py on small
horizons at s = 80-128 (the golden-vector pinning of tests/test_golden.py does
not reach these sizes)."""
import numpy as np
import pytest

from conftest import rel_err
from dense_ref import qdldl_equivalent, riccati_optimum
from oracle.oracle import OracleKKT, OracleParallel, OracleSerial
from pdplqr.model import PackedModel
from pdplqr.problems import random_batch_arrays


def _case(n, m, N, nc, seed):
    E, c, H, h, x0 = random_batch_arrays(n, m, N, 1, seed)
    s = n + m
    g = np.random.default_rng(seed + 1)
    ncs = np.full(N + 1, nc, dtype=np.int32)
    D = np.concatenate([g.standard_normal(nc * dk) for dk in [s] * N + [n]]) if nc else np.zeros(0)
    ny = int(ncs.sum())
    pm = PackedModel(n, m, N, ncs, E[0], c[0], H[0], h[0], D)
    ws = 0.1 * g.standard_normal(N * s + n)
    ys, zs, irho = g.standard_normal(ny), g.standard_normal(ny), 0.05 + g.random(ny)
    return pm, x0[0], ws, ys, zs, irho


@pytest.mark.parametrize("n,m,N,nc", [(60, 20, 5, 0), (100, 28, 3, 3)])
def test_oracle_serial_and_parallel_xl_match_dense(n, m, N, nc):
    pm, x0, ws, ys, zs, irho = _case(n, m, N, nc, 11 * n + m)
    a = (ys, zs, irho) if nc else (None, None, None)
    rho = 1.0 / irho if nc else None
    ref = riccati_optimum(pm, x0, ws, ys if nc else np.zeros(0), zs if nc else np.zeros(0),
                          irho if nc else np.zeros(0), rho if nc else np.zeros(0), 1e-6)
    o = OracleSerial(pm)
    o.update_problem_data(ws, *a, 1e-6)
    o.backward(rho)
    assert rel_err(o.forward(x0), ref) < 1e-9
    for cond in ("CHOLESKY", "LU"):
        op = OracleParallel(pm, 2, True, cond)
        op.update_problem_data(ws, *a, 1e-6)
        op.backward(rho)
        assert rel_err(op.forward(x0), ref) < 1e-9, cond


@pytest.mark.parametrize("rho_dyn", [1e-6, 0.3])
def test_oracle_kkt_xl_matches_dense(rho_dyn):
    pm, x0, ws, ys, zs, irho = _case(50, 20, 4, 3, 5)
    o = OracleKKT(pm, rho_dyn=rho_dyn)
    o.update_problem_data(ws, ys, zs, irho, 1e-6)
    o.backward(irho)
    ref = qdldl_equivalent(pm, x0, ws, ys, zs, irho, 1e-6, rho_dyn=rho_dyn)
    assert rel_err(o.forward(x0), ref) < 1e-9


def _eigen_blocked_stop(Q):
    """numpy restatement of Eigen's llt_inplace<Lower>::blocked for order >= 32
    (block 8 below order 128): A11 left-looking, A21 <- A21 A11^{-T}, A22 -= A21
    A21^T; a pivot <= 0 in A11 returns with the later columns at the Schur
    complement of the finished blocks."""
    n = Q.shape[0]
    bs = max(8, min(128, (n // 8 // 16) * 16))
    A = np.tril(np.array(Q, dtype=np.float64))
    for k0 in range(0, n, bs):
        b = min(bs, n - k0)
        for kk in range(b):
            kg = k0 + kk
            x = A[kg, kg] - A[kg, k0:kg] @ A[kg, k0:kg]
            if x <= 0.0:
                return A
            A[kg, kg] = np.sqrt(x)
            A[kg + 1:k0 + b, kg] = (A[kg + 1:k0 + b, kg] - A[kg + 1:k0 + b, k0:kg] @ A[kg, k0:kg]) / A[kg, kg]
        A[k0 + b:, k0:k0 + b] = np.linalg.solve(A[k0:k0 + b, k0:k0 + b], A[k0 + b:, k0:k0 + b].T).T
        A[k0 + b:, k0 + b:] -= np.tril(A[k0 + b:, k0:k0 + b] @ A[k0 + b:, k0:k0 + b].T)
    return A


def test_oracle_llt_stop_is_eigen_blocked():
    """the oracle's llt_lower restates Eigen's blocked LLT from order
    32 on.  A dead state 20 of order 50 stops it in the block 16..23: the
    terminal value function P_N = L_N L_N^T of the oracle equals the blocked
    restatement's (and differs from the unblocked stop's)."""
    from psd_models import decoupled_dead_state, eigen_stop_factor

    n, m, N, k = 50, 15, 3, 20
    s = n + m
    E, c, H, h, x0 = decoupled_dead_state(n, m, N, 1, 77, k)
    o = OracleSerial(PackedModel(n, m, N, np.zeros(N + 1, dtype=np.int32), E[0], c[0], H[0], h[0], np.zeros(0)))
    o.update_problem_data(np.zeros(N * s + n), None, None, None, 0.0)
    o.backward(None)
    PN, _ = o.value_function(N)
    QN = H[0, N * s * s:].reshape(n, n, order="F")
    Lb, Lu = _eigen_blocked_stop(QN), eigen_stop_factor(QN)
    assert np.abs(PN - Lb @ Lb.T).max() < 1e-12
    assert np.abs(PN - Lu @ Lu.T).max() > 1e-3
