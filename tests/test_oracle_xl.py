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
