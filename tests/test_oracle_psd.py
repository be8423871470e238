"""The oracle on the semidefinite edge cases (tests/psd_models.py), pinned
against the dense KKT optimum (tests/dense_ref.py): the serial restatement
and the LU condensed system solve them; the CHOLESKY condensed system reports
failure where a boundary value function is singular (condensed_system.hpp:
217-226 returns false), as the reference's does.  sigma = 0, nc = 0."""
import numpy as np
import pytest

from conftest import rel_err
from dense_ref import riccati_optimum
from psd_models import psd_model

from oracle.oracle import OracleParallel, OracleSerial


def _dense(pm, x0):
    ws = np.zeros(pm.N * (pm.n + pm.m) + pm.n)
    return riccati_optimum(pm, x0, ws, np.zeros(0), np.zeros(0), np.zeros(0), np.zeros(0), 0.0)


def _solve(o, pm, x0):
    o.update_problem_data(np.zeros(pm.N * (pm.n + pm.m) + pm.n), None, None, None, 0.0)
    ok = o.backward(None)
    return ok, o.forward(x0)


@pytest.mark.parametrize("kind", ["zero_state_cost", "zero_terminal"])
def test_serial_oracle_semidefinite(kind):
    pm, _, x0 = psd_model(kind)
    _, w = _solve(OracleSerial(pm), pm, x0)
    assert rel_err(w, _dense(pm, x0)) < 1e-9


@pytest.mark.parametrize("kind", ["zero_state_cost", "zero_terminal"])
@pytest.mark.parametrize("ns", [2, 4, 7])
def test_parallel_lu_oracle_semidefinite(kind, ns):
    pm, _, x0 = psd_model(kind)
    ok, w = _solve(OracleParallel(pm, ns, True, "LU"), pm, x0)
    assert ok
    assert rel_err(w, _dense(pm, x0)) < 1e-9


def test_parallel_cholesky_oracle_fails_on_singular_value_function():
    pm, _, x0 = psd_model("zero_state_cost")
    ok, _ = _solve(OracleParallel(pm, 4, True, "CHOLESKY"), pm, x0)
    assert not ok


def test_parallel_cholesky_oracle_zero_terminal_only():
    """Q_N = 0 alone leaves every segment-start value function definite
    (Q_k > 0 before N): CHOLESKY succeeds."""
    pm, _, x0 = psd_model("zero_terminal")
    ok, w = _solve(OracleParallel(pm, 4, True, "CHOLESKY"), pm, x0)
    assert ok
    assert rel_err(w, _dense(pm, x0)) < 1e-9


def test_oracle_eigen_stop_coupled_dead_terminal():
    """Q_N's second pivot is exactly 0 after the first has reduced the trailing
    block (tests/psd_models.py).  The reference's L_N is Eigen's stopped
    factor (original values from column 1 on), so its solve equals the dense
    optimum of the model whose terminal cost is L_N L_N^T -- not of Q_N."""
    from psd_models import eigen_stop_factor

    pm, model, x0 = psd_model("coupled_dead_terminal")
    n, m, N = pm.n, pm.m, pm.N
    s = n + m
    _, w = _solve(OracleSerial(pm), pm, x0)
    QN = pm.H[N * s * s:].reshape(n, n, order="F")
    L = eigen_stop_factor(QN)
    assert abs((L @ L.T)[2, 2] - 1.64) < 1e-15
    H2 = pm.H.copy()
    H2[N * s * s:] = (L @ L.T).ravel(order="F")
    from pdplqr.model import PackedModel

    pm2 = PackedModel(n, m, N, pm.ncs, pm.E, pm.c, H2, pm.h, pm.D)
    assert rel_err(w, _dense(pm2, x0)) < 1e-9
    assert rel_err(w, _dense(pm, x0)) > 1e-6  # the stop changes the answer
