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
