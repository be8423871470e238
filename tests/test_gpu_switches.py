"""The library's runtime switches that have no test of their own elsewhere
(DESIGN.md section 6a lists all seven and where each is tested):

* PDPLQR_NO_X1 -- the one-wave-per-SIMD kernel instances (device_common.hpp
  simd_exclusive) run only when the batch fits the device's SIMDs once; their
  code is the plain instances' own, so every answer is bit-identical with the
  switch on or off (C5-shaped 12/4 batch with four rows per stage: the fused-
  penalty backward and gain rollout, the KKT backward / rollout, the nofact and
  ADMM passes);
* PDPLQR_MD_P2P -- a num_devices handle on distinct devices exchanges its slice
  elements over RCCL; with the switch, by device copies.  devices = [0] (one
  slice, a one-rank communicator) gives the same bits either way.

Both are read when a handle is created, so each mode builds its own handle."""
import numpy as np
import pytest

from conftest import rel_err

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    from pdplqr import device_count

    assert device_count() > 0, "no HIP device visible"


def _c5_like(N, batch, seed):
    from pdplqr.problems import random_batch_arrays

    n, m, nc = 12, 4, 4
    s = n + m
    E, c, H, h, x0 = random_batch_arrays(n, m, N, batch, seed)
    g = np.random.default_rng(seed + 1)
    ncs = np.array([nc] * N + [0], dtype=np.int32)
    D = np.tile(np.concatenate([np.eye(nc, s)[:, j] for j in range(s)]), (batch, N))  # u-box rows, column-major
    ny = nc * N
    ws = g.standard_normal((batch, N * s + n))
    ys, zs = g.standard_normal((batch, ny)), g.standard_normal((batch, ny))
    rho = 0.1 + g.random((batch, ny))
    return (n, m, N, batch, ncs), (E, c, H, h, D, x0), (ws, ys, zs, rho)


def _solve_all(shape, model, vecs):
    """Every batch kernel family that has an X1 instance, on one data set."""
    from pdplqr import BatchedLQRSolver

    n, m, N, batch, ncs = shape
    E, c, H, h, D, x0 = model
    ws, ys, zs, rho = vecs
    s = n + m
    out = {}
    for solver, keep in (("serial", False), ("serial", True), ("kkt", False)):
        bs = BatchedLQRSolver(n, m, N, batch, solver=solver, ncs=ncs, keep_factors=keep)
        bs.set_model(E, c, H, h, D)
        bs.update_problem_data(ws, ys, zs, 1.0 / rho, sigma=1e-6)
        bs.backward(1.0 / rho if solver == "kkt" else rho)
        w = np.zeros((batch, N * s + n))
        bs.forward(x0, w)
        out[(solver, keep, "solve")] = w
        if solver == "serial" and keep:
            bs.update_problem_data(ws * 0.5, ys, zs, 1.0 / rho, sigma=1e-6)
            bs.backward_without_factorization(rho)
            w2 = np.zeros_like(w)
            bs.forward(x0, w2)
            out[(solver, keep, "nofact")] = w2
        assert np.all(bs.status() == 0)
        lb, ub = -0.5 * np.ones_like(rho), 0.5 * np.ones_like(rho)
        wa, ya, za = np.zeros_like(ws), np.zeros_like(ys), np.zeros_like(zs)
        bs.admm_solve(x0, lb, ub, np.ones_like(rho), wa, ya, za, max_iter=12, check_every=4, eps_abs=0.0, eps_rel=0.0)
        out[(solver, keep, "admm")] = np.concatenate([wa, ya, za], axis=1)
        bs.close()
    return out


def test_one_wave_per_simd_instances_are_bit_identical(monkeypatch):
    shape, model, vecs = _c5_like(37, 64, 4100)
    on = _solve_all(shape, model, vecs)
    monkeypatch.setenv("PDPLQR_NO_X1", "1")
    off = _solve_all(shape, model, vecs)
    for k in on:
        assert np.array_equal(on[k], off[k]), k


def test_md_p2p_exchange_equals_rccl(monkeypatch):
    from oracle.oracle import OracleSerial
    from pdplqr import BatchedLQRSolver
    from pdplqr.model import PackedModel
    from pdplqr.problems import random_batch_arrays

    n, m, N, batch = 6, 3, 45, 2
    s = n + m
    E, c, H, h, x0 = random_batch_arrays(n, m, N, batch, 4200)
    ws = np.random.default_rng(4201).standard_normal((batch, N * s + n))
    outs = []
    for p2p in (False, True):
        if p2p:
            monkeypatch.setenv("PDPLQR_MD_P2P", "1")
        bs = BatchedLQRSolver(n, m, N, batch, solver="parallel", num_segments=3, devices=[0])
        bs.set_model(E, c, H, h)
        bs.update_problem_data(ws, sigma=1e-6)
        bs.backward()
        out = np.zeros((batch, N * s + n))
        bs.forward(x0, out)
        assert np.all(bs.status() == 0)
        outs.append(out)
        bs.close()
    assert np.array_equal(outs[0], outs[1])
    for b in range(batch):
        o = OracleSerial(PackedModel(n, m, N, np.zeros(N + 1, dtype=np.int32), E[b], c[b], H[b], h[b], np.zeros(0)))
        o.update_problem_data(ws[b], None, None, None, 1e-6)
        o.backward(None)
        assert rel_err(outs[0][b], o.forward(x0[b])) < 1e-9, b
