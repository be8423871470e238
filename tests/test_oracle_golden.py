"""The CPU oracle (oracle/pdplqr_oracle.c) against the golden fixtures.

Pins the oracle before it is trusted as the GPU parity checker: serial,
parallel (LU and CHOLESKY condensed systems, several segment counts) and the
QDLDL-path restatement, each against independent dense solves
(tests/golden/make_golden.py).  Tolerance: 1e-9 relative (fp64 on both sides;
observed ~1e-14), 1e-8 for the KKT path (condition ~1/rho_dyn).
"""
import numpy as np
import pytest

from conftest import golden_names, load_golden, rel_err, u_parts

from oracle.oracle import OracleKKT, OracleParallel, OracleSerial, segmentation

NAMES = golden_names()


def _run(o, d):
    o.update_problem_data(d["ws"], d["ys"], d["zs"], d["inv_rho"], float(d["sigma"]))
    o.backward(d["rho"])
    return o.forward(d["x0"])


@pytest.mark.parametrize("name", NAMES)
def test_serial_vs_dense(name):
    pm, d = load_golden(name)
    o = OracleSerial(pm)
    w = _run(o, d)
    assert rel_err(w, d["w_riccati"]) < 1e-9
    assert rel_err(u_parts(w, pm.n, pm.m, pm.N), u_parts(d["w_riccati"], pm.n, pm.m, pm.N)) < 1e-9
    for i, k in enumerate(d["P_k"]):
        P, p = o.value_function(int(k))
        assert rel_err(P, d["P"][i]) < 1e-9
        assert rel_err(p, d["p"][i]) < 1e-8


@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("condensed", ["LU", "CHOLESKY"])
@pytest.mark.parametrize("ns", [2, 4, 8])
def test_parallel_vs_dense(name, condensed, ns):
    pm, d = load_golden(name)
    ok, _, _ = segmentation(pm.N, ns, True)
    if not ok:
        pytest.skip("segmentation yields an empty segment")
    o = OracleParallel(pm, ns, True, condensed)
    w = _run(o, d)
    assert rel_err(w, d["w_riccati"]) < 1e-9


@pytest.mark.parametrize("name", [n for n in NAMES if "w_qdldl" in np.load(f"tests/golden/{n}.npz").files])
def test_kkt_vs_qdldl_equivalent(name):
    pm, d = load_golden(name)
    o = OracleKKT(pm)
    o.update_problem_data(d["ws"], d["ys"], d["zs"], d["inv_rho"], float(d["sigma"]))
    o.backward(d["inv_rho"])
    w = o.forward(d["x0"])
    assert rel_err(w, d["w_qdldl"]) < 1e-8
    # QDLDL != Riccati by O(rho_dyn): 1e-7 .. 1e-4 relative
    assert 1e-9 < rel_err(w, d["w_riccati"]) < 1e-3


def test_example_known_answer():
    """Quadrotor KAT: serial/parallel u0 and x_N[2]."""
    pm, d = load_golden("quadrotor_N100")
    w = _run(OracleSerial(pm), d)
    u0 = np.array([-2.8980566697, 2.8980566697, -2.8980566697, 2.8980566697])
    assert np.allclose(w[:4], u0, rtol=0, atol=5e-10)
    assert abs(w[100 * 16 + 2] - 0.9999999000) < 5e-10
    wp = _run(OracleParallel(pm, 4, True, "CHOLESKY"), d)
    assert np.allclose(wp[:4], u0, rtol=0, atol=5e-10)
    ok = OracleKKT(pm)
    ok.update_problem_data(d["ws"], d["ys"], d["zs"], d["inv_rho"], float(d["sigma"]))
    ok.backward(d["inv_rho"])
    wk = ok.forward(d["x0"])
    assert abs(wk[0] - (-2.8980026778)) < 5e-9


def test_segmentation_kat():
    """lqr_solver_parallel.hpp:64-88 (alpha = 1.55)."""
    ok, st, ln = segmentation(100, 4, True)
    assert ok and list(ln) == [21, 21, 21, 37] and list(st) == [0, 21, 42, 63]
    ok, st, ln = segmentation(1024, 8, True)
    assert ok and list(ln) == [119] * 7 + [191]
    ok, st, ln = segmentation(100, 4, False)
    assert ok and list(ln) == [25, 25, 25, 25]
    ok, _, _ = segmentation(3, 4, True)  # N < ns + 0.55: an empty segment
    assert not ok


def test_backward_without_factorization_matches_refactor():
    """After a full backward, changing only the linear data (h via w-bar, y, z)
    and calling backward_without_factorization equals a fresh full solve
    (lqr_solver.hpp:65-70)."""
    pm, d = load_golden("random_n12_m4_N64_nc4")
    o = OracleSerial(pm)
    _run(o, d)
    g = np.random.default_rng(0)
    ws2 = d["ws"] + 0.1 * g.standard_normal(d["ws"].shape)
    zs2 = d["zs"] + 0.1 * g.standard_normal(d["zs"].shape)
    o.update_problem_data(ws2, d["ys"], zs2, d["inv_rho"], float(d["sigma"]))
    # H~ is reset by update_problem_data and must not get rho D^T D again
    o.backward_without_factorization(d["rho"])
    w1 = o.forward(d["x0"])
    f = OracleSerial(pm)
    f.update_problem_data(ws2, d["ys"], zs2, d["inv_rho"], float(d["sigma"]))
    f.backward(d["rho"])
    w2 = f.forward(d["x0"])
    assert rel_err(w1, w2) < 1e-12
    for condensed in ["LU", "CHOLESKY"]:
        op = OracleParallel(pm, 4, True, condensed)
        _run(op, d)
        op.update_problem_data(ws2, d["ys"], zs2, d["inv_rho"], float(d["sigma"]))
        op.backward_without_factorization(d["rho"])
        assert rel_err(op.forward(d["x0"]), w2) < 1e-9
