"""GPU parity of the QDLDLSolver path (kkt.hip) against the CPU oracle's
restatement of kkt.hpp + QDLDL (oracle/pdplqr_oracle.c) and the golden
QDLDL-equivalent fixtures (dense KKT solve, tests/golden/make_golden.py).

Tolerance: 1e-8 relative on the full primal trajectory (the KKT system is
conditioned ~1/rho_dyn; the oracle-vs-dense pin uses the same bound), and
u* to 1e-6 (north_star).  The GPU path factors the same matrix in QDLDL's
elimination order (all primal pivots first, then the dual groups) with a
block Cholesky of the condensed dual system.
"""
import numpy as np
import pytest

from conftest import golden_names, load_golden, rel_err, u_parts

pytestmark = pytest.mark.gpu

TOL = 1e-8


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    from pdplqr import device_count

    assert device_count() > 0, "no HIP device visible: GPU tests must run on an MI355X"


def _lists(pm, d):
    from pdplqr.model import unpack_model, unpack_ws

    model = unpack_model(pm)
    n, m, N = pm.n, pm.m, pm.N
    ws = unpack_ws(d["ws"], n, m, N)
    off = np.concatenate([[0], np.cumsum(pm.ncs)])
    cut = lambda v: [v[off[k]:off[k + 1]] for k in range(N + 1)]
    return model, ws, cut(d["ys"]), cut(d["zs"]), cut(d["rho"]), cut(d["inv_rho"])


def _oracle(pm, d, x0=None, forwards=1):
    from oracle.oracle import OracleKKT

    o = OracleKKT(pm)
    o.update_problem_data(d["ws"], d["ys"], d["zs"], d["inv_rho"], float(d["sigma"]))
    o.backward(d["inv_rho"])
    w = None
    for _ in range(forwards):
        w = o.forward(d["x0"] if x0 is None else x0)
    return w


@pytest.mark.parametrize("name", golden_names())
def test_qdldl_solver_matches_oracle(name):
    from pdplqr import QDLDLSolver

    pm, d = load_golden(name)
    model, ws, ys, zs, rho, irho = _lists(pm, d)
    sol = QDLDLSolver(model)
    sol.update_problem_data(ws, ys, zs, irho, float(d["sigma"]))
    sol.backward(irho)
    out = [w.copy() for w in ws]
    sol.forward(d["x0"], out)
    w = np.concatenate(out)
    wo = _oracle(pm, d)
    n, m, N = pm.n, pm.m, pm.N
    assert sol.status() == 0
    assert rel_err(w, wo) < TOL
    assert rel_err(u_parts(w, n, m, N), u_parts(wo, n, m, N)) < 1e-6
    if "w_qdldl" in d:
        assert rel_err(w, d["w_qdldl"]) < TOL


def test_qdldl_known_answer():
    """Quadrotor example (lqr_example.cpp): QDLDL u0[0]."""
    from pdplqr import QDLDLSolver

    pm, d = load_golden("quadrotor_N100")
    model, ws, ys, zs, rho, irho = _lists(pm, d)
    sol = QDLDLSolver(model)
    sol.update_problem_data(ws, ys, zs, irho, float(d["sigma"]))
    sol.backward(irho)
    out = [w.copy() for w in ws]
    sol.forward(d["x0"], out)
    assert abs(out[0][0] - (-2.8980026778)) < 5e-9


def test_forward_accumulates_initial_stage_rhs():
    """update_rhs_initial_stage adds -S0 x0, -A0 x0 into the stored rhs on
    every forward (kkt.hpp:207-222): a second forward without a new
    update_problem_data solves a different system -- as the reference does."""
    from pdplqr import QDLDLSolver

    pm, d = load_golden("random_n12_m4_N64_nc4")
    model, ws, ys, zs, rho, irho = _lists(pm, d)
    sol = QDLDLSolver(model)
    sol.update_problem_data(ws, ys, zs, irho, float(d["sigma"]))
    sol.backward(irho)
    out = [w.copy() for w in ws]
    sol.forward(d["x0"], out)
    sol.forward(d["x0"], out)
    w2 = np.concatenate(out)
    wo2 = _oracle(pm, d, forwards=2)
    assert rel_err(w2, wo2) < TOL
    assert rel_err(w2, _oracle(pm, d)) > 1e-6  # really a different answer


def test_refactor_with_new_inv_rho():
    """backward re-writes -inv_rho on the y diagonal and refactors
    (qdldl_solver.hpp:88-109); the rest of the matrix stays frozen."""
    from pdplqr import QDLDLSolver

    pm, d = load_golden("ubox_n12_m4_N48_nc4")
    model, ws, ys, zs, rho, irho = _lists(pm, d)
    sol = QDLDLSolver(model)
    g = np.random.default_rng(3)
    for it in range(3):
        ir = [v * (0.5 + g.random(v.shape)) for v in irho]
        sol.update_problem_data(ws, ys, zs, ir, float(d["sigma"]))
        sol.backward(ir)
        out = [w.copy() for w in ws]
        sol.forward(d["x0"], out)
        d2 = dict(d)
        d2["inv_rho"] = np.concatenate(ir)
        assert rel_err(np.concatenate(out), _oracle(pm, d2)) < TOL, it


@pytest.mark.parametrize("n,m,N,batch,nc", [(12, 4, 64, 5, 4), (4, 2, 33, 3, 2), (6, 3, 20, 2, 0), (12, 4, 3, 2, 4),
                                          (20, 6, 10, 2, 5)])
def test_batched_kkt_matches_oracle(n, m, N, batch, nc):
    from oracle.oracle import OracleKKT
    from pdplqr import BatchedLQRSolver
    from pdplqr.model import PackedModel
    from pdplqr.problems import random_batch_arrays

    E, c, H, h, x0 = random_batch_arrays(n, m, N, batch, 7 * n + m + nc)
    s = n + m
    g = np.random.default_rng(11 + nc)
    ncs = np.full(N + 1, nc, dtype=np.int32)
    dims = [s] * N + [n]
    D = np.concatenate([g.standard_normal((batch, nc * dk)) for dk in dims], axis=1) if nc else np.zeros((batch, 0))
    ny = int(ncs.sum())
    ws = g.standard_normal((batch, N * s + n))
    ys, zs = g.standard_normal((batch, ny)), g.standard_normal((batch, ny))
    irho = 0.05 + g.random((batch, ny))
    bs = BatchedLQRSolver(n, m, N, batch, solver="kkt", ncs=ncs)
    bs.set_model(E, c, H, h, D if nc else None)
    bs.update_problem_data(ws, ys if nc else None, zs if nc else None, irho if nc else None, sigma=1e-6)
    bs.backward(irho if nc else None)
    out = np.zeros((batch, N * s + n))
    bs.forward(x0, out)
    assert np.all(bs.status() == 0)
    for b in range(batch):
        pm = PackedModel(n, m, N, ncs, E[b], c[b], H[b], h[b], D[b] if nc else np.zeros(0))
        o = OracleKKT(pm)
        o.update_problem_data(ws[b], ys[b], zs[b], irho[b], 1e-6)
        o.backward(irho[b])
        assert rel_err(out[b], o.forward(x0[b])) < TOL, b


@pytest.mark.parametrize("n,m,N,batch,nc0", [(12, 4, 40, 3, 3), (5, 3, 17, 2, 3), (12, 4, 24, 2, 8)])
def test_batched_kkt_varying_constraints(n, m, N, batch, nc0):
    """Per-stage constraint counts (kkt.hpp: ncs from time_step, lqr_model.hpp:87)
    vary 0..4 and the terminal has its own: exercises the y offsets of the
    16-wide tile path (dual groups of mixed size, group 0 possibly empty).
    nc0 = 8 with n = 12: every dual group still fits 16, but stage 0's y columns
    do not fit beside lambda_1's in the coupling tile G_0 (kkt.hip PPK), so the
    build takes the P = 32 kernels."""
    from oracle.oracle import OracleKKT
    from pdplqr import BatchedLQRSolver
    from pdplqr.model import PackedModel
    from pdplqr.problems import random_batch_arrays

    E, c, H, h, x0 = random_batch_arrays(n, m, N, batch, 31 * n + N)
    s = n + m
    g = np.random.default_rng(5 + N)
    ncs = g.integers(0, 5, size=N + 1).astype(np.int32)
    ncs[0] = nc0
    dims = [s] * N + [n]
    D = np.concatenate([g.standard_normal((batch, int(ncs[k]) * dims[k])) for k in range(N + 1)], axis=1)
    ny = int(ncs.sum())
    ws = g.standard_normal((batch, N * s + n))
    ys, zs = g.standard_normal((batch, ny)), g.standard_normal((batch, ny))
    irho = 0.05 + g.random((batch, ny))
    bs = BatchedLQRSolver(n, m, N, batch, solver="kkt", ncs=ncs)
    bs.set_model(E, c, H, h, D)
    bs.update_problem_data(ws, ys, zs, irho, sigma=1e-6)
    bs.backward(irho)
    out = np.zeros((batch, N * s + n))
    bs.forward(x0, out)
    assert np.all(bs.status() == 0)
    for b in range(batch):
        pm = PackedModel(n, m, N, ncs, E[b], c[b], H[b], h[b], D[b])
        o = OracleKKT(pm)
        o.update_problem_data(ws[b], ys[b], zs[b], irho[b], 1e-6)
        o.backward(irho[b])
        assert rel_err(out[b], o.forward(x0[b])) < TOL, b


def test_kkt_protocol():
    from pdplqr import BatchedLQRSolver, PdplqrError

    bs = BatchedLQRSolver(4, 2, 5, 1, solver="kkt")
    with pytest.raises(PdplqrError):
        bs.backward_without_factorization()  # QDLDLSolver has none
    with pytest.raises(PdplqrError):
        bs.forward(np.zeros((1, 4)), np.zeros((1, 5 * 6 + 4)))  # before backward


@pytest.mark.parametrize("N", [1, 2, 3, 4, 65, 200])
def test_twisted_ldl_equals_riccati_order(N, monkeypatch):
    """P = 16 (12/4, nc = 4): QDLDL's natural-order elimination on the GPU
    (PDPLQR_KKT_LDL=1: the two-wave twisted block factorisation and solve,
    k_kkt_factor16_tw / k_kkt_solve2_16_tw) and the default Riccati-order
    elimination of the same KKT matrix (kkt_riccati.hip) agree to 1e-10 and
    each matches the oracle to 1e-8; short horizons put the twist's middle
    group at 0 and 1."""
    from oracle.oracle import OracleKKT
    from pdplqr import BatchedLQRSolver
    from pdplqr.model import PackedModel
    from pdplqr.problems import random_batch_arrays

    n, m, nc, batch = 12, 4, 4, 6
    s = n + m
    E, c, H, h, x0 = random_batch_arrays(n, m, N, batch, 900 + N)
    g = np.random.default_rng(N)
    ncs = np.full(N + 1, nc, dtype=np.int32)
    ncs[N] = 0
    D = np.concatenate([g.standard_normal((batch, nc * s)) for _ in range(N)], axis=1)
    ny = int(ncs.sum())
    ws = g.standard_normal((batch, N * s + n))
    ys, zs = g.standard_normal((batch, ny)), g.standard_normal((batch, ny))
    irho = 0.05 + g.random((batch, ny))
    outs = {}
    for mode in ("ldl", "riccati"):
        if mode == "ldl":
            monkeypatch.setenv("PDPLQR_KKT_LDL", "1")  # read at handle creation
        else:
            monkeypatch.delenv("PDPLQR_KKT_LDL", raising=False)
        bs = BatchedLQRSolver(n, m, N, batch, solver="kkt", ncs=ncs)
        bs.set_model(E, c, H, h, D)
        bs.update_problem_data(ws, ys, zs, irho, sigma=1e-6)
        bs.backward(irho)
        out = np.zeros((batch, N * s + n))
        bs.forward(x0, out)
        assert np.all(bs.status() == 0)
        outs[mode] = out
        bs.close()
    d = np.linalg.norm(outs["ldl"] - outs["riccati"], axis=1) / np.linalg.norm(outs["riccati"], axis=1)
    assert float(d.max()) < 1e-10, float(d.max())
    for b in (0, batch - 1):
        pm = PackedModel(n, m, N, ncs, E[b], c[b], H[b], h[b], D[b])
        o = OracleKKT(pm)
        o.update_problem_data(ws[b], ys[b], zs[b], irho[b], 1e-6)
        o.backward(irho[b])
        ref = o.forward(x0[b])
        assert rel_err(outs["ldl"][b], ref) < TOL and rel_err(outs["riccati"][b], ref) < TOL, b


def test_register_tile_stage_varying_rows():
    """P = 16 model setup on register tiles (k_kkt_stage16 + k_kkt_pack16d) on
    a batch with varying constraint counts (the QDLDL-order path: the
    Riccati-order one needs a uniform row layout) against the oracle."""
    from oracle.oracle import OracleKKT
    from pdplqr import BatchedLQRSolver
    from pdplqr.model import PackedModel
    from pdplqr.problems import random_batch_arrays

    n, m, N, batch = 12, 4, 37, 4
    s = n + m
    E, c, H, h, x0 = random_batch_arrays(n, m, N, batch, 4242)
    g = np.random.default_rng(7)
    ncs = g.integers(0, 5, N + 1).astype(np.int32)
    ncs[N] = min(int(ncs[N]), 4)
    dims = [s] * N + [n]
    D = np.concatenate([g.standard_normal((batch, int(ncs[k]) * dims[k])) for k in range(N + 1)], axis=1)
    ny = int(ncs.sum())
    ws = g.standard_normal((batch, N * s + n))
    ys, zs = g.standard_normal((batch, ny)), g.standard_normal((batch, ny))
    irho = 0.05 + g.random((batch, ny))
    bs = BatchedLQRSolver(n, m, N, batch, solver="kkt", ncs=ncs)
    bs.set_model(E, c, H, h, D)
    bs.update_problem_data(ws, ys, zs, irho, sigma=1e-6)
    bs.backward(irho)
    out = np.zeros((batch, N * s + n))
    bs.forward(x0, out)
    assert np.all(bs.status() == 0)
    bs.close()
    for b in range(batch):
        pm = PackedModel(n, m, N, ncs, E[b], c[b], H[b], h[b], D[b])
        o = OracleKKT(pm)
        o.update_problem_data(ws[b], ys[b], zs[b], irho[b], 1e-6)
        o.backward(irho[b])
        assert rel_err(out[b], o.forward(x0[b])) < TOL, b


@pytest.mark.parametrize("name", ["e0.05_state_cost", "e0.5_state_box", "e3_rho_dyn", "wide_e0.5", "wide_e3"])
def test_kkt_exact_moreau_envelope(name):
    """P~ = (I + rho_dyn P)^{-1} P past the Neumann range:
    rho_dyn ||P||_F of 0.05 (large state cost), 0.5 (state-box rows at
    rho = 3e5) and 3 (rho = 1e5 with rho_dyn = 2e-5), on the 12/4 register
    kernel and the wide LDS kernel (28/8).  QDLDL factors any quasi-definite
    KKT (qdldl_solver.hpp:88-109), so the bar is the same 1e-8 against the
    oracle's QDLDL and against the dense QDLDL-equivalent solve."""
    from dense_ref import qdldl_equivalent
    from kkt_cases import TARGET, e_max, kkt_case, packed
    from oracle.oracle import OracleKKT
    from pdplqr import BatchedLQRSolver

    n, m, N, batch, rd, E, c, H, h, x0, ncs, D, ws, ys, zs, irho = kkt_case(name)
    bs = BatchedLQRSolver(n, m, N, batch, solver="kkt", ncs=ncs, rho_dyn=rd)
    bs.set_model(E, c, H, h, D)
    bs.update_problem_data(ws, ys, zs, irho, sigma=1e-6)
    bs.backward(irho)
    out = np.zeros((batch, N * (n + m) + n))
    bs.forward(x0, out)
    assert np.all(bs.status() == 0)
    for b in range(batch):
        pm = packed(n, m, N, ncs, E, c, H, h, D, b)
        e = e_max(pm, ws[b], ys[b], zs[b], irho[b], 1e-6, rd)
        assert TARGET[name] / 2 < e < 2 * TARGET[name], e
        o = OracleKKT(pm, rho_dyn=rd)
        o.update_problem_data(ws[b], ys[b], zs[b], irho[b], 1e-6)
        o.backward(irho[b])
        assert rel_err(out[b], o.forward(x0[b])) < TOL, b
        wd = qdldl_equivalent(pm, x0[b], ws[b], ys[b], zs[b], irho[b], 1e-6, rho_dyn=rd)
        assert rel_err(out[b], wd) < TOL, b
        assert rel_err(u_parts(out[b], n, m, N), u_parts(wd, n, m, N)) < 1e-6


def test_kkt_moreau_envelope_across_threshold():
    """The same problems on either side of the Neumann / exact switch
    (e = 0.015): a sweep of rho_dyn from 1e-6 to 1e-3 on one model, each solve
    against the oracle at 1e-8 -- no seam at the switch."""
    from kkt_cases import kkt_case, packed
    from oracle.oracle import OracleKKT
    from pdplqr import BatchedLQRSolver

    n, m, N, batch, _, E, c, H, h, x0, ncs, D, ws, ys, zs, irho = kkt_case("e0.5_state_box")
    irho = np.where(irho < 1e-3, 1e-2, irho)  # box rows at rho = 100: ||P|| ~ 1e2..1e3
    for rd in (1e-6, 1e-5, 3e-5, 1e-4, 3e-4, 1e-3):
        bs = BatchedLQRSolver(n, m, N, batch, solver="kkt", ncs=ncs, rho_dyn=rd)
        bs.set_model(E, c, H, h, D)
        bs.update_problem_data(ws, ys, zs, irho, sigma=1e-6)
        bs.backward(irho)
        out = np.zeros((batch, N * (n + m) + n))
        bs.forward(x0, out)
        assert np.all(bs.status() == 0)
        for b in range(batch):
            o = OracleKKT(packed(n, m, N, ncs, E, c, H, h, D, b), rho_dyn=rd)
            o.update_problem_data(ws[b], ys[b], zs[b], irho[b], 1e-6)
            o.backward(irho[b])
            assert rel_err(out[b], o.forward(x0[b])) < TOL, (rd, b)


def test_kkt_h_upload_keeps_protocol_state():
    """QDLDLSolver freezes its matrix at construction (qdldl_solver.hpp:36-45)
    and forms the right-hand side in update_problem_data: a later H upload
    (the facade's forward syncs H for update_rhs_initial_stage) must not
    invalidate the protocol -- backward without a new update_problem_data is
    valid, and the frozen matrix gives the same answer as an untouched solver."""
    from pdplqr import BatchedLQRSolver
    from pdplqr.problems import random_batch_arrays

    n, m, N, batch, nc = 12, 4, 20, 2, 4
    E, c, H, h, x0 = random_batch_arrays(n, m, N, batch, 77)
    g = np.random.default_rng(78)
    ncs = np.full(N + 1, nc, dtype=np.int32)
    D = np.concatenate([g.standard_normal((batch, nc * dk)) for dk in [n + m] * N + [n]], axis=1)
    ny = int(ncs.sum())
    ws = g.standard_normal((batch, N * (n + m) + n))
    ys, zs = g.standard_normal((batch, ny)), g.standard_normal((batch, ny))
    irho = 0.05 + g.random((batch, ny))
    outs = []
    for touch in (False, True):
        bs = BatchedLQRSolver(n, m, N, batch, solver="kkt", ncs=ncs)
        bs.set_model(E, c, H, h, D)
        bs.update_problem_data(ws, ys, zs, irho, sigma=1e-6)
        bs.backward(irho)
        out = np.zeros((batch, N * (n + m) + n))
        bs.forward(x0, out)
        if touch:
            bs.set_model(E, c, 2.0 * H, h, D)
        bs.backward(irho)
        bs.forward(x0, out)
        assert np.all(bs.status() == 0)
        outs.append(out)
    assert rel_err(outs[1], outs[0]) < 1e-13


def test_record_form_follows_last_backward_kkt():
    """The 12/4 KKT path writes the E^ record in a plain backward and the P~
    record in an ADMM run's cache-writing backward; the forward follows the
    last one (pdplqr_handle_s::rec_gain).  Plain solve -> ADMM run -> plain
    solve on one handle, with and without hipGraph replay (PDPLQR_GRAPH=1 is
    read at library load: child processes): both plain answers match OracleKKT."""
    import os
    import subprocess
    import sys
    import textwrap

    code = textwrap.dedent(r"""
        import os, sys, numpy as np
        sys.path[:0] = [os.environ["ROOT"], os.path.join(os.environ["ROOT"], "pdp-lqr_amd")]
        from oracle.oracle import OracleKKT
        from pdplqr import BatchedLQRSolver
        from pdplqr.model import PackedModel
        from pdplqr.problems import random_batch_arrays
        n, m, N, batch, nc = 12, 4, 37, 3, 4
        s = n + m
        E, c, H, h, x0 = random_batch_arrays(n, m, N, batch, 1234)
        g = np.random.default_rng(5)
        ncs = np.full(N + 1, nc, dtype=np.int32)
        ncs[N] = 0
        D = np.concatenate([g.standard_normal((batch, nc * s)) for _ in range(N)], axis=1)
        ny = int(ncs.sum())
        ws = g.standard_normal((batch, N * s + n))
        ys, zs = g.standard_normal((batch, ny)), g.standard_normal((batch, ny))
        irho = 0.05 + g.random((batch, ny))
        refs = []
        for b in range(batch):
            o = OracleKKT(PackedModel(n, m, N, ncs, E[b], c[b], H[b], h[b], D[b]))
            o.update_problem_data(ws[b], ys[b], zs[b], irho[b], 1e-6)
            o.backward(irho[b])
            refs.append(o.forward(x0[b]))
        bs = BatchedLQRSolver(n, m, N, batch, solver="kkt", ncs=ncs)
        bs.set_model(E, c, H, h, D)
        worst = 0.0
        for step in ("plain", "admm", "plain", "admm", "plain"):
            if step == "admm":
                lb, ub = np.full((batch, ny), -0.5), np.full((batch, ny), 0.5)
                w, y, z = np.zeros((batch, N * s + n)), np.zeros((batch, ny)), np.zeros((batch, ny))
                bs.admm_solve(x0, lb, ub, np.full((batch, ny), 3.0), w, y, z, max_iter=6, eps_abs=0.0, eps_rel=0.0)
                assert np.all(np.isfinite(w))
                continue
            bs.update_problem_data(ws, ys, zs, irho, sigma=1e-6)
            bs.backward(irho)
            out = np.zeros((batch, N * s + n))
            bs.forward(x0, out)
            assert np.all(bs.status() == 0)
            for b in range(batch):
                worst = max(worst, np.linalg.norm(out[b] - refs[b]) / np.linalg.norm(refs[b]))
        print("worst", worst)
        assert worst < 1e-8, worst
    """)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for graph in ("0", "1"):
        env = dict(os.environ, ROOT=root)
        if graph == "1":
            env["PDPLQR_GRAPH"] = "1"
        else:
            env.pop("PDPLQR_GRAPH", None)
        subprocess.run([sys.executable, "-c", code], check=True, env=env, timeout=300)
