"""GPU parity of LQRParallelSolver (segment Riccati + associative segment
combine + segment rollout) against the CPU oracle's restatement of the
reference parallel solver (lqr_solver_parallel.hpp) and the golden fixtures.

Tolerance: 1e-9 relative on w = [u; x] (north_star bound 1e-6 on u*).  The
device refines every reference segment into sub-segments (segment_len);
results must not depend on that refinement beyond rounding.
"""
import numpy as np
import pytest

from conftest import golden_names, load_golden, rel_err, u_parts

pytestmark = pytest.mark.gpu
TOL = 1e-9


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    from pdplqr import device_count

    assert device_count() > 0, "no HIP device visible"


def _lists(pm, d):
    from pdplqr.model import unpack_model, unpack_ws

    model = unpack_model(pm)
    N = pm.N
    off = np.concatenate([[0], np.cumsum(pm.ncs)])
    sl = lambda v: [v[off[k]:off[k + 1]] for k in range(N + 1)]
    return model, unpack_ws(d["ws"], pm.n, pm.m, N), sl(d["ys"]), sl(d["zs"]), sl(d["rho"]), sl(d["inv_rho"])


def _oracle_par(pm, d, ns, condensed):
    from oracle.oracle import OracleParallel

    o = OracleParallel(pm, ns, True, condensed)
    o.update_problem_data(d["ws"], d["ys"], d["zs"], d["inv_rho"], float(d["sigma"]))
    o.backward(d["rho"])
    return o.forward(d["x0"])


@pytest.mark.parametrize("name", golden_names())
@pytest.mark.parametrize("ns,condensed,seglen", [(4, "CHOLESKY", 0), (2, "LU", 0), (8, "CHOLESKY", 3), (4, "LU", 1)])
def test_parallel_matches_oracle(name, ns, condensed, seglen):
    from oracle.oracle import segmentation
    from pdplqr import CondensedSystemSolverType, LQRParallelSolver

    pm, d = load_golden(name)
    if not segmentation(pm.N, ns, True)[0]:
        pytest.skip("empty segment")
    model, ws, ys, zs, rho, irho = _lists(pm, d)
    sol = LQRParallelSolver(model, ns, True, CondensedSystemSolverType[condensed], segment_len=seglen)
    sol.update_problem_data(ws, ys, zs, irho, float(d["sigma"]))
    sol.backward(rho)
    out = [w.copy() for w in ws]
    sol.forward(d["x0"], out)
    w = np.concatenate(out)
    ref = _oracle_par(pm, d, ns, condensed)
    assert rel_err(w, ref) < TOL
    assert rel_err(w, d["w_riccati"]) < TOL
    n, m, N = pm.n, pm.m, pm.N
    assert rel_err(u_parts(w, n, m, N), u_parts(d["w_riccati"], n, m, N)) < 1e-6
    assert sol.status() == 0
    st, ln = sol.segments()
    ost, oln = segmentation(pm.N, ns, True)[1:]
    assert list(st) == list(ost) and list(ln) == list(oln)


def test_quadrotor_example_parallel_kat():
    """lqr_example.cpp:212-221: 4 segments, load balancing, CHOLESKY."""
    from pdplqr import CondensedSystemSolverType, LQRParallelSolver
    from pdplqr.model import initialize_vectors
    from pdplqr.problems import quadrotor_model

    model, x0 = quadrotor_model(100)
    ws, ys, zs, rho, irho = initialize_vectors(model, 0.01)
    sol = LQRParallelSolver(model, 4, True, CondensedSystemSolverType.CHOLESKY)
    sol.update_problem_data(ws, ys, zs, irho, 1e-6)
    sol.backward(rho)
    sol.forward(x0, ws)
    assert np.allclose(ws[0][:4], [-2.8980566697, 2.8980566697, -2.8980566697, 2.8980566697], atol=5e-10)
    assert abs(ws[100][2] - 0.9999999000) < 5e-10


def test_cholesky_single_segment_rejected():
    from pdplqr import CondensedSystemSolverType, LQRParallelSolver, PdplqrError
    from pdplqr.problems import random_model

    model, _ = random_model(4, 2, 10, seed=1)
    with pytest.raises(PdplqrError):
        LQRParallelSolver(model, 1, True, CondensedSystemSolverType.CHOLESKY)
    LQRParallelSolver(model, 1, True, CondensedSystemSolverType.LU)  # LU with one segment is valid


@pytest.mark.parametrize("n,m,N,batch,seglen", [(12, 4, 1024, 1, 0), (12, 4, 96, 6, 5), (24, 8, 64, 2, 8),
                                                (4, 2, 33, 3, 2)])
def test_batched_parallel_matches_oracle(n, m, N, batch, seglen):
    from oracle.oracle import OracleSerial
    from pdplqr import BatchedLQRSolver
    from pdplqr.model import PackedModel
    from pdplqr.problems import random_batch_arrays

    E, c, H, h, x0 = random_batch_arrays(n, m, N, batch, n * 7 + m)
    s = n + m
    ws0 = np.zeros((batch, N * s + n))
    bs = BatchedLQRSolver(n, m, N, batch, solver="parallel", num_segments=4, keep_factors=True,
                          segment_len=seglen)
    bs.set_model(E, c, H, h)
    bs.update_problem_data(ws0, sigma=1e-6)
    bs.backward()
    out = np.zeros_like(ws0)
    bs.forward(x0, out)
    assert np.all(bs.status() == 0)
    for b in range(batch):
        pm = PackedModel(n, m, N, np.zeros(N + 1, dtype=np.int32), E[b], c[b], H[b], h[b], np.zeros(0))
        o = OracleSerial(pm)
        o.update_problem_data(ws0[b], None, None, None, 1e-6)
        o.backward(None)
        assert rel_err(out[b], o.forward(x0[b])) < TOL, b


@pytest.mark.parametrize("name", ["random_n12_m4_N64_nc4", "quadrotor_N30_constrained", "random_n24_m8_N40",
                                  "ubox_n12_m4_N48_nc4"])
@pytest.mark.parametrize("ns,condensed,seglen", [(4, "CHOLESKY", 0), (2, "LU", 5), (8, "CHOLESKY", 3)])
def test_parallel_backward_without_factorization(name, ns, condensed, seglen):
    """LQRParallelSolver::backward_without_factorization (lqr_solver_parallel.hpp:
    148-154,190-211): after a factorising backward, new linear data (w-bar, y, z)
    with the same rho reuses the cached factors; the solution equals a fresh full
    solve of the new data (oracle, serial refactor)."""
    from oracle.oracle import OracleSerial, segmentation
    from pdplqr import CondensedSystemSolverType, LQRParallelSolver
    from pdplqr.model import unpack_ws

    pm, d = load_golden(name)
    if not segmentation(pm.N, ns, True)[0]:
        pytest.skip("empty segment")
    model, ws, ys, zs, rho, irho = _lists(pm, d)
    sol = LQRParallelSolver(model, ns, True, CondensedSystemSolverType[condensed], segment_len=seglen)
    sol.update_problem_data(ws, ys, zs, irho, float(d["sigma"]))
    sol.backward(rho)
    out = [w.copy() for w in ws]
    sol.forward(d["x0"], out)
    g = np.random.default_rng(5)
    ws2 = d["ws"] + 0.1 * g.standard_normal(d["ws"].shape)
    zs2 = d["zs"] + 0.1 * g.standard_normal(d["zs"].shape)
    ys2 = d["ys"] + 0.1 * g.standard_normal(d["ys"].shape)
    off = np.concatenate([[0], np.cumsum(pm.ncs)])
    sl = lambda v: [v[off[k]:off[k + 1]] for k in range(pm.N + 1)]
    for it in range(2):  # twice: the second reuse starts from a nofact state
        sol.update_problem_data(unpack_ws(ws2, pm.n, pm.m, pm.N), sl(ys2), sl(zs2), irho, float(d["sigma"]))
        sol.backward_without_factorization(rho)
        out = [w.copy() for w in ws]
        sol.forward(d["x0"], out)
        o = OracleSerial(pm)
        o.update_problem_data(ws2, ys2, zs2, d["inv_rho"], float(d["sigma"]))
        o.backward(d["rho"])
        ref = o.forward(d["x0"])
        assert rel_err(np.concatenate(out), ref) < TOL, it
        ws2 = ws2 + 0.05 * g.standard_normal(ws2.shape)


@pytest.mark.parametrize("n,m,N,batch,seglen,condensed",
                         [(12, 4, 1024, 1, 0, "CHOLESKY"), (12, 4, 1024, 1, 0, "LU"), (12, 4, 96, 3, 5, "CHOLESKY"),
                          (12, 4, 40, 2, 2, "LU"), (12, 4, 7, 2, 3, "CHOLESKY"), (12, 4, 12, 1, 4, "CHOLESKY"),
                          (24, 8, 96, 2, 5, "CHOLESKY"), (24, 8, 40, 1, 3, "CHOLESKY"), (24, 8, 7, 2, 3, "CHOLESKY"),
                          (24, 8, 512, 1, 0, "CHOLESKY"), (20, 6, 130, 2, 4, "LU"), (24, 8, 12, 1, 4, "CHOLESKY"),
                          (18, 4, 33, 3, 2, "CHOLESKY"), (24, 8, 96, 1, 5, "LU")])
def test_scan_forms_match_serial(n, m, N, batch, seglen, condensed):
    """Every suffix-scan form on the shapes that take it, against the serial
    solve and so the oracle: n <= 16 CHOLESKY takes the radix-4 Hillis-Steele
    launches (k_seg_scan4, two rounds per launch); LU takes Sklansky rounds
    through the one-wave combine, in place after the first (tcombine_parts'
    aliasing contract, combine_tiles.hpp); 16 < n <= 32 CHOLESKY takes
    Sklansky rounds on the 4-wave combine.  Segment counts 1..~200 cover the
    partial upper halves, every case of the two-level round (i + d, i + 2d,
    i + 3d past the end) and the terminal element's (P, p)-only combines."""
    from pdplqr import BatchedLQRSolver
    from pdplqr.problems import random_batch_arrays

    E, c, H, h, x0 = random_batch_arrays(n, m, N, batch, 2000 + N + n)
    ws0 = np.zeros((batch, N * (n + m) + n))
    bs = BatchedLQRSolver(n, m, N, batch, solver="parallel", num_segments=4, keep_factors=False,
                          segment_len=seglen, condensed=condensed)
    bs.set_model(E, c, H, h)
    bs.update_problem_data(ws0, sigma=1e-6)
    bs.backward()
    out = np.zeros_like(ws0)
    bs.forward(x0, out)
    assert np.all(bs.status() == 0)
    bs.close()
    ser = BatchedLQRSolver(n, m, N, batch, solver="serial")
    ser.set_model(E, c, H, h)
    ser.update_problem_data(ws0, sigma=1e-6)
    ser.backward()
    ref = np.zeros_like(ws0)
    ser.forward(x0, ref)
    ser.close()
    assert rel_err(out, ref) < TOL


def test_graph_replay_matches_direct():
    """Protocol calls replayed from a captured hipGraph (PDPLQR_GRAPH=1, read at
    library load: run in a child process) give the same trajectory as direct
    issue, across repeated calls and a changed x0."""
    import subprocess
    import sys
    import textwrap

    code = textwrap.dedent(r"""
        import os, sys, numpy as np
        sys.path[:0] = [os.environ["ROOT"], os.path.join(os.environ["ROOT"], "pdp-lqr_amd")]
        import torch
        from pdplqr import BatchedLQRSolver
        from pdplqr.problems import random_batch_arrays
        n, m, N, batch = 12, 4, 200, 3
        E, c, H, h, x0 = random_batch_arrays(n, m, N, batch, 5)
        dev = torch.device("cuda", 0)
        t = lambda a: torch.as_tensor(a, device=dev)
        outs = []
        for solver in ("parallel", "serial"):
            bs = BatchedLQRSolver(n, m, N, batch, solver=solver, num_segments=4)
            bs.set_model(t(E), t(c), t(H), t(h))
            bs.update_problem_data(torch.zeros(batch, N * (n + m) + n, dtype=torch.float64, device=dev), sigma=1e-6)
            out = torch.zeros(batch, N * (n + m) + n, dtype=torch.float64, device=dev)
            X0 = t(x0)
            for it in range(3):
                bs.backward()
                bs.forward(X0 * (1 + it), out)
            torch.cuda.synchronize()
            outs.append(out.cpu().numpy())
            bs.close()
        np.save(os.environ["OUT"], np.stack(outs))
    """)
    import os
    import tempfile
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = []
    for graph in ("0", "1"):
        fd, path = tempfile.mkstemp(suffix=".npy")
        os.close(fd)
        env = dict(os.environ, ROOT=root, OUT=path)
        if graph == "1":
            env["PDPLQR_GRAPH"] = "1"
        else:
            env.pop("PDPLQR_GRAPH", None)
        subprocess.run([sys.executable, "-c", code], check=True, env=env, timeout=300)
        res.append(np.load(path))
        os.unlink(path)
    assert np.all(np.isfinite(res[0]))
    assert np.array_equal(res[0], res[1])


def test_parallel_non_spd_status_is_per_problem():
    """An indefinite stage in one problem of a batch is reported for that
    problem only (stage + 1); the other problems' combines stay clean."""
    from pdplqr import BatchedLQRSolver
    from pdplqr.problems import random_batch_arrays

    n, m, N, batch = 4, 2, 40, 3
    E, c, H, h, x0 = random_batch_arrays(n, m, N, batch, 3)
    s = n + m
    H = H.copy()
    H[1, 17 * s * s:18 * s * s] = -np.eye(s).reshape(-1)  # stage 17 of problem 1 indefinite
    bs = BatchedLQRSolver(n, m, N, batch, solver="parallel", num_segments=4)
    bs.set_model(E, c, H, h)
    bs.update_problem_data(np.zeros((batch, N * s + n)), sigma=0.0)
    bs.backward()
    bs.forward(x0, np.zeros((batch, N * s + n)))
    st = bs.status()
    assert st[0] == 0 and st[2] == 0 and st[1] != 0, st
