"""GPU parity of the num_devices split (pdp-lqr_amd/csrc/multidev.hip): one
LQRParallelSolver / BatchedLQRSolver handle over a list of devices, the
horizon cut into one slice per device, one all-gather of the slice elements
per backward.  On a one-GPU box:

* devices = [0]: the split with one slice, the exchange through a one-rank
  RCCL communicator (ncclCommInitAll / ncclAllGather, dlopen'ed librccl);
* devices = [0, 0, ...]: R slices on the same GPU, the exchange by device
  copies (RCCL needs distinct devices) -- the slicing, the row / D offsets,
  the per-slice terminals, the rank fold and the assembly of ws are the ones an
  R-GPU run takes.

Every answer is checked against the serial oracle (1e-9 relative, as
tests/test_gpu_parallel.py).  Distinct GPUs with RCCL are not reachable here
(unmeasured until an 8-GPU node runs it)."""
import numpy as np
import pytest

from conftest import golden_names, load_golden, rel_err

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


def _oracle_serial(pm, d):
    from oracle.oracle import OracleSerial

    o = OracleSerial(pm)
    o.update_problem_data(d["ws"], d["ys"], d["zs"], d["inv_rho"], float(d["sigma"]))
    o.backward(d["rho"])
    return o.forward(d["x0"])


@pytest.mark.parametrize("name", golden_names())
@pytest.mark.parametrize("devices,condensed", [([0], "CHOLESKY"), ([0, 0], "CHOLESKY"), ([0, 0, 0], "LU"),
                                               ([0, 0, 0, 0, 0], "CHOLESKY")])
def test_multidev_solver_matches_oracle(name, devices, condensed):
    from pdplqr import CondensedSystemSolverType, LQRParallelSolver

    pm, d = load_golden(name)
    if len(devices) > pm.N:
        pytest.skip("more slices than stages")
    model, ws, ys, zs, rho, irho = _lists(pm, d)
    sol = LQRParallelSolver(model, 4, True, CondensedSystemSolverType[condensed], devices=devices)
    sol.update_problem_data(ws, ys, zs, irho, float(d["sigma"]))
    sol.backward(rho)
    out = [w.copy() for w in ws]
    sol.forward(d["x0"], out)
    assert sol.status() == 0
    assert rel_err(np.concatenate(out), _oracle_serial(pm, d)) < TOL


@pytest.mark.parametrize("R", [1, 3, 8])
def test_multidev_batched_constraints_device_buffers(R):
    """batch 3, 12/4, per-stage constraint counts 0..4 (the row / D offsets of
    every slice differ), torch device buffers and host buffers give the same
    bits, every problem against the serial oracle; twice in a row (the handle
    re-solves after a new update_problem_data)."""
    import torch

    from oracle.oracle import OracleSerial
    from pdplqr import BatchedLQRSolver
    from pdplqr.model import PackedModel
    from pdplqr.problems import random_batch_arrays

    n, m, N, batch = 12, 4, 61, 3
    s = n + m
    E, c, H, h, x0 = random_batch_arrays(n, m, N, batch, 515)
    g = np.random.default_rng(516)
    ncs = g.integers(0, 5, size=N + 1).astype(np.int32)
    dims = [s] * N + [n]
    D = np.concatenate([g.standard_normal((batch, int(ncs[k]) * dims[k])) for k in range(N + 1)], axis=1)
    ny = int(ncs.sum())
    outs = []
    for mode in ("host", "device"):
        bs = BatchedLQRSolver(n, m, N, batch, solver="parallel", num_segments=4, ncs=ncs, devices=[0] * R)
        cv = (lambda a: a) if mode == "host" else (lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda())
        bs.set_model(cv(E), cv(c), cv(H), cv(h), cv(D))
        res = []
        for it in range(2):
            ws = g.standard_normal((batch, N * s + n)) if mode == "host" or it else None
            if mode == "host":
                ys, zs = g.standard_normal((batch, ny)), g.standard_normal((batch, ny))
                rho = 0.1 + g.random((batch, ny))
                outs.append((ws, ys, zs, rho))
            else:
                ws, ys, zs, rho = outs[it]
            irho = 1.0 / rho
            bs.update_problem_data(cv(ws), cv(ys), cv(zs), cv(irho), sigma=1e-6)
            bs.backward(cv(rho))
            out = np.zeros((batch, N * s + n)) if mode == "host" else torch.zeros(batch, N * s + n,
                                                                                   dtype=torch.float64).cuda()
            bs.forward(cv(x0), out)
            bs.synchronize()
            assert np.all(bs.status() == 0)
            res.append(out if mode == "host" else out.cpu().numpy())
        bs.close()
        if mode == "host":
            host_res = res
        else:
            for a, b in zip(host_res, res):
                assert np.array_equal(a, b)
    for it, (ws, ys, zs, rho) in enumerate(outs):
        for b in range(batch):
            o = OracleSerial(PackedModel(n, m, N, ncs, E[b], c[b], H[b], h[b], D[b]))
            o.update_problem_data(ws[b], ys[b], zs[b], 1.0 / rho[b], 1e-6)
            o.backward(rho[b])
            assert rel_err(host_res[it][b], o.forward(x0[b])) < TOL, (it, b)


def test_multidev_c4_shape():
    """24/8 over 8 slices of a 4096-stage horizon (C4's shape, 1/16 of its
    length): the 8-device layout of config C4 against the serial oracle."""
    from oracle.oracle import OracleSerial
    from pdplqr import BatchedLQRSolver
    from pdplqr.model import PackedModel
    from pdplqr.problems import random_batch_arrays

    n, m, N = 24, 8, 4096
    s = n + m
    E, c, H, h, x0 = random_batch_arrays(n, m, N, 1, 4242)
    bs = BatchedLQRSolver(n, m, N, 1, solver="parallel", num_segments=8, devices=[0] * 8)
    bs.set_model(E, c, H, h)
    ws = np.zeros((1, N * s + n))
    bs.update_problem_data(ws, sigma=1e-6)
    bs.backward()
    out = np.zeros_like(ws)
    bs.forward(x0, out)
    assert np.all(bs.status() == 0)
    o = OracleSerial(PackedModel(n, m, N, np.zeros(N + 1, dtype=np.int32), E[0], c[0], H[0], h[0], np.zeros(0)))
    o.update_problem_data(ws[0], None, None, None, 1e-6)
    o.backward(None)
    assert rel_err(out[0], o.forward(x0[0])) < TOL


@pytest.mark.parametrize("name", golden_names())
@pytest.mark.parametrize("devices,condensed", [([0], "CHOLESKY"), ([0, 0, 0], "LU"), ([0, 0, 0, 0, 0], "CHOLESKY")])
def test_multidev_backward_without_factorization(name, devices, condensed):
    """LQRParallelSolver::backward_without_factorization (lqr_solver_parallel.hpp:
    148-154,190-211) over the slices: after a factorising backward, new linear
    data (w-bar, y, z) with the same rho reuses every slice's factors and the
    last gather's F, C, P; the exchange carries only the slices' (f, p).  Twice
    in a row (the second starts from a nofact state), against the reference-
    shaped parallel oracle's backward_without_factorization and a fresh serial
    solve of the new data."""
    from oracle.oracle import OracleParallel, segmentation
    from pdplqr import CondensedSystemSolverType, LQRParallelSolver
    from pdplqr.model import unpack_ws

    pm, d = load_golden(name)
    if len(devices) > pm.N:
        pytest.skip("more slices than stages")
    model, ws, ys, zs, rho, irho = _lists(pm, d)
    sol = LQRParallelSolver(model, 4, True, CondensedSystemSolverType[condensed], devices=devices)
    sol.update_problem_data(ws, ys, zs, irho, float(d["sigma"]))
    sol.backward(rho)
    out = [w.copy() for w in ws]
    sol.forward(d["x0"], out)
    ns = 4 if segmentation(pm.N, 4, True)[0] else 1
    op = OracleParallel(pm, ns, True, condensed if ns > 1 else "LU")
    op.update_problem_data(d["ws"], d["ys"], d["zs"], d["inv_rho"], float(d["sigma"]))
    op.backward(d["rho"])
    g = np.random.default_rng(7)
    ws2 = d["ws"] + 0.1 * g.standard_normal(d["ws"].shape)
    zs2 = d["zs"] + 0.1 * g.standard_normal(d["zs"].shape)
    ys2 = d["ys"] + 0.1 * g.standard_normal(d["ys"].shape)
    off = np.concatenate([[0], np.cumsum(pm.ncs)])
    sl = lambda v: [v[off[k]:off[k + 1]] for k in range(pm.N + 1)]
    for it in range(2):
        sol.update_problem_data(unpack_ws(ws2, pm.n, pm.m, pm.N), sl(ys2), sl(zs2), irho, float(d["sigma"]))
        sol.backward_without_factorization(rho)
        out = [w.copy() for w in ws]
        sol.forward(d["x0"], out)
        assert sol.status() == 0
        op.update_problem_data(ws2, ys2, zs2, d["inv_rho"], float(d["sigma"]))
        op.backward_without_factorization(d["rho"])
        assert rel_err(np.concatenate(out), op.forward(d["x0"])) < TOL, it
        d2 = dict(d)
        d2.update(ws=ws2, ys=ys2, zs=zs2)
        assert rel_err(np.concatenate(out), _oracle_serial(pm, d2)) < TOL, it
        ws2 = ws2 + 0.05 * g.standard_normal(ws2.shape)


@pytest.mark.parametrize("R", [1, 2, 3])
def test_multidev_admm_matches_oracle(R):
    """admm_solve on a num_devices split (vectors and the update pass on the
    first device, the x-updates on the slices, nofact exchanges of (f, p) from
    iteration 2 on) against the oracle's ADMM over the parallel solver: fixed
    iterations, then an adaptive-rho run to tolerance (iteration counts and
    flags equal)."""
    from test_gpu_admm import _batch, _ubox_models

    from oracle.oracle import admm_solve as oracle_admm
    from pdplqr import BatchedLQRSolver

    models, x0s = _ubox_models(3, n=6, m=3, N=41, nc=3, bound=0.3, seed0=700)
    pms, ncs, A, lb, ub, x0, ws, ys, zs = _batch(models, x0s, seed=9)
    p = pms[0]
    for st in (dict(max_iter=30, eps_abs=0.0, eps_rel=0.0, adaptive_rho=False),
               dict(max_iter=400, check_every=10, eps_abs=1e-6, eps_rel=1e-6)):
        rho = np.full(lb.shape, 10.0)
        bs = BatchedLQRSolver(p.n, p.m, p.N, len(pms), solver="parallel", num_segments=4, condensed="CHOLESKY",
                              ncs=ncs, devices=[0] * R)
        bs.set_model(A["E"], A["c"], A["H"], A["h"], A["D"])
        w, y, z = ws.copy(), ys.copy(), zs.copy()
        info = bs.admm_solve(x0, lb, ub, rho, w, y, z, **st)
        assert np.count_nonzero(bs.status()) == 0
        bs.close()
        for b in range(len(pms)):
            ow, oy, oz, oi = oracle_admm(pms[b], x0[b], lb[b], ub[b], rho[b], ws[b], ys[b], zs[b], solver="parallel",
                                         num_segments=4, condensed="CHOLESKY", **st)
            assert rel_err(w[b], ow) < TOL and rel_err(y[b], oy) < TOL and rel_err(z[b], oz) < TOL, (b, st)
            assert info["iters"][b] == oi["iters"] and bool(info["converged"][b]) == bool(oi["converged"]), b


def test_multidev_mixed_device_host_calls():
    """a device-memory backward followed by a host-memory backward
    (no forward in between) on a same-device split: the exchange copies of the
    first backward read every slice's element on the reading slice's stream, and
    the second backward must not rewrite an element before they are done.  Both
    answers against the oracle."""
    import torch

    from oracle.oracle import OracleSerial
    from pdplqr import BatchedLQRSolver
    from pdplqr.model import PackedModel
    from pdplqr.problems import random_batch_arrays

    n, m, N, batch, R = 12, 4, 400, 64, 4
    s = n + m
    E, c, H, h, x0 = random_batch_arrays(n, m, N, batch, 808)
    bs = BatchedLQRSolver(n, m, N, batch, solver="parallel", num_segments=4, devices=[0] * R)
    bs.set_model(E, c, H, h)
    g = np.random.default_rng(809)
    refs, outs = [], []
    for mode in ("device", "host", "device", "host"):
        ws = g.standard_normal((batch, N * s + n))
        if mode == "device":
            bs.update_problem_data(torch.from_numpy(ws).cuda(), sigma=1e-6)
            bs.backward(torch.zeros(batch, 0, dtype=torch.float64).cuda())
        else:
            bs.update_problem_data(ws, sigma=1e-6)
            bs.backward()
        refs.append(ws)
    out = np.zeros((batch, N * s + n))
    bs.forward(x0, out)
    assert np.all(bs.status() == 0)
    for b in (0, batch // 2, batch - 1):
        o = OracleSerial(PackedModel(n, m, N, np.zeros(N + 1, dtype=np.int32), E[b], c[b], H[b], h[b], np.zeros(0)))
        o.update_problem_data(refs[-1][b], None, None, None, 1e-6)
        o.backward(None)
        assert rel_err(out[b], o.forward(x0[b])) < TOL, b


def test_multidev_model_upload_bytes():
    """host uploads through a split handle are counted (they were 0)."""
    from pdplqr import BatchedLQRSolver
    from pdplqr.problems import random_batch_arrays

    n, m, N = 4, 2, 20
    E, c, H, h, x0 = random_batch_arrays(n, m, N, 2, 3)
    bs = BatchedLQRSolver(n, m, N, 2, solver="parallel", num_segments=2, devices=[0, 0])
    bs.set_model(E, c, H, h)
    assert bs.handle.model_upload_bytes() == 8 * (E.size + c.size + H.size + h.size)


def test_multidev_unsupported_calls():
    from pdplqr import BatchedLQRSolver, PdplqrError

    n, m, N = 4, 2, 20
    bs = BatchedLQRSolver(n, m, N, 1, solver="parallel", num_segments=2, devices=[0, 0])
    bs.handle.set_stream(0)  # NULL: the default (drain before device inputs)
    with pytest.raises(PdplqrError):  # the split needs the PARALLEL solver
        BatchedLQRSolver(n, m, N, 1, solver="serial", devices=[0, 0])


@pytest.mark.parametrize("devices", [[0], [0, 0, 0]])
def test_multidev_caller_stream_orders_device_inputs(devices):
    """a split handle given the caller's stream
    (pdplqr_set_stream) orders its slices after that stream by events, not device
    drains.  Inputs are produced on a side stream behind a slow chain of
    matmuls, every protocol call is issued on it with device tensors and no host
    synchronisation until the end; the answers match the oracle each round (a
    slice reading its inputs early would see the previous round's data)."""
    import torch

    from oracle.oracle import OracleSerial
    from pdplqr import BatchedLQRSolver
    from pdplqr.model import PackedModel
    from pdplqr.problems import random_batch_arrays

    n, m, N, batch = 12, 4, 300, 16
    s = n + m
    E, c, H, h, x0 = random_batch_arrays(n, m, N, batch, 909)
    bs = BatchedLQRSolver(n, m, N, batch, solver="parallel", num_segments=4, devices=devices)
    side = torch.cuda.Stream()
    bs.handle.set_stream(side.cuda_stream)
    assert bs.handle.stream() == side.cuda_stream
    g = np.random.default_rng(910)
    dev = torch.device("cuda", 0)
    with torch.cuda.stream(side):
        bs.set_model(*(torch.from_numpy(a).to(dev) for a in (E, c, H, h)))
        ws_d = torch.zeros(batch, N * s + n, dtype=torch.float64, device=dev)
        x0_d = torch.from_numpy(x0).to(dev)
        outs, refs = [], []
        for _ in range(3):
            ws = g.standard_normal((batch, N * s + n))
            big = torch.randn(2048, 2048, device=dev)
            for _ in range(8):  # ~ms of work ahead of the input write on this stream
                big = big @ big / 45.0
            ws_d.copy_(torch.from_numpy(ws).pin_memory(), non_blocking=True)
            ws_d += 0.0 * big[0, 0].double()
            bs.update_problem_data(ws_d, sigma=1e-6)
            bs.backward(torch.zeros(batch, 0, dtype=torch.float64, device=dev))
            out_d = torch.empty(batch, N * s + n, dtype=torch.float64, device=dev)
            bs.forward(x0_d, out_d)
            outs.append(out_d)
            refs.append(ws)
    side.synchronize()
    assert np.all(bs.status() == 0)
    for out_d, ws in zip(outs, refs):
        out = out_d.cpu().numpy()
        for b in (0, batch - 1):
            o = OracleSerial(PackedModel(n, m, N, np.zeros(N + 1, dtype=np.int32), E[b], c[b], H[b], h[b],
                                         np.zeros(0)))
            o.update_problem_data(ws[b], None, None, None, 1e-6)
            o.backward(None)
            assert rel_err(out[b], o.forward(x0[b])) < TOL, b
    bs.close()
