"""Every BASELINE.json config at its own size on the GPU.

  target  N=1024  12/4  batch 4096  serial (value-form backward, the bench path)
  C3      N=256   12/4  batch 4096  serial
  C5      N=512   12/4  nc=4 (D=[I 0])  batch 1024  KKT (QDLDLSolver) and Riccati
  C4      N=65536 24/8  one problem, horizon solve on 1 GPU and as R=8 virtual ranks

The batches are bench.py's own device generator (same seeds), so these are the
problems the bench times.  Checks: status() == 0 for every problem, all-finite
output, the value-form backward equal to the full-factor path on EVERY problem
(1e-12 rel), bitwise-repeatable outputs over repeated solves (an in-flight
load landing in a reused register -- the round-1 failure -- shows up as a
moving set of wrong problems), and oracle parity (1e-9 rel; 1e-8 for the KKT
path, as tests/test_gpu_kkt.py) on sampled problems, including the ones that
failed in round 1.  All solves go through the C ABI (libpdplqr.so).
"""
import numpy as np
import pytest

from conftest import rel_err

pytestmark = pytest.mark.gpu

TOL = 1e-9
TOL_KKT = 1e-8
TOL_FF = 1e-12  # value form vs full factor, same device, fp64
# problems of the bench batch (seed 1234) that came out wrong / NaN in round 1
ROUND1_FAILED = [16, 23, 31, 32, 48, 50, 70, 81, 93, 107, 138, 934, 1088]


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    from pdplqr import device_count

    assert device_count() > 0, "no HIP device visible: GPU tests must run on an MI355X"
    return torch.device("cuda", 0)


def _gen(n, m, N, B, seed, dev):
    from bench import gen_batch_device

    return gen_batch_device(n, m, N, B, seed=seed, device=dev)


def _oracle_serial(n, m, N, E, c, H, h, x0, ws=None, sigma=1e-6):
    from oracle.oracle import OracleSerial
    from pdplqr.model import PackedModel

    pm = PackedModel(n, m, N, np.zeros(N + 1, dtype=np.int32), E, c, H, h, np.zeros(0))
    o = OracleSerial(pm)
    o.update_problem_data(np.zeros(N * (n + m) + n) if ws is None else ws, None, None, None, sigma)
    o.backward(None)
    return o.forward(x0)


def _serial_batch_checks(n, m, N, B, seed, dev, samples):
    import torch

    from pdplqr import BatchedLQRSolver

    s = n + m
    E, c, H, h, x0 = _gen(n, m, N, B, seed, dev)
    ws0 = torch.zeros(B, N * s + n, dtype=torch.float64, device=dev)
    bs = BatchedLQRSolver(n, m, N, B, keep_factors=False)
    bs.set_model(E, c, H, h)
    bs.update_problem_data(ws0, sigma=1e-6)
    outs = []
    for _ in range(3):
        out = torch.full_like(ws0, float("nan"))
        bs.backward()
        bs.forward(x0, out)
        bs.synchronize()
        st = bs.status()
        assert np.count_nonzero(st) == 0, [(int(b), int(st[b]) - 1) for b in np.nonzero(st)[0][:16]]
        outs.append(out)
    for o in outs[1:]:
        assert torch.equal(o, outs[0]), "value-form backward not repeatable"
    out = outs[0]
    assert bool(torch.isfinite(out).all())
    bs.close()
    # the full-factor path (k_riccati_bwd_fast) on the same problems
    ff = BatchedLQRSolver(n, m, N, B, keep_factors=True)
    ff.set_model(E, c, H, h)
    ff.update_problem_data(ws0, sigma=1e-6)
    ref = torch.empty_like(ws0)
    ff.backward()
    ff.forward(x0, ref)
    ff.synchronize()
    assert np.count_nonzero(ff.status()) == 0
    ff.close()
    d = torch.linalg.norm(out - ref, dim=1) / torch.linalg.norm(ref, dim=1)
    worst = int(torch.argmax(d))
    assert float(d.max()) < TOL_FF, (worst, float(d.max()))
    rng = np.random.default_rng(seed)
    pick = sorted(set(samples) | set(rng.choice(B, 8, replace=False).tolist()) | {0, B - 1, worst})
    for b in pick:
        w = _oracle_serial(n, m, N, *(t[b].cpu().numpy() for t in (E, c, H, h, x0)))
        assert rel_err(out[b].cpu().numpy(), w) < TOL, b
    return out


def test_target_config_bench_batch(torch_dev):
    """N=1024, 12/4, batch 4096 -- the headline workload, bench.py's batch."""
    _serial_batch_checks(12, 4, 1024, 4096, 1234, torch_dev, ROUND1_FAILED)


def test_c3_batched_mpc(torch_dev):
    """BASELINE config 3: batch 4096 independent LQRs, N=256, 12/4."""
    _serial_batch_checks(12, 4, 256, 4096, 4321, torch_dev, [])


def test_c5_conic_kkt_full_size(torch_dev):
    """BASELINE config 5: N=512, 12/4, nc=4 (D=[I 0] box on u), batch 1024,
    rho=0.1, random y, z, w-bar (bench.py's bench_conic data).  KKT path vs
    the oracle's kkt.hpp + QDLDL restatement, Riccati path vs the serial
    oracle on the same data."""
    import torch

    from oracle.oracle import OracleKKT, OracleSerial
    from pdplqr import BatchedLQRSolver
    from pdplqr.model import PackedModel

    n, m, nc, N, B = 12, 4, 4, 512, 1024
    s = n + m
    dev = torch_dev
    E, c, H, h, x0 = _gen(n, m, N, B, 555, dev)
    ncs = np.array([nc] * N + [0], dtype=np.int32)
    Dk = torch.zeros(nc, s, dtype=torch.float64, device=dev)
    Dk[:, :m] = torch.eye(m, dtype=torch.float64, device=dev)
    D = Dk.t().contiguous().reshape(-1).repeat(B, N)
    g = torch.Generator(device=dev)
    g.manual_seed(556)
    ny = nc * N
    ws = torch.randn(B, N * s + n, dtype=torch.float64, device=dev, generator=g)
    ys = torch.randn(B, ny, dtype=torch.float64, device=dev, generator=g)
    zs = torch.randn(B, ny, dtype=torch.float64, device=dev, generator=g)
    rho = torch.full((B, ny), 0.1, dtype=torch.float64, device=dev)
    irho = 1.0 / rho
    res = {}
    for solver in ("kkt", "serial"):
        bs = BatchedLQRSolver(n, m, N, B, solver=solver, ncs=ncs)
        bs.set_model(E, c, H, h, D)
        bs.update_problem_data(ws, ys, zs, irho, sigma=1e-6)
        bs.backward(irho if solver == "kkt" else rho)
        out = torch.full_like(ws, float("nan"))
        bs.forward(x0, out)
        bs.synchronize()
        assert np.count_nonzero(bs.status()) == 0, solver
        assert bool(torch.isfinite(out).all()), solver
        res[solver] = out.cpu().numpy()
        bs.close()
    pick = sorted({0, 1, 511, B - 1} | set(np.random.default_rng(5).choice(B, 4, replace=False).tolist()))
    Dh = D.cpu().numpy()
    h_ = [t.cpu().numpy() for t in (E, c, H, h, x0, ws, ys, zs, rho, irho)]
    for b in pick:
        Eb, cb, Hb, hb, xb, wb, yb, zb, rb, ib = (a[b] for a in h_)
        pm = PackedModel(n, m, N, ncs, Eb, cb, Hb, hb, Dh[b])
        ok = OracleKKT(pm)
        ok.update_problem_data(wb, yb, zb, ib, 1e-6)
        assert ok.backward(ib) == N * s  # QDLDL_factor: number of positive D entries (the primal pivots)
        assert rel_err(res["kkt"][b], ok.forward(xb)) < TOL_KKT, b
        os_ = OracleSerial(pm)
        os_.update_problem_data(wb, yb, zb, ib, 1e-6)
        os_.backward(rb)
        assert rel_err(res["serial"][b], os_.forward(xb)) < TOL, b


def _c4_problem():
    from pdplqr.problems import random_batch_arrays

    return random_batch_arrays(24, 8, 65536, 1, 65536)


@pytest.fixture(scope="module")
def c4_ref():
    n, m, N = 24, 8, 65536
    E, c, H, h, x0 = _c4_problem()
    return (E, c, H, h, x0), _oracle_serial(n, m, N, E[0], c[0], H[0], h[0], x0[0])


@pytest.mark.parametrize("R", [1, 8])
def test_c4_horizon_full_size(torch_dev, c4_ref, R):
    """BASELINE config 4: N=65536, 24/8, horizon-sharded.  R=1 is the 1-GPU
    horizon solve; R=8 runs the 8 rank slices as virtual ranks on this GPU
    (the host all-gathers the slice elements, as RCCL does across GPUs) --
    checked against the serial oracle over the full horizon."""
    from pdplqr.horizon import HorizonShard, slice_arrays, split_horizon

    (E, c, H, h, x0), ref = c4_ref
    n, m, N = 24, 8, 65536
    s = n + m
    sl = split_horizon(N, R)
    shards, elems = [], []
    for r, (N0, N1) in enumerate(sl):
        last = r == R - 1
        Nl = N1 - N0
        sh = HorizonShard(n, m, Nl, 1)
        sh.set_model(*slice_arrays(E, c, H, h, n, m, N, N0, N1, last))
        sh.update_problem_data(np.zeros((1, Nl * s + n)), sigma=1e-6)
        e = np.zeros((1, 3 * n * n + 2 * n))
        sh.backward(e, last)
        shards.append(sh)
        elems.append(e)
    gathered = np.ascontiguousarray(np.stack(elems))
    full = np.zeros(N * s + n)
    for r, (N0, N1) in enumerate(sl):
        Nl = N1 - N0
        loc = np.zeros((1, Nl * s + n))
        shards[r].forward(x0, gathered, R, r, loc)
        full[N0 * s:N1 * s] = loc[0, :Nl * s]
        if r == R - 1:
            full[N * s:] = loc[0, Nl * s:]
        shards[r].close()
    assert np.all(np.isfinite(full))
    assert rel_err(full, ref) < TOL
