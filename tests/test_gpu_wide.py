"""GPU parity of the wide shapes 32 < n + m <= 64: the
serial solver's LDS kernels (kernels_big.hip), the parallel solver's
kernels_wide.hip (stage kernels for n + m > 32, element kernels for n > 32) in
both condensed forms, and the KKT solver, each against the CPU oracle's
restatement of the reference (OracleSerial / OracleParallel / OracleKKT) on
the same seeded inputs.

Tolerance: 1e-9 relative on w = [u; x] (the tiled shapes' bound, north_star
1e-6 on u*).  Shapes: 32/16 (n within the tiled element kernels, stage
kernels wide), 40/20 and 50/10 (everything wide), 20/30 (m > n)."""
import numpy as np
import pytest

from conftest import rel_err

pytestmark = pytest.mark.gpu
TOL = 1e-9
SHAPES = [(32, 16), (40, 20), (50, 10), (20, 30)]
# the 3 x 3 register-tile instances (kernels_riccati.hip wide3_dispatch):
# n % 4 = m % 4 = 0, m <= 16, 32 < n + m <= 48
WIDE3 = [(32, 4), (28, 8), (24, 12), (20, 16), (36, 4), (32, 8), (28, 12), (24, 16), (40, 4), (36, 8), (32, 12),
         (28, 16), (44, 4), (40, 8), (36, 12), (32, 16)]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    from pdplqr import device_count

    assert device_count() > 0, "no HIP device visible"


def _problem(n, m, N, batch, nc, seed):
    from pdplqr.problems import random_batch_arrays

    E, c, H, h, x0 = random_batch_arrays(n, m, N, batch, seed)
    s = n + m
    g = np.random.default_rng(seed + 1)
    ncs = np.full(N + 1, nc, dtype=np.int32)
    dims = [s] * N + [n]
    D = np.concatenate([g.standard_normal((batch, nc * dk)) for dk in dims], axis=1) if nc else np.zeros((batch, 0))
    ny = int(ncs.sum())
    ws = g.standard_normal((batch, N * s + n))
    ys, zs = g.standard_normal((batch, ny)), g.standard_normal((batch, ny))
    irho = 0.05 + g.random((batch, ny))
    return dict(E=E, c=c, H=H, h=h, x0=x0, ncs=ncs, D=D, ws=ws, ys=ys, zs=zs, irho=irho, nc=nc)


def _pm(p, b, n, m, N):
    from pdplqr.model import PackedModel

    return PackedModel(n, m, N, p["ncs"], p["E"][b], p["c"][b], p["H"][b], p["h"][b],
                       p["D"][b] if p["nc"] else np.zeros(0))


def _solve(bs, p, nc):
    bs.set_model(p["E"], p["c"], p["H"], p["h"], p["D"] if nc else None)
    bs.update_problem_data(p["ws"], p["ys"] if nc else None, p["zs"] if nc else None, p["irho"] if nc else None,
                           sigma=1e-6)
    bs.backward((1.0 / p["irho"]) if nc else None)
    out = np.zeros_like(p["ws"])
    bs.forward(p["x0"], out)
    return out


def _oracle_serial(p, b, n, m, N, ws=None):
    from oracle.oracle import OracleSerial

    o = OracleSerial(_pm(p, b, n, m, N))
    nc = p["nc"]
    o.update_problem_data(p["ws"][b] if ws is None else ws, p["ys"][b] if nc else None, p["zs"][b] if nc else None,
                          p["irho"][b] if nc else None, 1e-6)
    o.backward((1.0 / p["irho"][b]) if nc else None)
    return o.forward(p["x0"][b])


@pytest.mark.parametrize("n,m", SHAPES)
@pytest.mark.parametrize("keep", [True, False])
@pytest.mark.parametrize("nc", [0, 4])
def test_wide_serial_matches_oracle(n, m, keep, nc):
    from pdplqr import BatchedLQRSolver

    N, batch = 20, 3
    p = _problem(n, m, N, batch, nc, 3 * n + m + nc)
    bs = BatchedLQRSolver(n, m, N, batch, solver="serial", keep_factors=keep, ncs=p["ncs"])
    out = _solve(bs, p, nc)
    assert np.all(bs.status() == 0)
    for b in range(batch):
        assert rel_err(out[b], _oracle_serial(p, b, n, m, N)) < TOL, b


@pytest.mark.parametrize("n,m", WIDE3)
@pytest.mark.parametrize("nc", [0, 4])
@pytest.mark.parametrize("keep", [False, True])
def test_wide3_register_tile_shapes_match_oracle(n, m, nc, keep):
    """Every instantiated 3 x 3 register-tile shape (value-form backward
    k_riccati_bwd_vf3, or the full factor k_riccati_bwd_fast<3> with the factor
    cache, + DMA rollout k_rollout_dma3), penalties on and off; with the cache,
    backward_without_factorization on new linear terms as well."""
    from pdplqr import BatchedLQRSolver

    N, batch = 12, 2
    p = _problem(n, m, N, batch, nc, 7 * n + m + nc)
    bs = BatchedLQRSolver(n, m, N, batch, solver="serial", keep_factors=keep, ncs=p["ncs"])
    out = _solve(bs, p, nc)
    assert np.all(bs.status() == 0)
    for b in range(batch):
        assert rel_err(out[b], _oracle_serial(p, b, n, m, N)) < TOL, b
    if keep:
        ws2 = 0.5 * p["ws"]
        bs.update_problem_data(ws2, p["ys"] if nc else None, p["zs"] if nc else None, p["irho"] if nc else None,
                               sigma=1e-6)
        bs.backward_without_factorization((1.0 / p["irho"]) if nc else None)
        out2 = np.zeros_like(p["ws"])
        bs.forward(p["x0"], out2)
        for b in range(batch):
            assert rel_err(out2[b], _oracle_serial(p, b, n, m, N, ws=ws2[b])) < TOL, b
    bs.close()


@pytest.mark.parametrize("n,m", SHAPES)
@pytest.mark.parametrize("condensed", ["cholesky", "lu"])
@pytest.mark.parametrize("ns,seglen", [(4, 0), (3, 2)])
@pytest.mark.parametrize("nc", [0, 4])
def test_wide_parallel_matches_oracle(n, m, condensed, ns, seglen, nc):
    from pdplqr import BatchedLQRSolver

    N, batch = 24, 2
    p = _problem(n, m, N, batch, nc, 5 * n + m + nc + ns)
    bs = BatchedLQRSolver(n, m, N, batch, solver="parallel", num_segments=ns, keep_factors=True,
                          condensed=condensed.upper(), segment_len=seglen, ncs=p["ncs"])
    out = _solve(bs, p, nc)
    assert np.all(bs.status() == 0)
    for b in range(batch):
        assert rel_err(out[b], _oracle_serial(p, b, n, m, N)) < TOL, b


@pytest.mark.parametrize("n,m", [(40, 20), (32, 16)])
@pytest.mark.parametrize("condensed", ["cholesky", "lu"])
def test_wide_parallel_matches_parallel_oracle(n, m, condensed):
    """Against the restatement of the reference's parallel solver itself
    (OracleParallel: the same segmentation and condensed form)."""
    from oracle.oracle import OracleParallel
    from pdplqr import BatchedLQRSolver

    N, batch, ns = 30, 1, 4
    p = _problem(n, m, N, batch, 3, 17 * n + m)
    bs = BatchedLQRSolver(n, m, N, batch, solver="parallel", num_segments=ns, keep_factors=True,
                          condensed=condensed.upper(), ncs=p["ncs"])
    out = _solve(bs, p, 3)
    o = OracleParallel(_pm(p, 0, n, m, N), ns, True, condensed.upper())
    o.update_problem_data(p["ws"][0], p["ys"][0], p["zs"][0], p["irho"][0], 1e-6)
    o.backward(1.0 / p["irho"][0])
    assert rel_err(out[0], o.forward(p["x0"][0])) < TOL


@pytest.mark.parametrize("n,m", [(40, 20), (20, 30)])
@pytest.mark.parametrize("nc", [0, 4])
def test_wide_parallel_backward_without_factorization(n, m, nc):
    """backward_without_factorization (lqr_solver_parallel.hpp:148-154) on the
    wide shapes: new linear data, same rho, equals a fresh oracle solve."""
    from pdplqr import BatchedLQRSolver

    N, batch = 24, 2
    p = _problem(n, m, N, batch, nc, 9 * n + m + nc)
    bs = BatchedLQRSolver(n, m, N, batch, solver="parallel", num_segments=4, keep_factors=True, ncs=p["ncs"])
    _solve(bs, p, nc)
    g = np.random.default_rng(7)
    ws2 = p["ws"] + 0.1 * g.standard_normal(p["ws"].shape)
    bs.update_problem_data(ws2, p["ys"] if nc else None, p["zs"] if nc else None, p["irho"] if nc else None,
                           sigma=1e-6)
    bs.backward_without_factorization((1.0 / p["irho"]) if nc else None)
    out = np.zeros_like(ws2)
    bs.forward(p["x0"], out)
    for b in range(batch):
        assert rel_err(out[b], _oracle_serial(p, b, n, m, N, ws=ws2[b])) < TOL, b


@pytest.mark.parametrize("n,m", SHAPES)
@pytest.mark.parametrize("nc", [0, 4])
def test_wide_kkt_matches_oracle(n, m, nc):
    from oracle.oracle import OracleKKT
    from pdplqr import BatchedLQRSolver

    N, batch = 16, 2
    p = _problem(n, m, N, batch, nc, 13 * n + m + nc)
    bs = BatchedLQRSolver(n, m, N, batch, solver="kkt", ncs=p["ncs"])
    bs.set_model(p["E"], p["c"], p["H"], p["h"], p["D"] if nc else None)
    bs.update_problem_data(p["ws"], p["ys"] if nc else None, p["zs"] if nc else None, p["irho"] if nc else None,
                           sigma=1e-6)
    bs.backward(p["irho"] if nc else None)
    out = np.zeros_like(p["ws"])
    bs.forward(p["x0"], out)
    assert np.all(bs.status() == 0)
    for b in range(batch):
        o = OracleKKT(_pm(p, b, n, m, N))
        o.update_problem_data(p["ws"][b], p["ys"][b], p["zs"][b], p["irho"][b], 1e-6)
        o.backward(p["irho"][b])
        assert rel_err(out[b], o.forward(p["x0"][b])) < TOL, b


@pytest.mark.parametrize("n,m,N,batch,R,seglen", [(40, 20, 60, 2, 3, 4), (32, 16, 48, 1, 4, 0), (20, 30, 40, 2, 2, 3)])
def test_wide_horizon_shards_match_oracle(n, m, N, batch, R, seglen):
    """Horizon shards (pdplqr_shard_backward / shard_forward) on the wide
    shapes: virtual ranks in one process against the serial oracle (the n > 32
    element kernels fold the gathered rank elements by the scan form)."""
    from test_gpu_horizon import _run_virtual

    got, ref = _run_virtual(n, m, N, batch, R, seglen)
    for b in range(batch):
        assert rel_err(got[b], ref[b]) < TOL, b


@pytest.mark.parametrize("n,m", [(12, 4), (24, 8), (50, 10)])
@pytest.mark.parametrize("condensed", ["CHOLESKY", "LU"])
def test_boundary_maps_large_penalty(n, m, condensed):
    """Large constraint penalties (rho = 10 / inv_rho ~ 10..200) make |C P| at
    the segment boundaries ~1e4: Z = (I + C P)^{-1} is then small, and forming
    it as I - C Y cancels ~4 digits per boundary map (numpy: boundary states
    1e-10..1e-9 off at 24/8 and 50/10, against ~1e-11 for a solve).  The maps
    solve (I + C P) [Phi | phi] = [F | f - C p] instead (tmap_solve, the 4-wave
    V = Q^{-1} R^{-1} form, the wide kernels' triangular solves), so the
    trajectory stays at the 1e-9 bar with many short segments (seglen 2)."""
    from pdplqr import BatchedLQRSolver

    N, batch, nc = 24, 2, 4
    p = _problem(n, m, N, batch, nc, 7 * n + m)
    p["irho"] = 0.1 * p["irho"]
    bs = BatchedLQRSolver(n, m, N, batch, solver="parallel", num_segments=3, keep_factors=True, condensed=condensed,
                          segment_len=2, ncs=p["ncs"])
    out = _solve(bs, p, nc)
    assert np.all(bs.status() == 0)
    for b in range(batch):
        assert rel_err(out[b], _oracle_serial(p, b, n, m, N)) < TOL, b
