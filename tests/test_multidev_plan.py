"""The num_devices split of one PARALLEL handle (pdp-lqr_amd/csrc/multidev.hip)
on the CPU: the library's slicing plan (pdplqr_multidev_plan, host arithmetic
only) against the Python split (pdplqr/horizon.py split_horizon) and the
constraint-row / D offsets of the boundary layout, and the fold the driver
relies on -- each plan slice's element (numpy restatement, tests/seg_ref.py),
the all-gather, the rank prefix / suffix fold -- reproducing the golden
Riccati trajectory's slice boundary states.  The GPU side of the same path is
tests/test_gpu_multidev.py."""
import ctypes as C

import numpy as np
import pytest

import dense_ref as dr
import seg_ref as sr
from conftest import golden_names, load_golden


def _plan(N, R, ncs, n, m):
    from pdplqr._lib import lib

    out = np.zeros((R, 8), dtype=np.int64)
    nc = None if ncs is None else np.ascontiguousarray(np.asarray(ncs, dtype=np.int32))
    rc = lib().pdplqr_multidev_plan(N, R, None if nc is None else nc.ctypes.data_as(C.POINTER(C.c_int32)), n, m,
                                    out.ctypes.data_as(C.POINTER(C.c_int64)))
    assert rc == 0
    return out


@pytest.mark.parametrize("N,R", [(1, 1), (7, 3), (64, 8), (65536, 8), (100, 7), (5, 5)])
def test_plan_matches_split_and_offsets(N, R):
    from pdplqr.horizon import split_horizon

    n, m = 6, 3
    s = n + m
    ncs = np.random.default_rng(N + R).integers(0, 4, size=N + 1)
    p = _plan(N, R, ncs, n, m)
    yo = np.concatenate([[0], np.cumsum(ncs)])
    dims = np.array([s] * N + [n])
    do = np.concatenate([[0], np.cumsum(ncs * dims)])
    for r, (a, b) in enumerate(split_horizon(N, R)):
        N0, N1, last, y0, nys, nct, d0, nds = p[r]
        assert (N0, N1, bool(last)) == (a, b, r == R - 1)
        assert y0 == yo[a] and nys == yo[b] - yo[a]
        assert d0 == do[a] and nds == do[b] - do[a]
        assert nct == (ncs[N] if r == R - 1 else 0)


def test_plan_rejects_bad_arguments():
    from pdplqr._lib import lib

    out = np.zeros((4, 8), dtype=np.int64)
    ptr = out.ctypes.data_as(C.POINTER(C.c_int64))
    assert lib().pdplqr_multidev_plan(3, 4, None, 2, 1, ptr) < 0  # more slices than stages
    assert lib().pdplqr_multidev_plan(0, 1, None, 2, 1, ptr) < 0


@pytest.mark.parametrize("name", [g for g in golden_names() if "constrained" not in g][:4])
@pytest.mark.parametrize("R", [2, 3, 5])
def test_plan_slices_fold_to_the_riccati_trajectory(name, R):
    """Slices cut by the library's plan, each reduced to its element, gathered
    and folded (prefix of the earlier slices, suffix of the later ones) give
    every slice's start state of the golden trajectory -- the fold
    pdplqr_shard_forward does on the device after the driver's all-gather."""
    pm, d = load_golden(name)
    n, m, N = pm.n, pm.m, pm.N
    s = n + m
    if R > N:
        pytest.skip("more slices than stages")
    E, c, Ht, ht = dr.effective_cost(pm, d["ws"], d["ys"], d["zs"], d["inv_rho"], d["rho"], float(d["sigma"]))
    p = _plan(N, R, pm.ncs, n, m)
    elems = []
    for r in range(R):
        N0, N1, last = int(p[r, 0]), int(p[r, 1]), bool(p[r, 2])
        elems.append(sr.slice_element(E, c, Ht, ht, N0, N1, (Ht[N], ht[N]) if last else None))
    ref = d["w_riccati"]
    for r in range(R):
        if r == 0:
            pre = (np.eye(n), np.zeros((n, n)), np.zeros(n), np.zeros((n, n)), np.zeros(n))
        else:
            pre = elems[0]
            for j in range(1, r):
                pre = sr.combine(pre, elems[j])
        suf = elems[R - 1]
        for j in range(R - 2, r - 1, -1):
            suf = sr.combine(elems[j], suf)
        x = sr.boundary_state(pre, suf, d["x0"])
        N0 = int(p[r, 0])
        want = ref[N0 * s + m:(N0 + 1) * s]
        assert np.linalg.norm(x - want) <= 1e-9 * max(1.0, np.linalg.norm(want)), r
