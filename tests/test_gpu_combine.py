"""Unit parity of the device segment combine (combine_tiles.hpp: MFMA tiles,
blocked Cholesky, register triangular solve) against the numpy restatement of
SURVEY.md 0.1 (tests/seg_ref.py), through the pdplqr_debug_combine test hook.
Tolerance 1e-12 relative per block (fp64, well-conditioned random elements)."""
import ctypes as C

import numpy as np
import pytest

from seg_ref import combine

pytestmark = pytest.mark.gpu


def _elem(n, rng, zero_fcf=False):
    F = np.eye(n) + 0.2 * rng.standard_normal((n, n))
    G = rng.standard_normal((n, n))
    Cm = G @ G.T / n
    f = rng.standard_normal(n)
    H = rng.standard_normal((n, n))
    P = H @ H.T / n + np.eye(n)
    p = rng.standard_normal(n)
    if zero_fcf:
        F, Cm, f = np.zeros((n, n)), np.zeros((n, n)), np.zeros(n)
    return F, Cm, f, P, p


def _pack(e):
    F, Cm, f, P, p = e
    return np.concatenate([F.ravel(order="F"), Cm.ravel(order="F"), f, P.ravel(order="F"), p])


def _unpack(v, n):
    nn = n * n
    return (v[:nn].reshape(n, n, order="F"), v[nn:2 * nn].reshape(n, n, order="F"), v[2 * nn:2 * nn + n],
            v[2 * nn + n:3 * nn + n].reshape(n, n, order="F"), v[3 * nn + n:])


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 8, 12, 13, 16, 17, 20, 24, 31, 32, 33, 40, 50, 63])
@pytest.mark.parametrize("zero_b", [False, True])
def test_device_combine_matches_numpy(n, zero_b):
    """n > 32: the LDS combine of kernels_wide.hip (256-thread block)."""
    from pdplqr import _lib

    L = _lib.lib()
    L.pdplqr_debug_combine.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
    rng = np.random.default_rng(100 + n)
    a, b = _elem(n, rng), _elem(n, rng, zero_fcf=zero_b)
    va, vb = _pack(a), _pack(b)
    out = np.zeros_like(va)
    rc = L.pdplqr_debug_combine(n, va.ctypes.data, vb.ctypes.data, out.ctypes.data)
    assert rc == 0
    got, ref = _unpack(out, n), combine(a, b)
    for name, x, y in zip("FCfPp", got, ref):
        assert np.linalg.norm(x - y) <= 1e-12 * max(1.0, np.linalg.norm(y)), name


@pytest.mark.parametrize("n", [1, 2, 3, 5, 8, 12, 13, 16, 17, 20, 24, 31, 32])
@pytest.mark.parametrize("zero_b", [False, True])
@pytest.mark.parametrize("fcf", [True, False])
def test_multiwave_combine_matches_numpy(n, zero_b, fcf):
    """The 4-wave combine of the horizon scan (combine_mw.hpp): the same element
    as seg_ref.combine (1e-12).  fcf = False: only P, p are formed (the right
    operand holds the real terminal) and F, C, f are left untouched."""
    from pdplqr import _lib

    L = _lib.lib()
    L.pdplqr_debug_combine_mw.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
    rng = np.random.default_rng(500 + n)
    a, b = _elem(n, rng), _elem(n, rng, zero_fcf=zero_b or not fcf)
    va, vb = _pack(a), _pack(b)
    sentinel = 12345.0
    out = np.full_like(va, sentinel)
    rc = L.pdplqr_debug_combine_mw(n, va.ctypes.data, vb.ctypes.data, out.ctypes.data, int(fcf))
    assert rc == 0
    got, ref = _unpack(out, n), combine(a, b)
    for name, x, y in zip("FCfPp", got, ref):
        if not fcf and name in "FCf":
            assert np.all(x == sentinel), name
            continue
        assert np.linalg.norm(x - y) <= 1e-12 * max(1.0, np.linalg.norm(y)), name


def test_rsq_f64_accuracy_allows_one_newton_step():
    """rsqrt_f64 (device_common.hpp) refines v_rsq_f64 by Newton steps; record
    the hardware estimate's accuracy (one step squares the relative error)."""
    from pdplqr import _lib

    L = _lib.lib()
    L.pdplqr_debug_rsq.argtypes = [C.c_int, C.c_void_p, C.c_void_p]
    rng = np.random.default_rng(7)
    x = np.concatenate([10.0 ** rng.uniform(-30, 30, 200000), rng.uniform(0.5, 2.0, 200000)])
    y = np.zeros_like(x)
    assert L.pdplqr_debug_rsq(x.size, x.ctypes.data, y.ctypes.data) == 0
    rel = np.abs(y * np.sqrt(x) - 1.0)
    print(f"v_rsq_f64 max rel err {rel.max():.3e} (2^{np.log2(rel.max()):.1f})")
    assert rel.max() < 2.0 ** -22


def test_rsqrt_f64_full_precision():
    """The refined rsqrt_f64 is within 2 ulp of the correctly rounded 1/sqrt(x)."""
    from pdplqr import _lib

    L = _lib.lib()
    L.pdplqr_debug_rsqrt.argtypes = [C.c_int, C.c_void_p, C.c_void_p]
    rng = np.random.default_rng(8)
    x = np.concatenate([10.0 ** rng.uniform(-300, 300, 200000), rng.uniform(0.5, 2.0, 200000),
                        np.array([1.0, 4.0, 2.0, 1e-300, 1e300])])
    y = np.zeros_like(x)
    assert L.pdplqr_debug_rsqrt(x.size, x.ctypes.data, y.ctypes.data) == 0
    ref = 1.0 / np.sqrt(x)
    ulp = np.spacing(ref)
    err = np.abs(y - ref) / ulp
    print(f"rsqrt_f64 max error {err.max():.2f} ulp")
    assert err.max() <= 2.0


@pytest.mark.parametrize("n", [5, 24, 33, 40, 63])
def test_device_combine_lu_form_matches_numpy(n):
    """The LU form (Gauss-Jordan with partial pivoting, CondensedSystemLUSolver)
    gives the same element (1e-12): tiles for n <= 32, LDS past that."""
    from pdplqr import _lib

    L = _lib.lib()
    L.pdplqr_debug_combine_form.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
    rng = np.random.default_rng(900 + n)
    a, b = _elem(n, rng), _elem(n, rng)
    va, vb = _pack(a), _pack(b)
    out = np.zeros_like(va)
    assert L.pdplqr_debug_combine_form(n, va.ctypes.data, vb.ctypes.data, out.ctypes.data, 1) == 0
    got, ref = _unpack(out, n), combine(a, b)
    for name, x, y in zip("FCfPp", got, ref):
        assert np.linalg.norm(x - y) <= 1e-12 * max(1.0, np.linalg.norm(y)), name


@pytest.mark.parametrize("case", ["random", "zero_b", "no_fcf", "ill_Pb", "seg_elems"])
def test_qd_combine_matches_numpy(case):
    """The n = 24 blocked LDL^T combine of the horizon kernels (combine_qd.hpp):
    the same element as seg_ref.combine (1e-12; ill-conditioned P_b, where the
    two-Cholesky form itself drifts, 1e-10), untouched F, C, f without fcf."""
    from pdplqr import _lib

    L = _lib.lib()
    L.pdplqr_debug_combine_qd.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
    n = 24
    rng = np.random.default_rng(700 + len(case))
    fcf = case != "no_fcf"
    a, b = _elem(n, rng), _elem(n, rng, zero_fcf=(case in ("zero_b", "no_fcf")))
    tol = 1e-12
    if case == "ill_Pb":
        w, U = np.linalg.eigh(b[3])
        w[: n // 3] *= 1e-6
        b = (b[0], b[1], b[2], (U * w) @ U.T, b[4])
        tol = 1e-10
    if case == "seg_elems":  # real segment elements (24/8, 6 stages each)
        from seg_ref import slice_element

        m, Lseg = 8, 6
        E, c, Ht, ht = [], [], [], []
        for _ in range(2 * Lseg):
            A = np.eye(n) + 0.1 * rng.standard_normal((n, n))
            E.append(np.concatenate([rng.standard_normal((n, m)), A], 1))
            c.append(rng.standard_normal(n))
            M = rng.standard_normal((n + m, n + m))
            Ht.append(M @ M.T / (n + m) + np.eye(n + m))
            ht.append(rng.standard_normal(n + m))
        a = slice_element(E, c, Ht, ht, 0, Lseg, None)
        b = slice_element(E, c, Ht, ht, Lseg, 2 * Lseg, None)
    va, vb = _pack(a), _pack(b)
    sentinel = 12345.0
    out = np.full_like(va, sentinel)
    assert L.pdplqr_debug_combine_qd(va.ctypes.data, vb.ctypes.data, out.ctypes.data, int(fcf)) == 0
    got, ref = _unpack(out, n), combine(a, b)
    for name, x, y in zip("FCfPp", got, ref):
        if not fcf and name in "FCf":
            assert np.all(x == sentinel), name
            continue
        assert np.linalg.norm(x - y) <= tol * max(1.0, np.linalg.norm(y)), name
    for M in (got[1], got[3]):
        if fcf or M is got[3]:
            assert np.array_equal(M, M.T)  # written symmetric


def test_qd_combine_flags_zero_value_function():
    """P_b = 0 (a zero state cost): the first x pivot is 0 -- flagged, as chol(P_b)
    failing is in the Cholesky form (condensed_system.hpp:217-226)."""
    from pdplqr import _lib

    L = _lib.lib()
    L.pdplqr_debug_combine_qd.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
    n = 24
    rng = np.random.default_rng(71)
    a, b = _elem(n, rng), _elem(n, rng)
    b = (b[0], b[1], b[2], np.zeros((n, n)), b[4])
    va, vb = _pack(a), _pack(b)
    out = np.zeros_like(va)
    assert L.pdplqr_debug_combine_qd(va.ctypes.data, vb.ctypes.data, out.ctypes.data, 1) != 0


@pytest.mark.parametrize("n", [4, 8, 12])
@pytest.mark.parametrize("case", ["random", "zero_b", "no_fcf", "ill_Pb", "seg_elems"])
def test_qd1_combine_matches_numpy(n, case):
    """The one-wave blocked LDL^T combine of the n <= 12 scans (combine_qd1.hpp):
    the same element as seg_ref.combine (1e-12; ill-conditioned P_b 1e-10),
    untouched F, C, f without fcf, P and C written symmetric."""
    from pdplqr import _lib

    L = _lib.lib()
    L.pdplqr_debug_combine_qd1.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
    rng = np.random.default_rng(900 + 7 * n + len(case))
    fcf = case != "no_fcf"
    a, b = _elem(n, rng), _elem(n, rng, zero_fcf=(case in ("zero_b", "no_fcf")))
    tol = 1e-12
    if case == "ill_Pb":
        w, U = np.linalg.eigh(b[3])
        w[: max(1, n // 3)] *= 1e-6
        b = (b[0], b[1], b[2], (U * w) @ U.T, b[4])
        tol = 1e-10
    if case == "seg_elems":  # real segment elements (n/(n/3), 5 stages each)
        from seg_ref import slice_element

        m, Lseg = max(1, n // 3), 5
        E, c, Ht, ht = [], [], [], []
        for _ in range(2 * Lseg):
            A = np.eye(n) + 0.1 * rng.standard_normal((n, n))
            E.append(np.concatenate([rng.standard_normal((n, m)), A], 1))
            c.append(rng.standard_normal(n))
            M = rng.standard_normal((n + m, n + m))
            Ht.append(M @ M.T / (n + m) + np.eye(n + m))
            ht.append(rng.standard_normal(n + m))
        a = slice_element(E, c, Ht, ht, 0, Lseg, None)
        b = slice_element(E, c, Ht, ht, Lseg, 2 * Lseg, None)
    va, vb = _pack(a), _pack(b)
    sentinel = 12345.0
    out = np.full_like(va, sentinel)
    assert L.pdplqr_debug_combine_qd1(n, va.ctypes.data, vb.ctypes.data, out.ctypes.data, int(fcf)) == 0
    got, ref = _unpack(out, n), combine(a, b)
    for name, x, y in zip("FCfPp", got, ref):
        if not fcf and name in "FCf":
            assert np.all(x == sentinel), name
            continue
        assert np.linalg.norm(x - y) <= tol * max(1.0, np.linalg.norm(y)), (name, np.linalg.norm(x - y))
    assert np.array_equal(got[3], got[3].T)
    if fcf:
        assert np.array_equal(got[1], got[1].T)


@pytest.mark.parametrize("n", [4, 12])
def test_qd1_combine_flags_zero_value_function(n):
    """P_b = 0: the first x pivot is 0 -- flagged, as chol(P_b) failing is in the
    Cholesky form (condensed_system.hpp:217-226)."""
    from pdplqr import _lib

    L = _lib.lib()
    L.pdplqr_debug_combine_qd1.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
    rng = np.random.default_rng(72)
    a, b = _elem(n, rng), _elem(n, rng)
    b = (b[0], b[1], b[2], np.zeros((n, n)), b[4])
    out = np.zeros_like(_pack(a))
    assert L.pdplqr_debug_combine_qd1(n, _pack(a).ctypes.data, _pack(b).ctypes.data, out.ctypes.data, 1) != 0
