"""ctypes wrapper of the CPU oracle (``oracle/pdplqr_oracle.c``).

TEST INFRASTRUCTURE ONLY: imported by ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg.  The product path (``pdp-lqr_amd``)
never imports it.  Parity status: see the C file's header ("parity unpinned"
w.r.t. reference outputs; pinned to the dense-KKT golden fixtures).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import List, Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liborcpdplqr.so")
_lib = None

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int)


def build() -> str:
    subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        vp = C.c_void_p
        L.orc_serial_create.restype = vp
        L.orc_serial_create.argtypes = [C.c_int, C.c_int, C.c_int, _ip, _dp, _dp, _dp, _dp, _dp]
        for nm in ["orc_serial_destroy", "orc_serial_clear_workspace"]:
            getattr(L, nm).argtypes = [vp]
        L.orc_serial_update_problem_data.argtypes = [vp, _dp, _dp, _dp, _dp, C.c_double]
        L.orc_serial_backward.argtypes = [vp, _dp]
        L.orc_serial_backward_without_factorization.argtypes = [vp, _dp]
        L.orc_serial_forward.argtypes = [vp, _dp, _dp]
        L.orc_serial_get_stage.argtypes = [vp, C.c_int, _dp, _dp]
        L.orc_parallel_create.restype = vp
        L.orc_parallel_create.argtypes = [C.c_int, C.c_int, C.c_int, _ip, _dp, _dp, _dp, _dp, _dp, C.c_int,
                                          C.c_int, C.c_int]
        L.orc_parallel_destroy.argtypes = [vp]
        L.orc_parallel_update_problem_data.argtypes = [vp, _dp, _dp, _dp, _dp, C.c_double]
        L.orc_parallel_backward.argtypes = [vp, _dp]
        L.orc_parallel_backward_without_factorization.argtypes = [vp, _dp]
        L.orc_parallel_forward.argtypes = [vp, _dp, _dp]
        L.orc_parallel_backward_ok.argtypes = [vp]
        L.orc_parallel_backward_ok.restype = C.c_int
        L.orc_parallel_segments.argtypes = [vp, _ip, _ip]
        L.orc_parallel_set_threads.argtypes = [vp, C.c_int, C.c_int]
        L.orc_parallel_set_threads.restype = C.c_int
        L.orc_parallel_get_segment.argtypes = [vp, C.c_int, _dp, _dp, _dp, _dp]
        L.orc_segmentation.argtypes = [C.c_int, C.c_int, C.c_int, _ip, _ip]
        L.orc_segmentation.restype = C.c_int
        L.orc_kkt_create.restype = vp
        L.orc_kkt_create.argtypes = [C.c_int, C.c_int, C.c_int, _ip, _dp, _dp, _dp, _dp, _dp, C.c_double,
                                     C.c_double]
        L.orc_kkt_destroy.argtypes = [vp]
        for nm in ["orc_kkt_dim", "orc_kkt_nnz", "orc_kkt_sumLnz"]:
            getattr(L, nm).argtypes = [vp]
            getattr(L, nm).restype = C.c_int
        L.orc_kkt_update_problem_data.argtypes = [vp, _dp, _dp, _dp, _dp, C.c_double]
        L.orc_kkt_backward.argtypes = [vp, _dp]
        L.orc_kkt_backward.restype = C.c_int
        L.orc_kkt_forward.argtypes = [vp, _dp, _dp]
        L.orc_kkt_get_solution.argtypes = [vp, _dp]
        L.orc_kkt_get_csc.argtypes = [vp, _ip, _ip, _dp]
        L.orc_kkt_get_rhs.argtypes = [vp, _dp]
        L.orc_batched_serial_solve.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, _dp, _dp, _dp, _dp, _dp,
                                               C.c_double, _dp, C.c_int]
        L.orc_batched_serial_solve.restype = C.c_int
        _lib = L
    return _lib


def _d(a: Optional[np.ndarray]):
    if a is None:
        return C.cast(0, _dp)
    assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_dp)


def _i(a: np.ndarray):
    assert a.dtype == np.int32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_ip)


def _flat(vecs) -> np.ndarray:
    if isinstance(vecs, np.ndarray):
        return np.ascontiguousarray(vecs, dtype=np.float64)
    parts = [np.asarray(v, dtype=np.float64).reshape(-1) for v in vecs]
    return np.ascontiguousarray(np.concatenate(parts) if parts else np.zeros(0))


class _Base:
    def __init__(self, pm):
        self.pm = pm
        self._keep = [np.ascontiguousarray(x) for x in (pm.ncs.astype(np.int32), pm.E, pm.c, pm.H, pm.h, pm.D)]
        self.n, self.m, self.N = pm.n, pm.m, pm.N
        self.s = pm.n + pm.m

    def _model_args(self):
        ncs, E, c, H, h, D = self._keep
        if D.size == 0:
            D = np.zeros(1)
            self._keep[5] = D
        return [self.n, self.m, self.N, _i(ncs), _d(E), _d(c), _d(H), _d(h), _d(D)]

    def _ws_len(self):
        return self.N * self.s + self.n

    def _ny(self):
        return max(int(np.sum(self.pm.ncs)), 1)

    def _vecs(self, v, size):
        a = _flat(v) if v is not None else np.zeros(size)
        if a.size == 0:
            a = np.zeros(1)
        return a


class OracleSerial(_Base):
    """``LQRSolver`` restatement (``lqr_solver.hpp:9-77``)."""

    def __init__(self, pm):
        super().__init__(pm)
        self.h = lib().orc_serial_create(*self._model_args())
        if not self.h:
            raise RuntimeError("oracle serial create failed")

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_serial_destroy(self.h)
            self.h = None

    def clear_workspace(self):
        lib().orc_serial_clear_workspace(self.h)

    def update_problem_data(self, ws, ys, zs, inv_rho, sigma):
        a = [self._vecs(ws, self._ws_len()), self._vecs(ys, self._ny()), self._vecs(zs, self._ny()),
             self._vecs(inv_rho, self._ny())]
        lib().orc_serial_update_problem_data(self.h, *[_d(x) for x in a], float(sigma))

    def backward(self, rho):
        r = self._vecs(rho, self._ny())
        lib().orc_serial_backward(self.h, _d(r))

    def backward_without_factorization(self, rho):
        r = self._vecs(rho, self._ny())
        lib().orc_serial_backward_without_factorization(self.h, _d(r))

    def forward(self, x0) -> np.ndarray:
        out = np.zeros(self._ws_len())
        lib().orc_serial_forward(self.h, _d(np.ascontiguousarray(x0, dtype=np.float64)), _d(out))
        return out

    def stage(self, k):
        dim = self.s if k < self.N else self.n
        L = np.zeros(dim * dim)
        lp = np.zeros(dim)
        lib().orc_serial_get_stage(self.h, k, _d(L), _d(lp))
        return L.reshape(dim, dim, order="F"), lp

    def value_function(self, k):
        """(P_k, p_k) with P_k = Lxx Lxx^T (the reference's segment/condensed convention)."""
        L, lp = self.stage(k)
        Lxx = L[-self.n:, -self.n:]
        return Lxx @ Lxx.T, lp[-self.n:].copy()


class OracleParallel(_Base):
    """``LQRParallelSolver`` restatement (``lqr_solver_parallel.hpp:19-238``)."""

    def __init__(self, pm, num_segments, load_balancing=True, condensed="CHOLESKY"):
        super().__init__(pm)
        t = {"LU": 0, "CHOLESKY": 1}[condensed]
        self.ns = num_segments
        self.h = lib().orc_parallel_create(*self._model_args(), int(num_segments), int(bool(load_balancing)), t)
        if not self.h:
            raise RuntimeError("oracle parallel create failed (bad segmentation or CHOLESKY with 1 segment)")

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_parallel_destroy(self.h)
            self.h = None

    def set_threads(self, on=True, pin=True) -> int:
        """Run the segments on an OpenMP team of num_segments threads, pinned
        like the reference (lqr_solver_parallel.hpp:102-112); returns the
        number of threads pinned."""
        return int(lib().orc_parallel_set_threads(self.h, int(bool(on)), int(bool(pin))))

    def segments(self):
        a = np.zeros(self.ns, dtype=np.int32)
        b = np.zeros(self.ns, dtype=np.int32)
        lib().orc_parallel_segments(self.h, _i(a), _i(b))
        return a, b

    def update_problem_data(self, ws, ys, zs, inv_rho, sigma):
        a = [self._vecs(ws, self._ws_len()), self._vecs(ys, self._ny()), self._vecs(zs, self._ny()),
             self._vecs(inv_rho, self._ny())]
        lib().orc_parallel_update_problem_data(self.h, *[_d(x) for x in a], float(sigma))

    def backward(self, rho):
        r = self._vecs(rho, self._ny())
        lib().orc_parallel_backward(self.h, _d(r))
        return bool(lib().orc_parallel_backward_ok(self.h))

    def backward_without_factorization(self, rho):
        r = self._vecs(rho, self._ny())
        lib().orc_parallel_backward_without_factorization(self.h, _d(r))

    def forward(self, x0) -> np.ndarray:
        out = np.zeros(self._ws_len())
        lib().orc_parallel_forward(self.h, _d(np.ascontiguousarray(x0, dtype=np.float64)), _d(out))
        return out

    def segment_state(self, i):
        n = self.n
        P, p, xh, uh = np.zeros(n * n), np.zeros(n), np.zeros(n), np.zeros(n)
        lib().orc_parallel_get_segment(self.h, i, _d(P), _d(p), _d(xh), _d(uh))
        return P.reshape(n, n, order="F"), p, xh, uh


class OracleKKT(_Base):
    """``QDLDLSolver`` restatement (``qdldl_solver.hpp:14-151`` + ``kkt.hpp``)."""

    def __init__(self, pm, rho_dyn=1e-6, sigma=1e-6):
        super().__init__(pm)
        self.h = lib().orc_kkt_create(*self._model_args(), float(rho_dyn), float(sigma))
        if not self.h:
            raise RuntimeError("oracle kkt create failed")
        self.dim = lib().orc_kkt_dim(self.h)
        self.nnz = lib().orc_kkt_nnz(self.h)
        self.sumLnz = lib().orc_kkt_sumLnz(self.h)

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_kkt_destroy(self.h)
            self.h = None

    def update_problem_data(self, ws, ys, zs, inv_rho, sigma):
        a = [self._vecs(ws, self._ws_len()), self._vecs(ys, self._ny()), self._vecs(zs, self._ny()),
             self._vecs(inv_rho, self._ny())]
        lib().orc_kkt_update_problem_data(self.h, *[_d(x) for x in a], float(sigma))

    def backward(self, inv_rho) -> int:
        r = self._vecs(inv_rho, self._ny())
        st = lib().orc_kkt_backward(self.h, _d(r))
        if st < 0:
            raise RuntimeError(f"QDLDL factorization failed with status: {st}")
        return st

    def forward(self, x0) -> np.ndarray:
        out = np.zeros(self._ws_len())
        lib().orc_kkt_forward(self.h, _d(np.ascontiguousarray(x0, dtype=np.float64)), _d(out))
        return out

    def solution(self):
        x = np.zeros(self.dim)
        lib().orc_kkt_get_solution(self.h, _d(x))
        return x

    def rhs(self):
        r = np.zeros(self.dim)
        lib().orc_kkt_get_rhs(self.h, _d(r))
        return r

    def csc(self):
        Ap = np.zeros(self.dim + 1, dtype=np.int32)
        Ai = np.zeros(self.nnz, dtype=np.int32)
        Ax = np.zeros(self.nnz)
        lib().orc_kkt_get_csc(self.h, _i(Ap), _i(Ai), _d(Ax))
        return Ap, Ai, Ax


def batched_serial_solve(n, m, N, E, c, H, h, x0, sigma=1e-6, threads=0) -> np.ndarray:
    """CPU baseline: independent serial (``LQRSolver``) solves over a batch, OpenMP
    over problems.  Arrays are batch-major flat (see problems.random_batch_arrays)."""
    batch = E.shape[0]
    out = np.zeros((batch, N * (n + m) + n))
    lib().orc_batched_serial_solve(n, m, N, batch, _d(np.ascontiguousarray(E)), _d(np.ascontiguousarray(c)),
                                   _d(np.ascontiguousarray(H)), _d(np.ascontiguousarray(h)),
                                   _d(np.ascontiguousarray(x0)), float(sigma), _d(out), int(threads))
    return out


def segmentation(N, ns, load_balancing=True):
    a = np.zeros(ns, dtype=np.int32)
    b = np.zeros(ns, dtype=np.int32)
    ok = lib().orc_segmentation(N, ns, int(bool(load_balancing)), _i(a), _i(b))
    return bool(ok), a, b


def admm_solve(pm, x0, lb, ub, rho, ws=None, ys=None, zs=None, solver="serial", sigma=1e-6, alpha=1.6,
               max_iter=4000, check_every=25, eps_abs=1e-3, eps_rel=1e-3, adaptive_rho=True,
               adaptive_rho_tolerance=5.0, **solver_kw):
    """CPU restatement of the ADMM outer loop (TEST INFRASTRUCTURE).

    Not in the reference (README.md:8).  Restates OSQP's
    published iteration (Stellato et al. 2020, Algorithm 1) around the
    reference's x-update protocol, exactly as pdp-lqr_amd/csrc/admm.hip
    documents it: the LQ solve is this module's restatement of
    update_problem_data / backward / forward (lqr_solver.hpp:41-77), with
    backward_without_factorization from iteration 2 on (lqr_solver.hpp:65-70;
    the QDLDL path re-solves with its first factor), the bounds are
    e_lb / e_ub of lqr_model.hpp:21-24, and the termination test is the primal
    residual |Dw - z|_inf and the ADMM dual residual |D^T rho (z+ - z)|_inf
    with OSQP's absolute/relative tolerances, every check_every iterations and
    at max_iter.  Adaptive rho (OSQP's compute_rho_estimate / update_rho rule):
    at a test that does not terminate, rho scales by
    e = sqrt((r_prim / max(|Dw|, |z|)) / (r_dual / |D^T y|)) (guards 1e-30, rows
    clamped to [1e-6, 1e6]) when e leaves [1/tol, tol], and the next x-update
    re-forms and refactors; no rescale while no row is active (no z at a bound:
    y is rounding noise and the dual normalisation undefined) or |D^T y| <= 1e-30.  One problem (PackedModel arrays of one batch
    entry).  Returns (ws, ys, zs, info)."""
    n, m, N = pm.n, pm.m, pm.N
    s = n + m
    ncs = [int(x) for x in pm.ncs]
    ny = sum(ncs)
    w = np.zeros(N * s + n) if ws is None else np.array(ws, dtype=np.float64)
    y = np.zeros(ny) if ys is None else np.array(ys, dtype=np.float64)
    z = np.zeros(ny) if zs is None else np.array(zs, dtype=np.float64)
    lb = np.asarray(lb, dtype=np.float64)
    ub = np.asarray(ub, dtype=np.float64)
    rho = np.asarray(rho, dtype=np.float64)
    irho = 1.0 / rho
    cls = {"serial": OracleSerial, "parallel": OracleParallel, "kkt": OracleKKT}[solver]
    solv = cls(pm, **solver_kw)
    # stage blocks: D_k (nc x dim, column-major), w_k, y_k offsets
    blocks = []
    doff = yoff = 0
    for k in range(N + 1):
        nc, dim = ncs[k], (s if k < N else n)
        Dk = pm.D[doff:doff + nc * dim].reshape(nc, dim, order="F") if nc else np.zeros((0, dim))
        blocks.append((k * s, dim, yoff, nc, Dk))
        doff += nc * dim
        yoff += nc
    it = 0
    conv = False
    rp = rd = 0.0
    refactor = True
    rho_updates = 0
    for it in range(1, max_iter + 1):
        solv.update_problem_data(w, y if ny else None, z if ny else None, irho if ny else None, sigma)
        if refactor:
            solv.backward(irho if solver == "kkt" else rho)
            refactor = False
        elif solver != "kkt":
            solv.backward_without_factorization(rho)
        wt = solv.forward(x0)
        if ny == 0:
            w = wt
            conv = True
            break
        check = it == max_iter or it % check_every == 0
        wn = alpha * wt + (1.0 - alpha) * w
        zn = np.empty(ny)
        yn = np.empty(ny)
        rp = dwm = zm = rd = dty = 0.0
        act = False  # some row's z at one of its bounds (OSQP: an active constraint)
        for (wo, dim, yo, nc, Dk) in blocks:
            if nc == 0:
                continue
            sl = slice(yo, yo + nc)
            v = Dk @ wt[wo:wo + dim]
            vrel = alpha * v + (1.0 - alpha) * z[sl]
            zn[sl] = np.minimum(np.maximum(vrel + irho[sl] * y[sl], lb[sl]), ub[sl])
            yn[sl] = y[sl] + rho[sl] * (vrel - zn[sl])
            if check:
                dwn = alpha * v + (1.0 - alpha) * (Dk @ w[wo:wo + dim])
                rp = max(rp, float(np.max(np.abs(dwn - zn[sl]))))
                dwm = max(dwm, float(np.max(np.abs(dwn))))
                zm = max(zm, float(np.max(np.abs(zn[sl]))))
                rd = max(rd, float(np.max(np.abs(Dk.T @ (rho[sl] * (zn[sl] - z[sl]))))))
                dty = max(dty, float(np.max(np.abs(Dk.T @ yn[sl]))))
                act = act or bool(np.any((zn[sl] <= lb[sl]) | (zn[sl] >= ub[sl])))
        w, y, z = wn, yn, zn
        if check and rp <= eps_abs + eps_rel * max(dwm, zm) and rd <= eps_abs + eps_rel * dty:
            conv = True
            break
        if check and adaptive_rho and it < max_iter and act and dty > 1e-30:
            e = np.sqrt((rp / (max(dwm, zm) + 1e-30)) / (rd / (dty + 1e-30) + 1e-30))
            if e > adaptive_rho_tolerance or e < 1.0 / adaptive_rho_tolerance:
                rho = np.minimum(np.maximum(rho * e, 1e-6), 1e6)
                irho = 1.0 / rho
                refactor = True
                rho_updates += 1
    return w, y, z, {"iters": it, "converged": conv, "prim_res": rp, "dual_res": rd, "rho": rho,
                     "rho_updates": rho_updates}
