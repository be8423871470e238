"""Host-side mirror of the reference solver classes over the C ABI.

Same names, arguments and protocol as the reference (C++ namespace ``lqr``):

* ``LQRSolver(model)``                                   lqr_solver.hpp:9-77
* ``LQRParallelSolver(model, num_segments, load_balancing=True,
  solver_type=CondensedSystemSolverType.CHOLESKY)``      lqr_solver_parallel.hpp:19-238
* ``QDLDLSolver(model)``                                 qdldl_solver.hpp:14-151

each with ``update_problem_data(ws, ys, zs, inv_rho_vecs, sigma)``,
``backward(rho_vecs)`` (``QDLDLSolver``: ``inv_rho_vecs``),
``backward_without_factorization(rho_vecs)`` (Riccati solvers),
``forward(x0, ws)`` (writes ``ws`` in place, as the reference's
``std::vector<VectorXs>&``) and ``clear_workspace()``.  All compute runs in
HIP kernels on the MI355X (libpdplqr.so); there is no CPU fallback.

``BatchedLQRSolver`` is the batched entry point the reference lacks: ``batch``
independent problems of one shape, host numpy or device (torch) buffers.
"""
from __future__ import annotations

import atexit
import ctypes as C
import enum
import weakref
from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import AdmmSettings, Config, check, lib
from .model import LQRModel, pack_model, pack_stage_vectors, w_sizes


class CondensedSystemSolverType(enum.IntEnum):
    """lqr_solver_parallel.hpp:14-17"""

    LU = _lib.PDPLQR_CONDENSED_LU
    CHOLESKY = _lib.PDPLQR_CONDENSED_CHOLESKY


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch") and hasattr(x, "data_ptr")


def _ptr(x, what: str):
    """(pointer, mem) for a float64 contiguous numpy array or torch tensor."""
    if x is None:
        return None, None
    if _is_torch(x):
        import torch

        if x.dtype != torch.float64 or not x.is_contiguous():
            raise TypeError(f"{what}: torch tensor must be float64 and contiguous")
        mem = _lib.PDPLQR_MEM_DEVICE if x.is_cuda else _lib.PDPLQR_MEM_HOST
        return C.c_void_p(x.data_ptr()), mem
    a = x
    if not isinstance(a, np.ndarray) or a.dtype != np.float64 or not a.flags["C_CONTIGUOUS"]:
        raise TypeError(f"{what}: expected a C-contiguous float64 numpy array")
    return C.c_void_p(a.ctypes.data), _lib.PDPLQR_MEM_HOST


def _mem_of(*ps):
    mems = {m for (_, m) in ps if m is not None}
    if len(mems) > 1:
        raise TypeError("mixing host and device buffers in one call")
    return mems.pop() if mems else _lib.PDPLQR_MEM_HOST


_LIVE = weakref.WeakSet()  # open handles, closed by _close_all at interpreter exit
_ATEXIT = False


def _close_all():
    """Destroy every handle still open when the interpreter exits, while the
    HIP runtime (torch's, which libpdplqr.so binds to) is fully alive: this
    hook is registered after torch is imported, so it runs before torch's own
    exit hooks and long before the runtime's static destructors in exit()
    (teardown order)."""
    for hd in list(_LIVE):
        try:
            hd.close()
        except Exception:
            pass


class _Handle:
    """Owns one pdplqr_handle."""

    def __init__(self, nx, nu, N, batch=1, solver=_lib.PDPLQR_SOLVER_SERIAL, num_segments=1, load_balancing=True,
                 condensed_type=_lib.PDPLQR_CONDENSED_CHOLESKY, device=0, keep_factors=True, ncs=None,
                 rho_dyn=1e-6, kkt_sigma=1e-6, segment_len=0, devices=None):
        L = lib()
        cfg = Config()
        L.pdplqr_config_init(C.byref(cfg))
        cfg.nx, cfg.nu, cfg.N, cfg.batch = int(nx), int(nu), int(N), int(batch)
        cfg.solver = int(solver)
        cfg.num_segments = int(num_segments)
        cfg.load_balancing = int(bool(load_balancing))
        cfg.condensed_type = int(condensed_type)
        cfg.device = int(device)
        cfg.keep_factors = int(bool(keep_factors))
        cfg.rho_dyn = float(rho_dyn)
        cfg.kkt_sigma = float(kkt_sigma)
        cfg.segment_len = int(segment_len)
        self._devs = None
        if devices is not None and len(devices) > 0:
            # the horizon split over the listed GPUs by this one handle
            # (multidev.hip; one entry: the same split with one slice)
            self._devs = np.ascontiguousarray(np.asarray(devices, dtype=np.int32))
            cfg.num_devices = int(self._devs.size)
            cfg.devices = self._devs.ctypes.data_as(C.POINTER(C.c_int32))
        self._ncs = None
        if ncs is not None:
            self._ncs = np.ascontiguousarray(np.asarray(ncs, dtype=np.int32))
            cfg.ncs = self._ncs.ctypes.data_as(C.POINTER(C.c_int32))
        self.cfg = cfg
        h = C.c_void_p()
        check(L.pdplqr_create(C.byref(cfg), C.byref(h)))
        self.h = h
        global _ATEXIT
        if not _ATEXIT:  # (lib() imported torch first: this hook runs before torch's)
            atexit.register(_close_all)
            _ATEXIT = True
        _LIVE.add(self)
        self.nx, self.nu, self.N, self.batch = int(nx), int(nu), int(N), int(batch)
        self.ncs = self._ncs if self._ncs is not None else np.zeros(N + 1, dtype=np.int32)
        self.ny = int(np.sum(self.ncs))

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            lib().pdplqr_destroy(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # stream ordering with torch ---------------------------------------------
    # The handle launches on its own (non-blocking) stream.  When a call is
    # handed torch CUDA tensors, that stream first waits for torch's current
    # stream (the tensors may have been written there), and torch's current
    # stream waits for the handle's work after the call (outputs are read
    # there, inputs may be freed or overwritten there): events only, no host
    # synchronisation.  Host (numpy) calls are synchronous in the C ABI.
    def _torch_stream(self):
        import torch

        hs = getattr(self, "_ts", None)
        if hs is None:
            hs = self._ts = torch.cuda.ExternalStream(self.stream(), device=torch.device("cuda", self.cfg.device))
        return hs

    def _enter(self, *objs):
        if not any(o is not None and _is_torch(o) and o.is_cuda for o in objs):
            return None
        import torch

        hs = self._torch_stream()
        cur = torch.cuda.current_stream(hs.device)
        if cur.cuda_stream == hs.cuda_stream:
            return None
        hs.wait_stream(cur)
        return cur

    def _leave(self, cur):
        if cur is not None:
            cur.wait_stream(self._torch_stream())

    # raw protocol (pointers already validated) -----------------------------
    def set_model(self, E, c, H, h, D=None):
        ps = [_ptr(E, "E"), _ptr(c, "c"), _ptr(H, "H"), _ptr(h, "h"), _ptr(D, "D")]
        mem = _mem_of(*ps)
        cur = self._enter(E, c, H, h, D)
        check(lib().pdplqr_set_model(self.h, ps[0][0], ps[1][0], ps[2][0], ps[3][0], ps[4][0], mem))
        self._leave(cur)

    def update_problem_data(self, ws, ys, zs, inv_rho, sigma):
        ps = [_ptr(ws, "ws"), _ptr(ys, "ys"), _ptr(zs, "zs"), _ptr(inv_rho, "inv_rho")]
        mem = _mem_of(*ps)
        cur = self._enter(ws, ys, zs, inv_rho)
        check(lib().pdplqr_update_problem_data(self.h, ps[0][0], ps[1][0], ps[2][0], ps[3][0], float(sigma), mem))
        self._leave(cur)

    def backward(self, rho):
        p = _ptr(rho, "rho")
        cur = self._enter(rho)
        check(lib().pdplqr_backward(self.h, p[0], _mem_of(p)))
        self._leave(cur)

    def backward_without_factorization(self, rho):
        p = _ptr(rho, "rho")
        cur = self._enter(rho)
        check(lib().pdplqr_backward_without_factorization(self.h, p[0], _mem_of(p)))
        self._leave(cur)

    def forward(self, x0, ws_out):
        ps = [_ptr(x0, "x0"), _ptr(ws_out, "ws")]
        cur = self._enter(x0, ws_out)
        check(lib().pdplqr_forward(self.h, ps[0][0], ps[1][0], _mem_of(*ps)))
        self._leave(cur)

    def clear_workspace(self):
        check(lib().pdplqr_clear_workspace(self.h))

    def model_upload_bytes(self) -> int:
        """Host -> device model bytes since creation (pdplqr_get_model_upload_bytes)."""
        v = C.c_int64(0)
        check(lib().pdplqr_get_model_upload_bytes(self.h, C.byref(v)))
        return int(v.value)

    def synchronize(self):
        check(lib().pdplqr_synchronize(self.h))

    def stream(self) -> int:
        return int(lib().pdplqr_get_stream(self.h) or 0)

    def set_stream(self, stream_ptr: int):
        check(lib().pdplqr_set_stream(self.h, C.c_void_p(stream_ptr)))
        self._ts = None

    def status(self) -> np.ndarray:
        out = np.zeros(self.batch, dtype=np.int32)
        check(lib().pdplqr_get_status(self.h, out.ctypes.data_as(C.POINTER(C.c_int32))))
        return out

    def value_function(self, b: int, k: int):
        n = self.nx
        P = np.zeros(n * n)
        p = np.zeros(n)
        check(lib().pdplqr_get_value_function(self.h, int(b), int(k), C.c_void_p(P.ctypes.data),
                                              C.c_void_p(p.ctypes.data)))
        return P.reshape(n, n, order="F"), p

    def admm_solve(self, x0, lb, ub, rho, ws, ys, zs, settings: "AdmmSettings"):
        ps = [_ptr(x0, "x0"), _ptr(lb, "lb"), _ptr(ub, "ub"), _ptr(rho, "rho"), _ptr(ws, "ws"), _ptr(ys, "ys"),
              _ptr(zs, "zs")]
        mem = _mem_of(*ps)
        cur = self._enter(x0, lb, ub, rho, ws, ys, zs)
        check(lib().pdplqr_admm_solve(self.h, C.byref(settings), *[p[0] for p in ps], mem))
        self._leave(cur)

    def admm_info(self):
        it = np.zeros(self.batch, dtype=np.int32)
        cv = np.zeros(self.batch, dtype=np.int32)
        rp = np.zeros(self.batch)
        rd = np.zeros(self.batch)
        rho = np.zeros((self.batch, max(self.ny, 1)))
        i32 = C.POINTER(C.c_int32)
        n = check(lib().pdplqr_admm_info(self.h, it.ctypes.data_as(i32), cv.ctypes.data_as(i32),
                                         C.c_void_p(rp.ctypes.data), C.c_void_p(rd.ctypes.data),
                                         C.c_void_p(rho.ctypes.data)))
        return {"iterations": int(n), "iters": it, "converged": cv.astype(bool), "prim_res": rp, "dual_res": rd,
                "rho": rho[:, :self.ny]}

    def segments(self, ns: int):
        a = np.zeros(ns, dtype=np.int32)
        b = np.zeros(ns, dtype=np.int32)
        check(lib().pdplqr_get_segments(self.h, a.ctypes.data_as(C.POINTER(C.c_int32)),
                                        b.ctypes.data_as(C.POINTER(C.c_int32))))
        return a, b


def admm_settings(sigma=1e-6, alpha=1.6, max_iter=4000, check_every=25, eps_abs=1e-3, eps_rel=1e-3,
                  adaptive_rho=True, adaptive_rho_tolerance=5.0) -> AdmmSettings:
    st = AdmmSettings()
    lib().pdplqr_admm_settings_init(C.byref(st))
    st.sigma, st.alpha = float(sigma), float(alpha)
    st.max_iter, st.check_every = int(max_iter), int(check_every)
    st.eps_abs, st.eps_rel = float(eps_abs), float(eps_rel)
    st.adaptive_rho, st.adaptive_rho_tolerance = int(bool(adaptive_rho)), float(adaptive_rho_tolerance)
    return st


def _stage_vecs(model: LQRModel, vecs, what):
    return pack_stage_vectors(vecs, [int(x) for x in model.ncs]) if model.ncs else np.zeros(0)


class _ModelSolver:
    """Shared body of the reference-mirroring single-problem solvers."""

    _solver_kind = _lib.PDPLQR_SOLVER_SERIAL
    _reupload_model = True  # Riccati solvers re-read model_ on every call (lqr_solver.hpp:25)

    def _init_handle(self, model: LQRModel, device=0, keep_factors=True, **kw):
        self.model_ = model  # non-owning in the reference: the model must outlive the solver
        self._hd = _Handle(model.n, model.m, model.N, 1, self._solver_kind, device=device,
                           keep_factors=keep_factors, ncs=[int(x) for x in model.ncs], **kw)
        self._upload_model()

    def _upload_model(self):
        pm = pack_model(self.model_)
        self._pm = pm
        self._hd.set_model(pm.E, pm.c, pm.H, pm.h, pm.D if pm.D.size else None)

    def _y(self, v):
        if self._hd.ny == 0:
            return None
        return np.ascontiguousarray(pack_stage_vectors(v, [int(x) for x in self.model_.ncs]))

    def clear_workspace(self):
        self._hd.clear_workspace()

    def update_problem_data(self, ws: Sequence[np.ndarray], ys, zs, inv_rho_vecs, sigma: float):
        m = self.model_
        if self._reupload_model:
            self._upload_model()
        w = np.ascontiguousarray(pack_stage_vectors(ws, w_sizes(m.n, m.m, m.N)))
        self._hd.update_problem_data(w, self._y(ys), self._y(zs), self._y(inv_rho_vecs), sigma)

    def backward(self, rho_vecs):
        self._hd.backward(self._y(rho_vecs))

    def forward(self, x0, ws: List[np.ndarray]):
        m = self.model_
        out = np.zeros(m.N * (m.n + m.m) + m.n)
        self._hd.forward(np.ascontiguousarray(x0, dtype=np.float64), out)
        s = m.n + m.m
        for k in range(m.N):
            ws[k][:] = out[k * s:(k + 1) * s]
        ws[m.N][:] = out[m.N * s:]
        return ws

    def status(self) -> int:
        return int(self._hd.status()[0])

    def admm_solve(self, x0, ws: List[np.ndarray], ys, zs, rho_vecs, sigma: float = 1e-6, alpha: float = 1.6,
                   max_iter: int = 4000, check_every: int = 25, eps_abs: float = 1e-3, eps_rel: float = 1e-3,
                   adaptive_rho: bool = True, adaptive_rho_tolerance: float = 5.0):
        """ADMM outer loop over this solver (new: absent in the reference,
        README.md:8) for the bounds ``e_lb <= D_con w <= e_ub`` stored in the
        model's nodes (lqr_model.hpp:21-24).  ``ws, ys, zs`` are the warm start
        (``initialize_vectors``) and are overwritten in place with the solution;
        ``rho_vecs`` as the reference's.  Returns admm_info() of problem 0."""
        m = self.model_
        if self._reupload_model:
            self._upload_model()
        ncs = [int(x) for x in m.ncs]
        w = np.ascontiguousarray(pack_stage_vectors(ws, w_sizes(m.n, m.m, m.N)))
        lb = np.ascontiguousarray(pack_stage_vectors([nd.e_lb for nd in m.nodes], ncs)) if self._hd.ny else None
        ub = np.ascontiguousarray(pack_stage_vectors([nd.e_ub for nd in m.nodes], ncs)) if self._hd.ny else None
        y, z, r = self._y(ys), self._y(zs), self._y(rho_vecs)
        st = admm_settings(sigma, alpha, max_iter, check_every, eps_abs, eps_rel, adaptive_rho,
                           adaptive_rho_tolerance)
        self._hd.admm_solve(np.ascontiguousarray(x0, dtype=np.float64), lb, ub, r, w, y, z, st)
        s = m.n + m.m
        for k in range(m.N):
            ws[k][:] = w[k * s:(k + 1) * s]
        ws[m.N][:] = w[m.N * s:]
        off = 0
        for k, nc in enumerate(ncs):
            if nc:
                ys[k][:] = y[off:off + nc]
                zs[k][:] = z[off:off + nc]
            off += nc
        info = self._hd.admm_info()
        return {"iterations": info["iterations"], "iters": int(info["iters"][0]),
                "converged": bool(info["converged"][0]), "prim_res": float(info["prim_res"][0]),
                "dual_res": float(info["dual_res"][0])}


class LQRSolver(_ModelSolver):
    """Serial square-root Riccati (lqr_solver.hpp:9-77), HIP backward/forward."""

    _solver_kind = _lib.PDPLQR_SOLVER_SERIAL

    def __init__(self, model: LQRModel, device: int = 0, keep_factors: bool = True):
        self._init_handle(model, device=device, keep_factors=keep_factors)

    def backward_without_factorization(self, rho_vecs):
        self._hd.backward_without_factorization(self._y(rho_vecs))

    def value_function(self, k: int):
        """(P_k, p_k) with P_k = Lxx Lxx^T of the stage-k workspace."""
        return self._hd.value_function(0, k)


class LQRParallelSolver(_ModelSolver):
    """Parallel DP over horizon segments (lqr_solver_parallel.hpp:19-238)."""

    _solver_kind = _lib.PDPLQR_SOLVER_PARALLEL

    def __init__(self, model: LQRModel, num_segments: int, load_balancing: bool = True,
                 solver_type: CondensedSystemSolverType = CondensedSystemSolverType.CHOLESKY, device: int = 0,
                 segment_len: int = 0, devices=None):
        """``devices``: a list of HIP ordinals; more than one splits the horizon
        across them (one slice per device, one RCCL all-gather of the slice
        elements per backward; include/pdplqr.h num_devices) -- the multi-GPU
        form of the reference's OpenMP team (lqr_solver_parallel.hpp:102-113)."""
        self.num_segments = int(num_segments)
        self._init_handle(model, device=device, keep_factors=True, num_segments=num_segments,
                          load_balancing=load_balancing, condensed_type=int(solver_type), segment_len=segment_len,
                          devices=devices)

    def backward_without_factorization(self, rho_vecs):
        self._hd.backward_without_factorization(self._y(rho_vecs))

    def segments(self):
        return self._hd.segments(self.num_segments)


class QDLDLSolver(_ModelSolver):
    """KKT + sparse LDL^T path (qdldl_solver.hpp:14-151).  The KKT matrix is
    frozen at construction with rho_dyn = sigma = 1e-6 (qdldl_solver.hpp:38-42)."""

    _solver_kind = _lib.PDPLQR_SOLVER_KKT
    # form_rhs / update_rhs_initial_stage read model_ on every call
    # (kkt.hpp:207-300); the matrix itself stays the one formed at construction
    # (the C ABI forms it on the first model upload only).
    _reupload_model = True

    def __init__(self, model: LQRModel, device: int = 0):
        self._init_handle(model, device=device, keep_factors=False, rho_dyn=1e-6, kkt_sigma=1e-6)

    def backward(self, inv_rho_vecs):  # NOTE: inverse rho, as the reference (qdldl_solver.hpp:24)
        self._hd.backward(self._y(inv_rho_vecs))


class BatchedLQRSolver:
    """``batch`` independent LQ problems of one shape (n, m, N), solved by one
    set of HIP launches.  Buffers are batch-major flat arrays in the boundary
    layout (include/pdplqr.h): numpy (host) or torch CUDA tensors (device)."""

    def __init__(self, n: int, m: int, N: int, batch: int, solver: str = "serial", num_segments: int = 1,
                 load_balancing: bool = True, condensed: str = "CHOLESKY", keep_factors: bool = False,
                 ncs=None, device: int = 0, segment_len: int = 0, rho_dyn: float = 1e-6, kkt_sigma: float = 1e-6,
                 devices=None):
        kind = {"serial": _lib.PDPLQR_SOLVER_SERIAL, "parallel": _lib.PDPLQR_SOLVER_PARALLEL,
                "kkt": _lib.PDPLQR_SOLVER_KKT}[solver]
        self.n, self.m, self.N, self.batch = n, m, N, batch
        self._hd = _Handle(n, m, N, batch, kind, num_segments=num_segments, load_balancing=load_balancing,
                           condensed_type=int(CondensedSystemSolverType[condensed]), device=device,
                           keep_factors=keep_factors, ncs=ncs, segment_len=segment_len, rho_dyn=rho_dyn,
                           kkt_sigma=kkt_sigma, devices=devices)

    @property
    def handle(self) -> _Handle:
        return self._hd

    def set_model(self, E, c, H, h, D=None):
        self._hd.set_model(E, c, H, h, D)

    def update_problem_data(self, ws, ys=None, zs=None, inv_rho=None, sigma: float = 0.0):
        self._hd.update_problem_data(ws, ys, zs, inv_rho, sigma)

    def backward(self, rho=None):
        self._hd.backward(rho)

    def backward_without_factorization(self, rho=None):
        self._hd.backward_without_factorization(rho)

    def forward(self, x0, ws_out):
        self._hd.forward(x0, ws_out)
        return ws_out

    def synchronize(self):
        self._hd.synchronize()

    def status(self):
        return self._hd.status()

    def admm_solve(self, x0, lb, ub, rho, ws, ys=None, zs=None, sigma: float = 1e-6, alpha: float = 1.6,
                   max_iter: int = 4000, check_every: int = 25, eps_abs: float = 1e-3, eps_rel: float = 1e-3,
                   adaptive_rho: bool = True, adaptive_rho_tolerance: float = 5.0):
        """ADMM outer loop for the box constraints lb <= D w <= ub on the device
        (include/pdplqr.h: pdplqr_admm_solve).  ws/ys/zs hold the warm start and
        are overwritten with the solution; returns admm_info()."""
        st = admm_settings(sigma, alpha, max_iter, check_every, eps_abs, eps_rel, adaptive_rho,
                           adaptive_rho_tolerance)
        self._hd.admm_solve(x0, lb, ub, rho, ws, ys, zs, st)
        return self._hd.admm_info()

    def admm_info(self):
        return self._hd.admm_info()

    def value_function(self, b, k):
        return self._hd.value_function(b, k)

    def close(self):
        self._hd.close()
