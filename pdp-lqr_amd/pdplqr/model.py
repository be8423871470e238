"""Problem model: ``Node`` and ``LQRModel``, mirroring the reference's
``include/clqr/lqr_model.hpp`` (``Node`` :8-64, ``LQRModel`` :66-89), plus the
flat packing used at the C-ABI boundary (``include/pdplqr.h``).

Stage variables are ordered ``w_k = [u_k; x_k]`` (control first), exactly as the
reference (``lqr_model.hpp:14,18-19``).  Matrices are numpy ``float64`` arrays; the
packed form is Eigen column-major (Fortran order) per block, stage-major.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

LQR_INFTY = float("inf")  # typedefs.hpp:23


class Node:
    """One stage of the horizon (``lqr_model.hpp:8-64``).

    ``E = [B A]`` (n x (n+m)), ``c`` (n), ``H = [R S; S^T Q]`` ((n+m)^2),
    ``h = [r; q]``, ``D_con = [Du Dx]`` (nc x (n+m)), ``e_lb``/``e_ub`` (nc).
    The terminal node holds ``H = Q_N`` (n x n) and ``h = q_N`` only.
    """

    def __init__(self, state_dim: int, control_dim: int, n_constraints: int, time_step: int,
                 is_terminal_stage: bool = False):
        self.n = int(state_dim)
        self.m = int(control_dim)
        self.n_con = int(n_constraints)
        self.is_terminal = bool(is_terminal_stage)
        self.time_step = int(time_step)
        n, m = self.n, self.m
        dim = n if self.is_terminal else n + m
        if self.is_terminal:
            self.E = np.zeros((0, 0))
            self.c = np.zeros(0)
        else:
            self.E = np.zeros((n, n + m))
            self.c = np.zeros(n)
        self.H = np.zeros((dim, dim))
        self.h = np.zeros(dim)
        if self.n_con > 0:
            self.D_con = np.zeros((self.n_con, dim))
            self.e_lb = np.zeros(self.n_con)
            self.e_ub = np.zeros(self.n_con)
        else:
            self.D_con = np.zeros((0, dim))
            self.e_lb = np.zeros(0)
            self.e_ub = np.zeros(0)

    def set_zero(self) -> None:  # lqr_model.hpp:49-61
        if not self.is_terminal:
            self.E[:] = 0.0
            self.c[:] = 0.0
        self.H[:] = 0.0
        self.h[:] = 0.0
        self.D_con[:] = 0.0
        self.e_lb[:] = 0.0
        self.e_ub[:] = 0.0

    def get_constraint_dim(self) -> int:
        return self.n_con


class LQRModel:
    """Horizon container (``lqr_model.hpp:66-89``).  ``add_node`` appends in call
    order and sets ``ncs[time_step]`` (:85-88).  Raises for ``N < 1`` (:75-77)."""

    def __init__(self, n: int, m: int, horizon: int):
        if horizon < 1:
            raise RuntimeError("Horizon must be at least 1.")
        self.n = int(n)
        self.m = int(m)
        self.N = int(horizon)
        self.ncs = [0] * (self.N + 1)
        self.nodes: List[Node] = []

    def get_node(self, k: int) -> Node:
        return self.nodes[k]

    def add_node(self, n: int, m: int, nc: int, time_step: int, is_terminal_stage: bool = False) -> None:
        self.nodes.append(Node(n, m, nc, time_step, is_terminal_stage))
        self.ncs[time_step] = nc


@dataclass
class PackedModel:
    """Flat, stage-major, Eigen column-major packing of one problem (the
    boundary format of ``pdplqr_set_model``)."""

    n: int
    m: int
    N: int
    ncs: np.ndarray  # int32 (N+1)
    E: np.ndarray  # N * n*s
    c: np.ndarray  # N * n
    H: np.ndarray  # N * s*s + n*n
    h: np.ndarray  # N * s + n
    D: np.ndarray  # sum_k nc_k * dim_k

    @property
    def s(self) -> int:
        return self.n + self.m

    @property
    def y_off(self) -> np.ndarray:
        return np.concatenate([[0], np.cumsum(self.ncs)]).astype(np.int64)


def _fortran_flat(a: np.ndarray) -> np.ndarray:
    return np.asarray(a, dtype=np.float64).reshape(-1, order="F")


def pack_model(model: LQRModel) -> PackedModel:
    """Pack ``model.nodes`` (in index order, as the reference iterates them) into
    the flat boundary arrays."""
    n, m, N = model.n, model.m, model.N
    s = n + m
    if len(model.nodes) != N + 1:
        raise RuntimeError(f"model has {len(model.nodes)} nodes, expected N+1 = {N + 1}")
    E = np.empty(N * n * s)
    c = np.empty(N * n)
    H = np.empty(N * s * s + n * n)
    h = np.empty(N * s + n)
    ncs = np.array([model.nodes[k].n_con for k in range(N + 1)], dtype=np.int32)
    D_parts = []
    for k in range(N + 1):
        nd = model.nodes[k]
        if k < N:
            E[k * n * s:(k + 1) * n * s] = _fortran_flat(nd.E)
            c[k * n:(k + 1) * n] = nd.c
            H[k * s * s:(k + 1) * s * s] = _fortran_flat(nd.H)
            h[k * s:(k + 1) * s] = nd.h
        else:
            H[N * s * s:] = _fortran_flat(nd.H)
            h[N * s:] = nd.h
        if nd.n_con > 0:
            D_parts.append(_fortran_flat(nd.D_con))
    D = np.concatenate(D_parts) if D_parts else np.zeros(0)
    return PackedModel(n, m, N, ncs, E, c, H, h, D)


def pack_stage_vectors(vecs: Sequence[np.ndarray], sizes: Sequence[int]) -> np.ndarray:
    """Concatenate a ``std::vector<VectorXs>``-like list after checking sizes."""
    out = []
    for k, (v, sz) in enumerate(zip(vecs, sizes)):
        v = np.asarray(v, dtype=np.float64).reshape(-1)
        if v.size != sz:
            raise ValueError(f"vector {k} has size {v.size}, expected {sz}")
        out.append(v)
    return np.concatenate(out) if out else np.zeros(0)


def w_sizes(n: int, m: int, N: int) -> List[int]:
    return [n + m] * N + [n]


def unpack_ws(flat: np.ndarray, n: int, m: int, N: int) -> List[np.ndarray]:
    s = n + m
    return [flat[k * s:(k + 1) * s].copy() for k in range(N)] + [flat[N * s:N * s + n].copy()]


def initialize_vectors(model: LQRModel, rho: float):
    """``initialize_vectors`` of ``examples/lqr_example.cpp:12-46``."""
    n, m, N = model.n, model.m, model.N
    ws = [np.zeros(n + m) for _ in range(N)] + [np.zeros(n)]
    ys = [np.zeros(model.ncs[k]) for k in range(N + 1)]
    zs = [np.zeros(model.ncs[k]) for k in range(N + 1)]
    rho_vecs = [np.full(model.ncs[k], rho) for k in range(N + 1)]
    inv_rho_vecs = [np.full(model.ncs[k], 1.0 / rho) for k in range(N + 1)]
    return ws, ys, zs, rho_vecs, inv_rho_vecs


def unpack_model(pm: PackedModel) -> LQRModel:
    """Inverse of ``pack_model`` (nodes in time order)."""
    n, m, N = pm.n, pm.m, pm.N
    s = n + m
    model = LQRModel(n, m, N)
    off = 0
    for k in range(N + 1):
        nc = int(pm.ncs[k])
        model.add_node(n, m, nc, k, k == N)
        nd = model.nodes[k]
        if k < N:
            nd.E[:] = pm.E[k * n * s:(k + 1) * n * s].reshape(n, s, order="F")
            nd.c[:] = pm.c[k * n:(k + 1) * n]
            nd.H[:] = pm.H[k * s * s:(k + 1) * s * s].reshape(s, s, order="F")
            nd.h[:] = pm.h[k * s:(k + 1) * s]
        else:
            nd.H[:] = pm.H[N * s * s:].reshape(n, n, order="F")
            nd.h[:] = pm.h[N * s:]
        dim = s if k < N else n
        if nc > 0:
            nd.D_con[:] = pm.D[off:off + nc * dim].reshape(nc, dim, order="F")
            off += nc * dim
    return model
