"""Problem generators: the reference example (quadrotor MPC,
``examples/lqr_example.cpp:53-168``) and the seeded synthetic LQR distribution
of ``BASELINE.md`` section 3 / ``SURVEY.md`` section 8(d):

    A = I + 0.1 N(0,1), B ~ N(0,1), c ~ N(0,1),
    H = M M^T / s + I (M ~ N(0,1) s x s), h ~ N(0,1),
    Q_N = M M^T / n + I, x0 ~ N(0,1), nc = 0 unless stated.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np

from .model import LQR_INFTY, LQRModel


def quadrotor_model(N: int = 100, nc_on: bool = False) -> Tuple[LQRModel, np.ndarray]:
    """The reference example problem (``lqr_example.cpp:53-168``).  Constraints
    are disabled there (``nc = 0``, :127,158); ``nc_on`` re-enables the box
    constraints the example builds (u at stage 0, u and x after, x at N)."""
    nx, nu = 12, 4
    x0 = np.zeros(nx)
    x_ref = np.array([0.0, 0.0, 1.0, 0, 0, 0, 0, 0, 0, 0, 0, 0])
    x_min = np.array([-0.52359878, -0.52359878, -LQR_INFTY, -LQR_INFTY, -LQR_INFTY, -1.0,
                      -LQR_INFTY, -LQR_INFTY, -LQR_INFTY, -LQR_INFTY, -LQR_INFTY, -LQR_INFTY])
    x_max = np.array([0.52359878, 0.52359878, LQR_INFTY, LQR_INFTY, LQR_INFTY, LQR_INFTY,
                      LQR_INFTY, LQR_INFTY, 2.5, LQR_INFTY, LQR_INFTY, LQR_INFTY])
    u_min = np.full(nu, -0.9916)
    u_max = np.full(nu, 2.4084)
    A = np.array([
        [1., 0., 0., 0., 0., 0., 0.1, 0., 0., 0., 0., 0.],
        [0., 1., 0., 0., 0., 0., 0., 0.1, 0., 0., 0., 0.],
        [0., 0., 1., 0., 0., 0., 0., 0., 0.1, 0., 0., 0.],
        [0.0488, 0., 0., 1., 0., 0., 0.0016, 0., 0., 0.0992, 0., 0.],
        [0., -0.0488, 0., 0., 1., 0., 0., -0.0016, 0., 0., 0.0992, 0.],
        [0., 0., 0., 0., 0., 1., 0., 0., 0., 0., 0., 0.0992],
        [0., 0., 0., 0., 0., 0., 1., 0., 0., 0., 0., 0.],
        [0., 0., 0., 0., 0., 0., 0., 1., 0., 0., 0., 0.],
        [0., 0., 0., 0., 0., 0., 0., 0., 1., 0., 0., 0.],
        [0.9734, 0., 0., 0., 0., 0., 0.0488, 0., 0., 0.9846, 0., 0.],
        [0., -0.9734, 0., 0., 0., 0., 0., -0.0488, 0., 0., 0.9846, 0.],
        [0., 0., 0., 0., 0., 0., 0., 0., 0., 0., 0., 0.9846]])
    B = np.array([
        [0., -0.0726, 0., 0.0726],
        [-0.0726, 0., 0.0726, 0.],
        [-0.0152, 0.0152, -0.0152, 0.0152],
        [-0., -0.0006, -0., 0.0006],
        [0.0006, 0., -0.0006, 0.0000],
        [0.0106, 0.0106, 0.0106, 0.0106],
        [0., -1.4512, 0., 1.4512],
        [-1.4512, 0., 1.4512, 0.],
        [-0.3049, 0.3049, -0.3049, 0.3049],
        [-0., -0.0236, 0., 0.0236],
        [0.0236, 0., -0.0236, 0.],
        [0.2107, 0.2107, 0.2107, 0.2107]])
    c = np.zeros(nx)
    Q = np.diag([0., 0., 10., 10., 10., 10., 0., 0., 0., 5., 5., 5.])
    R = np.diag([0.1] * 4)
    S = np.zeros((nu, nx))
    q = -x_ref @ Q
    r = np.zeros(nu)
    model = LQRModel(nx, nu, N)
    for k in range(N):
        nc = (nx + nu if k > 0 else nu) if nc_on else 0
        model.add_node(nx, nu, nc, k)
        kp = model.nodes[k]
        kp.E[:, :nu] = B
        kp.E[:, nu:] = A
        kp.c[:] = c
        kp.H[:nu, :nu] = R
        kp.H[nu:, nu:] = Q
        kp.H[:nu, nu:] = S
        kp.H[nu:, :nu] = S.T
        kp.h[:nu] = r
        kp.h[nu:] = q
        if nc > 0:
            kp.D_con[:] = 0.0
            kp.D_con[:nu, :nu] = np.eye(nu)
            if k == 0:
                kp.e_lb[:] = u_min
                kp.e_ub[:] = u_max
            else:
                kp.D_con[nu:, nu:] = np.eye(nx)
                kp.e_lb[:] = np.concatenate([u_min, x_min])
                kp.e_ub[:] = np.concatenate([u_max, x_max])
    ncN = nx if nc_on else 0
    model.add_node(nx, nu, ncN, N, True)
    kp = model.nodes[N]
    kp.H[:] = Q
    kp.h[:] = q
    if ncN > 0:
        kp.D_con[:] = np.eye(nx)
        kp.e_lb[:] = x_min
        kp.e_ub[:] = x_max
    return model, x0


def random_model(n: int, m: int, N: int, seed: int = 0, nc: int = 0, D_kind: str = "random",
                 rng: Optional[np.random.Generator] = None) -> Tuple[LQRModel, np.ndarray]:
    """Synthetic LQR of the BASELINE.md section 3 distribution.  ``nc > 0`` adds
    ``nc`` constraint rows per stage; ``D_kind='ubox'`` uses ``D = [I 0]`` (box on
    u, as config C5), ``'random'`` a dense N(0,1) ``D``."""
    g = rng if rng is not None else np.random.default_rng(seed)
    s = n + m
    model = LQRModel(n, m, N)
    for k in range(N + 1):
        term = k == N
        model.add_node(n, m, nc, k, term)
        kp = model.nodes[k]
        if not term:
            A = np.eye(n) + 0.1 * g.standard_normal((n, n))
            B = g.standard_normal((n, m))
            kp.E[:, :m] = B
            kp.E[:, m:] = A
            kp.c[:] = g.standard_normal(n)
            M = g.standard_normal((s, s))
            kp.H[:] = M @ M.T / s + np.eye(s)
            kp.h[:] = g.standard_normal(s)
        else:
            M = g.standard_normal((n, n))
            kp.H[:] = M @ M.T / n + np.eye(n)
            kp.h[:] = g.standard_normal(n)
        if nc > 0:
            dim = n if term else s
            if D_kind == "ubox" and not term:
                kp.D_con[:] = 0.0
                kp.D_con[:min(nc, m), :min(nc, m)] = np.eye(min(nc, m))
            elif D_kind == "ubox" and term:
                kp.D_con[:] = 0.0
                kp.D_con[:min(nc, n), :min(nc, n)] = np.eye(min(nc, n))
            else:
                kp.D_con[:] = g.standard_normal((nc, dim))
            kp.e_lb[:] = -1.0
            kp.e_ub[:] = 1.0
    x0 = g.standard_normal(n)
    return model, x0


def random_admm_vectors(model: LQRModel, seed: int = 1, rho: float = 0.1, scale: float = 1.0):
    """Random ADMM iterate data (w-bar, y, z) and constant rho vectors for a model,
    as the conic config C5 uses (random y, z, w-bar, rho = 0.1)."""
    g = np.random.default_rng(seed)
    n, m, N = model.n, model.m, model.N
    ws = [scale * g.standard_normal(n + m) for _ in range(N)] + [scale * g.standard_normal(n)]
    ys = [scale * g.standard_normal(model.ncs[k]) for k in range(N + 1)]
    zs = [scale * g.standard_normal(model.ncs[k]) for k in range(N + 1)]
    rho_vecs = [np.full(model.ncs[k], rho) for k in range(N + 1)]
    inv_rho = [np.full(model.ncs[k], 1.0 / rho) for k in range(N + 1)]
    return ws, ys, zs, rho_vecs, inv_rho


def random_batch_arrays(n: int, m: int, N: int, batch: int, seed: int = 0):
    """Batched synthetic data as flat boundary arrays, batch-major:
    E (batch, N*n*s), c (batch, N*n), H (batch, N*s*s + n*n), h (batch, N*s + n),
    x0 (batch, n).  Same distribution as ``random_model``."""
    g = np.random.default_rng(seed)
    s = n + m
    A = np.eye(n)[None, None] + 0.1 * g.standard_normal((batch, N, n, n))
    B = g.standard_normal((batch, N, n, m))
    E = np.concatenate([B, A], axis=3)  # (batch, N, n, s)
    c = g.standard_normal((batch, N, n))
    M = g.standard_normal((batch, N, s, s))
    H = M @ np.swapaxes(M, -1, -2) / s + np.eye(s)
    h = g.standard_normal((batch, N, s))
    MN = g.standard_normal((batch, n, n))
    HN = MN @ np.swapaxes(MN, -1, -2) / n + np.eye(n)
    hN = g.standard_normal((batch, n))
    x0 = g.standard_normal((batch, n))
    Ef = np.swapaxes(E, -1, -2).reshape(batch, N * n * s)  # column-major blocks
    Hf = np.concatenate([np.swapaxes(H, -1, -2).reshape(batch, N * s * s),
                         np.swapaxes(HN, -1, -2).reshape(batch, n * n)], axis=1)
    hf = np.concatenate([h.reshape(batch, N * s), hN], axis=1)
    return (np.ascontiguousarray(Ef), np.ascontiguousarray(c.reshape(batch, N * n)), np.ascontiguousarray(Hf),
            np.ascontiguousarray(hf), np.ascontiguousarray(x0))
