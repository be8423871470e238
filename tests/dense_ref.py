"""Independent numpy solvers used to generate and check golden fixtures.

These are NOT restatements of the reference algorithm.  They compute the same
mathematical objects by different routes, so they pin the oracle:

* ``dense_kkt_solve``: assembles the full symmetric KKT matrix of the LQ problem
  in the reference's variable order (``kkt.hpp:124-205``) and solves it with
  LAPACK.  With ``rho_dyn = 0`` and the Riccati's data conventions it is the
  exact optimum the Riccati solvers compute; with the ``QDLDLSolver`` quirks
  (``rho_dyn = sigma_K = 1e-6`` frozen into the matrix, ``qdldl_solver.hpp:38-41``;
  stage-0 ``Dx0 x0`` dropped from the rhs, ``kkt.hpp:218-221``) it is the
  QDLDL-equivalent answer.
* ``standard_riccati``: textbook (non-square-root) Riccati recursion giving the
  value function ``(P_k, p_k)`` for the ``P = Lxx Lxx^T`` parity check.
"""
from __future__ import annotations

import numpy as np


def _blocks(pm):
    n, m, N = pm.n, pm.m, pm.N
    s = n + m
    E = [pm.E[k * n * s:(k + 1) * n * s].reshape(n, s, order="F") for k in range(N)]
    c = [pm.c[k * n:(k + 1) * n] for k in range(N)]
    H = [pm.H[k * s * s:(k + 1) * s * s].reshape(s, s, order="F") for k in range(N)]
    H.append(pm.H[N * s * s:].reshape(n, n, order="F"))
    h = [pm.h[k * s:(k + 1) * s] for k in range(N)] + [pm.h[N * s:]]
    D = []
    off = 0
    for k in range(N + 1):
        dim = s if k < N else n
        nc = int(pm.ncs[k])
        D.append(pm.D[off:off + nc * dim].reshape(nc, dim, order="F"))
        off += nc * dim
    return E, c, H, h, D


def _stagevecs(flat, sizes):
    out, o = [], 0
    for sz in sizes:
        out.append(np.asarray(flat[o:o + sz], dtype=np.float64))
        o += sz
    return out


def effective_cost(pm, ws, ys, zs, inv_rho, rho, sigma):
    """H~_k, h~_k of the Riccati solvers: update_problem_data (lqr_solver.hpp:41-56)
    followed by the rho penalty of backward (lqr_kernel.hpp:82-88,106-112)."""
    n, m, N = pm.n, pm.m, pm.N
    s = n + m
    E, c, H, h, D = _blocks(pm)
    wl = _stagevecs(ws, [s] * N + [n])
    ncs = [int(x) for x in pm.ncs]
    yl, zl, irl, rl = (_stagevecs(v, ncs) for v in (ys, zs, inv_rho, rho))
    Ht, ht = [], []
    for k in range(N + 1):
        dim = s if k < N else n
        Hk = H[k] + sigma * np.eye(dim)
        hk = h[k] - sigma * wl[k]
        if ncs[k] > 0:
            g = zl[k] - irl[k] * yl[k]
            Hk = Hk + D[k].T @ np.diag(rl[k]) @ D[k]
            hk = hk - D[k].T @ (rl[k] * g)
        Ht.append(Hk)
        ht.append(hk)
    return E, c, Ht, ht


def riccati_optimum(pm, x0, ws, ys, zs, inv_rho, rho, sigma):
    """Exact optimum of min sum 1/2 w^T H~ w + h~^T w s.t. dynamics, x0 fixed,
    by a dense solve over [u0, x1, u1, ..., x_{N-1}, u_{N-1}, x_N] and costates.
    Returns the flat ws vector ([u;x] per stage, x_N last)."""
    n, m, N = pm.n, pm.m, pm.N
    s = n + m
    E, c, Ht, ht = effective_cost(pm, ws, ys, zs, inv_rho, rho, sigma)
    nprim = N * s  # u0 (m) + (N-1)*s + n
    ndual = N * n
    K = np.zeros((nprim + ndual, nprim + ndual))
    r = np.zeros(nprim + ndual)
    # primal index of u_k and x_k
    def ui(k):
        return 0 if k == 0 else m + (k - 1) * s + n

    def xi(k):
        return None if k == 0 else m + (k - 1) * s

    for k in range(N + 1):
        Hk, hk = Ht[k], ht[k]
        if k == 0:
            Ru = Hk[:m, :m]
            K[0:m, 0:m] += Ru
            r[0:m] -= hk[:m] + Hk[:m, m:] @ x0
        elif k < N:
            idx = np.r_[ui(k):ui(k) + m, xi(k):xi(k) + n]
            K[np.ix_(idx, idx)] += Hk
            r[idx] -= hk
        else:
            idx = np.arange(xi(N), xi(N) + n)
            K[np.ix_(idx, idx)] += Hk
            r[idx] -= hk
    for k in range(N):
        A = E[k][:, m:]
        B = E[k][:, :m]
        lam = nprim + k * n
        # x_{k+1} - A x_k - B u_k = c_k
        rows = np.arange(lam, lam + n)
        xn = np.arange(xi(k + 1), xi(k + 1) + n)
        K[np.ix_(rows, xn)] += np.eye(n)
        K[np.ix_(xn, rows)] += np.eye(n)
        uu = np.arange(ui(k), ui(k) + m)
        K[np.ix_(rows, uu)] -= B
        K[np.ix_(uu, rows)] -= B.T
        rhs = c[k].copy()
        if k == 0:
            rhs = rhs + A @ x0
        else:
            xx = np.arange(xi(k), xi(k) + n)
            K[np.ix_(rows, xx)] -= A
            K[np.ix_(xx, rows)] -= A.T
        r[rows] = rhs
    sol = np.linalg.solve(K, r)
    out = np.zeros(N * s + n)
    out[m:s] = x0
    out[0:m] = sol[0:m]
    for k in range(1, N):
        out[k * s:k * s + m] = sol[ui(k):ui(k) + m]
        out[k * s + m:(k + 1) * s] = sol[xi(k):xi(k) + n]
    out[N * s:] = sol[xi(N):xi(N) + n]
    return out


def qdldl_equivalent(pm, x0, ws, ys, zs, inv_rho, sigma_rhs, rho_dyn=1e-6, sigma_mat=1e-6):
    """Dense solve of the KKT the reference's QDLDLSolver factors
    (kkt.hpp:124-300, qdldl_solver.hpp:36-151): natural order
    [u0, x1,u1, ..., x_N | y0, lam1,y1, ..., lamN,yN], sigma_mat on the H
    diagonals, -rho_dyn on the lambda diagonals, -inv_rho on the y diagonals,
    rhs from form_rhs (with sigma_rhs) plus update_rhs_initial_stage."""
    n, m, N = pm.n, pm.m, pm.N
    s = n + m
    E, c, H, h, D = _blocks(pm)
    ncs = [int(x) for x in pm.ncs]
    wl = _stagevecs(ws, [s] * N + [n])
    yl, zl, irl = (_stagevecs(v, ncs) for v in (ys, zs, inv_rho))
    nprim = N * s
    dim = nprim + sum(ncs) + N * n
    K = np.zeros((dim, dim))
    r = np.zeros(dim)

    def pidx(k):  # primal rows of stage k in KKT order (x first for k >= 1)
        if k == 0:
            return np.arange(0, m), None
        base = m + (k - 1) * s
        if k < N:
            return np.arange(base + n, base + s), np.arange(base, base + n)
        return None, np.arange(base, base + n)

    # dual offsets
    yoff, loff = [], [None]
    o = nprim
    yoff.append(o)
    o += ncs[0]
    for k in range(1, N + 1):
        loff.append(o)
        o += n
        yoff.append(o)
        o += ncs[k]
    for k in range(N + 1):
        ur, xr = pidx(k)
        if k < N:
            Hk = H[k] + sigma_mat * np.eye(s)
            if ur is not None:
                K[np.ix_(ur, ur)] += Hk[:m, :m]
            if xr is not None:
                K[np.ix_(xr, xr)] += Hk[m:, m:]
                K[np.ix_(xr, ur)] += Hk[m:, :m]
                K[np.ix_(ur, xr)] += Hk[:m, m:]
            # rhs
            r[ur] = -h[k][:m] + sigma_rhs * wl[k][:m]
            if xr is not None:
                r[xr] = -h[k][m:] + sigma_rhs * wl[k][m:]
            # dynamics duals lam_{k+1}
            lr = np.arange(loff[k + 1], loff[k + 1] + n)
            A, B = E[k][:, m:], E[k][:, :m]
            K[np.ix_(lr, ur)] += B
            K[np.ix_(ur, lr)] += B.T
            if xr is not None:
                K[np.ix_(lr, xr)] += A
                K[np.ix_(xr, lr)] += A.T
            r[lr] = -c[k]
            if k == 0:
                r[lr] += -A @ x0
                r[ur] += -H[0][:m, m:] @ x0
        else:
            HN = H[N] + sigma_mat * np.eye(n)
            K[np.ix_(xr, xr)] += HN
            r[xr] = -h[N] + sigma_rhs * wl[N]
        if k >= 1:  # -I coupling of x_k with lam_k
            lr = np.arange(loff[k], loff[k] + n)
            K[np.ix_(lr, xr)] -= np.eye(n)
            K[np.ix_(xr, lr)] -= np.eye(n)
            K[np.ix_(lr, lr)] -= rho_dyn * np.eye(n)
        if ncs[k] > 0:
            yr = np.arange(yoff[k], yoff[k] + ncs[k])
            Dk = D[k]
            if k == 0:
                K[np.ix_(yr, ur)] += Dk[:, :m]
                K[np.ix_(ur, yr)] += Dk[:, :m].T
            elif k < N:
                K[np.ix_(yr, ur)] += Dk[:, :m]
                K[np.ix_(ur, yr)] += Dk[:, :m].T
                K[np.ix_(yr, xr)] += Dk[:, m:]
                K[np.ix_(xr, yr)] += Dk[:, m:].T
            else:
                K[np.ix_(yr, xr)] += Dk
                K[np.ix_(xr, yr)] += Dk.T
            K[np.ix_(yr, yr)] -= np.diag(irl[k])
            r[yr] = zl[k] - irl[k] * yl[k]
    sol = np.linalg.solve(K, r)
    out = np.zeros(N * s + n)
    out[m:s] = x0
    out[0:m] = sol[0:m]
    for k in range(1, N):
        ur, xr = pidx(k)
        out[k * s:k * s + m] = sol[ur]
        out[k * s + m:(k + 1) * s] = sol[xr]
    out[N * s:] = sol[pidx(N)[1]]
    return out


def standard_riccati(pm, ws, ys, zs, inv_rho, rho, sigma):
    """Value functions (P_k, p_k), k = 0..N, by the textbook Riccati recursion."""
    n, m, N = pm.n, pm.m, pm.N
    E, c, Ht, ht = effective_cost(pm, ws, ys, zs, inv_rho, rho, sigma)
    P = [None] * (N + 1)
    p = [None] * (N + 1)
    P[N] = Ht[N].copy()
    p[N] = ht[N].copy()
    for k in range(N - 1, -1, -1):
        A, B = E[k][:, m:], E[k][:, :m]
        R, S, Q = Ht[k][:m, :m], Ht[k][:m, m:], Ht[k][m:, m:]
        r_, q_ = ht[k][:m], ht[k][m:]
        Pn, pn = P[k + 1], p[k + 1]
        b = Pn @ c[k] + pn
        Huu = R + B.T @ Pn @ B
        Hux = S + B.T @ Pn @ A
        gu = r_ + B.T @ b
        Kk = -np.linalg.solve(Huu, Hux)
        dk = -np.linalg.solve(Huu, gu)
        P[k] = Q + A.T @ Pn @ A + Hux.T @ Kk
        P[k] = 0.5 * (P[k] + P[k].T)
        p[k] = q_ + A.T @ b + Hux.T @ dk
    return P, p
