"""numpy restatement of the segment element and its associative combine
(reference lqr_kernel_parallel.hpp:97-135, condensed_system.hpp).
Test infrastructure for the CPU (gloo) check of the horizon-sharding protocol."""
import numpy as np


def combine(a, b):
    """a (x) b, a earlier: Z = (I + C_a P_b)^{-1} (SPD form via R = chol(P_b))."""
    Fa, Ca, fa, Pa, pa = a
    Fb, Cb, fb, Pb, pb = b
    n = Fa.shape[0]
    R = np.linalg.cholesky(Pb)
    Ls = np.linalg.cholesky(np.eye(n) + R.T @ Ca @ R)
    U = np.linalg.solve(Ls, R.T)
    Y = U.T @ U
    Z = np.eye(n) - Ca @ Y
    F = Fb @ Z @ Fa
    C = Fb @ Z @ Ca @ Fb.T + Cb
    f = Fb @ Z @ (fa - Ca @ pb) + fb
    P = Pa + Fa.T @ Y @ Fa
    p = pa + Fa.T @ Z.T @ (pb + Pb @ fa)
    return (F, 0.5 * (C + C.T), f, 0.5 * (P + P.T), p)


def slice_element(E, c, Ht, ht, k0, k1, terminal):
    """Element of stages [k0, k1) from a zero terminal (terminal=None) or the
    real one ((P_N, p_N)); F, C, f by the reference recursion."""
    n = E[0].shape[0]
    m = E[0].shape[1] - n
    if terminal is None:
        P, p, F, C, f = np.zeros((n, n)), np.zeros(n), np.eye(n), np.zeros((n, n)), np.zeros(n)
    else:
        (P, p), F, C, f = terminal, None, None, None
    for k in range(k1 - 1, k0 - 1, -1):
        A, B = E[k][:, m:], E[k][:, :m]
        R_, S_, Q_ = Ht[k][:m, :m], Ht[k][:m, m:], Ht[k][m:, m:]
        b = P @ c[k] + p
        Huu, Hux, gu = R_ + B.T @ P @ B, S_ + B.T @ P @ A, ht[k][:m] + B.T @ b
        K, d = -np.linalg.solve(Huu, Hux), -np.linalg.solve(Huu, gu)
        Pn = Q_ + A.T @ P @ A + Hux.T @ K
        pn = ht[k][m:] + A.T @ b + Hux.T @ d
        if F is not None:
            G = -np.linalg.solve(np.linalg.cholesky(Huu), B.T @ F.T)
            F, f, C = F @ (A + B @ K), F @ (c[k] + B @ d) + f, C + G.T @ G
        P, p = 0.5 * (Pn + Pn.T), pn
    if F is None:
        F, C, f = np.zeros((n, n)), np.zeros((n, n)), np.zeros(n)
    return (F, C, f, P, p)


def pack(e):
    F, C, f, P, p = e
    return np.concatenate([F.ravel(order="F"), C.ravel(order="F"), f, P.ravel(order="F"), p])


def unpack(v, n):
    nn = n * n
    F = v[:nn].reshape(n, n, order="F")
    C = v[nn:2 * nn].reshape(n, n, order="F")
    f = v[2 * nn:2 * nn + n]
    P = v[2 * nn + n:3 * nn + n].reshape(n, n, order="F")
    p = v[3 * nn + n:]
    return (F, C, f, P, p)


def boundary_state(pre, suf, x0):
    """x = (I + C_pre P_suf)^{-1} (F_pre x0 + f_pre - C_pre p_suf)."""
    Fp, Cp, fp, _, _ = pre
    _, _, _, Ps, ps = suf
    n = Fp.shape[0]
    return np.linalg.solve(np.eye(n) + Cp @ Ps, Fp @ x0 + fp - Cp @ ps)


def combine_lu(a, b):
    """a (x) b in the LU form (condensed_system.hpp:82-137): Z = (I + C_a P_b)^{-1}
    by a general solve -- no definiteness needed (P_b, C_a semidefinite)."""
    Fa, Ca, fa, Pa, pa = a
    Fb, Cb, fb, Pb, pb = b
    n = Fa.shape[0]
    Z = np.linalg.solve(np.eye(n) + Ca @ Pb, np.eye(n))
    F = Fb @ Z @ Fa
    C = Fb @ Z @ Ca @ Fb.T + Cb
    f = Fb @ Z @ (fa - Ca @ pb) + fb
    P = Pa + Fa.T @ Pb @ Z @ Fa
    p = pa + Fa.T @ Z.T @ (pb + Pb @ fa)
    return (F, 0.5 * (C + C.T), f, 0.5 * (P + P.T), p)
