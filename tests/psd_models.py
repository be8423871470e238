"""Semidefinite edge cases of the reference's path, as
packed models: zero state cost (Q_k = S_k = 0 and Q_N = 0: every value function
P_k = 0, only the linear costate survives) and a zero terminal cost only
(Q_N = 0).  With sigma = 0 the reference's serial solver handles both (Eigen's
LLT stops at the first non-positive pivot, lqr_kernel.hpp:89,126), the LU
condensed system combines P = 0, and the CHOLESKY one fails (llt of P,
condensed_system.hpp:217-226).

"coupled_dead_terminal" (ADVICE r2): Q_N is the identity except that state 1
has no cost and states 0 and 2 are coupled (Q_N[0,2] = 0.8).  Its second
pivot is exactly 0 AFTER the first pivot has reduced the trailing block, so
Eigen's left-looking LLT stops there with columns >= 1 at their ORIGINAL
values: the reference's L_N is not a factor of Q_N (L_N L_N^T has 1.64 at
(2, 2)), and every L-form path must reproduce that L_N."""
import numpy as np


def psd_model(kind, n=12, m=4, N=64, seed=0):
    from pdplqr.model import pack_model
    from pdplqr.problems import random_model

    model, x0 = random_model(n, m, N, seed=seed)
    for k, nd in enumerate(model.nodes):
        if k == N and kind == "coupled_dead_terminal":
            nd.H[:] = np.eye(n)
            nd.H[1, 1] = 0.0
            nd.H[0, 2] = nd.H[2, 0] = 0.8
        elif k == N:
            nd.H[:] = 0.0
        elif kind == "zero_state_cost":
            nd.H[m:, :] = 0.0
            nd.H[:, m:] = 0.0
    return pack_model(model), model, x0


def eigen_stop_factor(Q):
    """Eigen's llt_inplace::unblocked on Q (left-looking): the lower triangle it
    leaves, including the untouched columns after a pivot <= 0 (the restated
    semantics the tests pin; the reference ignores info())."""
    Q = np.array(Q, dtype=np.float64)
    n = Q.shape[0]
    L = np.tril(Q).copy()
    for k in range(n):
        x = Q[k, k] - L[k, :k] @ L[k, :k]
        if x <= 0.0:
            return L
        L[k, k] = np.sqrt(x)
        L[k + 1:, k] = (Q[k + 1:, k] - L[k + 1:, :k] @ L[k, :k]) / L[k, k]
    return L


def decoupled_dead_state(n, m, N, batch, seed, k):
    """State k decoupled (x_{t+1}[k] = x_t[k], no input, no offset) and
    costless in every stage and the terminal: with sigma = 0 every value
    function has a zero pivot at state k, so Eigen's LLT stops there -- in
    the terminal factor (order n) and at pivot m + k of every stage."""
    from pdplqr.problems import random_batch_arrays

    E, c, H, h, x0 = random_batch_arrays(n, m, N, batch, seed)
    s = n + m
    E, c, H, h = E.copy(), c.copy(), H.copy(), h.copy()
    for b in range(batch):
        for t in range(N):
            Et = E[b, t * n * s:(t + 1) * n * s].reshape(n, s, order="F")  # [B A], column-major
            Et[k, :] = 0.0
            Et[:, m + k] = 0.0
            Et[k, m + k] = 1.0
            E[b, t * n * s:(t + 1) * n * s] = Et.ravel(order="F")
            c[b, t * n + k] = 0.0
            Ht = H[b, t * s * s:(t + 1) * s * s].reshape(s, s, order="F")
            Ht[m + k, :] = 0.0
            Ht[:, m + k] = 0.0
            H[b, t * s * s:(t + 1) * s * s] = Ht.ravel(order="F")
            h[b, t * s + m + k] = 0.0
        HN = H[b, N * s * s:].reshape(n, n, order="F")
        HN[k, :] = 0.0
        HN[:, k] = 0.0
        H[b, N * s * s:] = HN.ravel(order="F")
        h[b, N * s + k] = 0.0
    return E, c, H, h, x0
