"""CPU: the algebraic identities the round-4 stage kernels rely on, checked in
numpy on random data (the kernels themselves are checked against the oracle by
the -m gpu tests; these pin the rearrangements they are built from).

* KKT record (kkt_riccati.hip, PDPLQR_KKT_EHAT): the lambda correction
  x+ = v - rho_dyn (P~ (v - rho_dyn p) + p), v = A x + B u + c, equals
  E^ [u; x] + c^ with E^ = (I - rho_dyn P~) E, c^ = (I - rho_dyn P~)(c - rho_dyn p),
  and the linear ADMM pass's c^ = M^ c - rho_dyn M^ p (M^ = I - rho_dyn P~).
* P~ series by a product tree (PDPLQR_KKT_POW_TREE): the terms
  (-rho_dyn)^j P^{j+1} from P^2 | P^3 = P^2 P, P^4 = P^2 P^2 | P^5..P^8 = P^4 P^{1..4}
  | P^9 = P^8 P equal the chain T_{j+1} = (-rho_dyn P) T_j, and the sum is
  (I + rho_dyn P)^{-1} P to the truncation bound.
* The u-block step with lu carried in W's column 0 (schur_stage.hpp,
  PDPLQR_SCHUR_LPW): with column 0 of the u rows replaced by lu, lane column 0
  forms W_0 = Luu^{-1} lu = lu' and Luu^{-T} W_0 = k~, and M - W W^T keeps the
  value function P_k = Mxx - Mxu Muu^{-1} Mux on the x block while its column 0
  carries lp_x - Lxu lu'.
"""
import numpy as np


def _spd(rng, k, scale=1.0):
    a = rng.standard_normal((k, k))
    return scale * (a @ a.T / k + np.eye(k))


def test_kkt_ehat_record_identity():
    rng = np.random.default_rng(7)
    n, m = 12, 4
    for rd in (1e-6, 0.05, 1.0):
        P = _spd(rng, n, 3.0)
        Pt = np.linalg.solve(np.eye(n) + rd * P, P)  # (I + rho_dyn P)^{-1} P
        E = rng.standard_normal((n, m + n))          # [B A]
        c, p = rng.standard_normal(n), rng.standard_normal(n)
        u, x = rng.standard_normal(m), rng.standard_normal(n)
        v = E @ np.concatenate([u, x]) + c
        ref = v - rd * (Pt @ (v - rd * p) + p)
        Mh = np.eye(n) - rd * Pt
        Eh, ch = Mh @ E, Mh @ (c - rd * p)
        assert np.allclose(Eh @ np.concatenate([u, x]) + ch, ref, rtol=1e-13, atol=1e-13)
        # the linear pass rewrites c^ from the cached M^ and M^ c
        assert np.allclose(Mh @ c - rd * (Mh @ p), ch, rtol=1e-13, atol=1e-13)
        # E^ = E~ - rho_dyn G with G = P~ E~ (what the backward stores)
        assert np.allclose(E - rd * (Pt @ E), Eh, rtol=1e-13, atol=1e-13)


def test_ptilde_power_tree_equals_chain():
    rng = np.random.default_rng(11)
    n = 12
    P = _spd(rng, n, 50.0)
    for e_target in (1e-4, 3e-3, 0.015):
        rd = e_target / np.linalg.norm(P)
        e = rd * np.linalg.norm(P)
        J, ej = 0, e
        while J < 8 and ej > 1e-16:
            J += 1
            ej *= e
        # chain (PDPLQR_KKT_POW_TREE = 0)
        chain, T = P.copy(), P.copy()
        for _ in range(J):
            T = (-rd * P) @ T
            chain += T
        # tree
        Q = {1: P}
        if J >= 1:
            Q[2] = P @ P
        if J >= 2:
            Q[3] = Q[2] @ P
        if J >= 3:
            Q[4] = Q[2] @ Q[2]
        if J >= 4:
            Q[5] = Q[4] @ P
        if J >= 5:
            Q[6] = Q[4] @ Q[2]
        if J >= 6:
            Q[7] = Q[4] @ Q[3]
        if J >= 7:
            Q[8] = Q[4] @ Q[4]
        if J >= 8:
            Q[9] = Q[8] @ P
        tree = P.copy()
        for j in range(J, 0, -1):  # smallest terms first, as the kernel adds them
            tree += (-rd) ** j * Q[j + 1]
        exact = np.linalg.solve(np.eye(n) + rd * P, P)
        assert np.allclose(tree, chain, rtol=1e-14, atol=1e-12 * np.linalg.norm(P))
        assert np.linalg.norm(tree - exact) <= 1e-14 * np.linalg.norm(exact) + e ** (J + 1) / (1 - e) * np.linalg.norm(exact)


def test_u_block_with_lu_in_w():
    rng = np.random.default_rng(3)
    m, n = 4, 12
    s = m + n
    M = _spd(rng, s, 2.0)
    lp = rng.standard_normal(s)
    Muu, Mxu = M[:m, :m], M[m:, :m]
    L = np.linalg.cholesky(Muu)
    lu = lp[:m]
    # reference: the Schur step of lqr_kernel.hpp:104-147 in value form
    luq = np.linalg.solve(L, lu)                       # lu' = Luu^{-1} lu
    Lxu = np.linalg.solve(L, Mxu.T).T                  # Lxu = Mxu Luu^{-T}
    P_ref = M[m:, m:] - Lxu @ Lxu.T
    p_ref = lp[m:] - Lxu @ luq
    K_ref = np.linalg.solve(L.T, Lxu.T)                # K~ = Luu^{-T} Lxu^T
    k_ref = np.linalg.solve(L.T, luq)                  # k~ = Luu^{-T} lu'
    # LPW: the u rows' column 0 replaced by lu before the columns are gathered
    U = M[:m, :].copy()
    U[:, 0] = lu
    W = np.linalg.solve(L, U).T                        # W[c][:] = Luu^{-1} U[:, c] (every lane column c)
    assert np.allclose(W[0], luq)                      # lane column 0: lu'
    Kcols = np.linalg.solve(L.T, W.T)                  # Luu^{-T} W_c per column
    assert np.allclose(Kcols[:, 0], k_ref)             # column 0: k~
    assert np.allclose(Kcols[:, m:], K_ref)            # x columns: K~
    # the tile update: column 0 of M carries lp in, B operand = w everywhere
    T = M.copy()
    T[:, 0] = lp
    D = T - W @ W.T
    assert np.allclose(D[m:, m:], P_ref)               # the value function
    assert np.allclose(D[m:, 0], p_ref)                # column 0, x rows: lp_x - Lxu lu'
