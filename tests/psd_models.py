"""Semidefinite edge cases of the reference's path, as
packed models: zero state cost (Q_k = S_k = 0 and Q_N = 0: every value function
P_k = 0, only the linear costate survives) and a zero terminal cost only
(Q_N = 0).  With sigma = 0 the reference's serial solver handles both (Eigen's
LLT stops at the first non-positive pivot, lqr_kernel.hpp:89,126), the LU
condensed system combines P = 0, and the CHOLESKY one fails (llt of P,
condensed_system.hpp:217-226)."""
import numpy as np


def psd_model(kind, n=12, m=4, N=64, seed=0):
    from pdplqr.model import pack_model
    from pdplqr.problems import random_model

    model, x0 = random_model(n, m, N, seed=seed)
    for k, nd in enumerate(model.nodes):
        if k == N:
            nd.H[:] = 0.0
        elif kind == "zero_state_cost":
            nd.H[m:, :] = 0.0
            nd.H[:, m:] = 0.0
    return pack_model(model), model, x0
