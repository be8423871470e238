"""KKT problems whose lambda elimination leaves the Neumann range.

The Riccati-ordered KKT path (pdp-lqr_amd/csrc/kkt_riccati.hip) forms
P~ = (I + rho_dyn P)^{-1} P per stage.  These cases push e = rho_dyn ||P_k||_F
(the largest over k, measured here with the textbook Riccati of
tests/dense_ref.py) to a chosen size with the three levers the product meets:
a large state cost, state-box rows with a large ADMM penalty (inv_rho small),
and a user-set rho_dyn.
"""
from __future__ import annotations

import numpy as np


def _case_arrays(n, m, N, batch, seed, q_scale, box_irho, nc_rand):
    from pdplqr.problems import random_batch_arrays

    E, c, H, h, x0 = random_batch_arrays(n, m, N, batch, seed)
    s = n + m
    # scale the state block of every stage cost (PSD is kept: q_scale >= 1)
    Hs = H[:, :N * s * s].reshape(batch, N, s, s)  # column-major blocks: [j][i]
    Hs[:, :, m:, m:] *= q_scale
    H[:, :N * s * s] = Hs.reshape(batch, N * s * s)
    H[:, N * s * s:] *= q_scale
    g = np.random.default_rng(seed + 1)
    # per stage: nc_rand random rows, then 2 state-box rows (x_0, x_1) when box_irho
    nbox = 2 if box_irho is not None else 0
    nc = nc_rand + nbox
    ncs = np.full(N + 1, nc, dtype=np.int32)
    Ds, irhos = [], []
    for k in range(N + 1):
        dim = s if k < N else n
        off = m if k < N else 0
        Dk = np.zeros((batch, nc, dim))
        Dk[:, :nc_rand, :] = g.standard_normal((batch, nc_rand, dim))
        for r in range(nbox):
            Dk[:, nc_rand + r, off + r] = 1.0
        Ds.append(np.swapaxes(Dk, 1, 2).reshape(batch, nc * dim))  # column-major
        ir = 0.05 + g.random((batch, nc))
        if nbox:
            ir[:, nc_rand:] = box_irho
        irhos.append(ir)
    D = np.concatenate(Ds, axis=1)
    irho = np.concatenate(irhos, axis=1)
    ny = int(ncs.sum())
    ws = g.standard_normal((batch, N * s + n))
    ys, zs = g.standard_normal((batch, ny)), g.standard_normal((batch, ny))
    return E, c, H, h, x0, ncs, D, ws, ys, zs, irho


# name -> (n, m, N, batch, seed, q_scale, box_irho, nc_rand, rho_dyn); the
# e reached is asserted by the tests (``e_max``)
CASES = {
    "e0.05_state_cost": (12, 4, 24, 2, 3, 2.0e3, None, 4, 1e-6),
    "e0.5_state_box": (12, 4, 24, 2, 4, 1.0, 3e-6, 2, 1e-6),
    "e3_rho_dyn": (12, 4, 24, 2, 5, 1.0, 1e-5, 2, 2e-5),
    "wide_e0.5": (28, 8, 12, 2, 6, 1.0, 3e-6, 2, 1e-6),
    "wide_e3": (28, 8, 12, 2, 7, 1.0, 1e-5, 0, 2e-5),
}
TARGET = {"e0.05_state_cost": 0.05, "e0.5_state_box": 0.5, "e3_rho_dyn": 3.0, "wide_e0.5": 0.5, "wide_e3": 3.0}


def kkt_case(name):
    n, m, N, batch, seed, q_scale, box_irho, nc_rand, rho_dyn = CASES[name]
    arrs = _case_arrays(n, m, N, batch, seed, q_scale, box_irho, nc_rand)
    return (n, m, N, batch, rho_dyn) + arrs


def packed(n, m, N, ncs, E, c, H, h, D, b):
    from pdplqr.model import PackedModel

    return PackedModel(n, m, N, ncs, E[b], c[b], H[b], h[b], D[b])


def e_max(pm, ws, ys, zs, irho, sigma, rho_dyn):
    """rho_dyn max_k ||P_k||_F of the penalised problem (textbook Riccati)."""
    from dense_ref import standard_riccati

    P, _ = standard_riccati(pm, ws, ys, zs, irho, 1.0 / irho, sigma)
    return rho_dyn * max(np.linalg.norm(Pk) for Pk in P[1:])
