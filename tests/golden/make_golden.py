"""Generate the golden fixtures under tests/golden/ (committed, small).

The reference ships no tests or golden vectors and cannot be built here (Eigen3
and QDLDL are absent), so the fixtures come from
independent numpy solves (tests/dense_ref.py): the dense KKT optimum (what the
Riccati solvers compute), the QDLDL-equivalent dense KKT (what QDLDLSolver
computes, with its frozen rho_dyn = sigma = 1e-6) and the textbook Riccati
value functions.  Each fixture stores its inputs (packed model, x0, ADMM
vectors, rho, sigma) and expected outputs.

Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pdp-lqr_amd"), os.path.dirname(HERE)]

from pdplqr.model import initialize_vectors, pack_model  # noqa: E402
from pdplqr.problems import quadrotor_model, random_admm_vectors, random_model  # noqa: E402
import dense_ref as dr  # noqa: E402


def _flat(v):
    return np.concatenate([np.asarray(x, dtype=np.float64).ravel() for x in v]) if len(v) else np.zeros(0)


def make_case(name, model, x0, ws, ys, zs, rho, irho, sigma, pk_list, qdldl=True):
    pm = pack_model(model)
    f = dict(ws=_flat(ws), ys=_flat(ys), zs=_flat(zs), rho=_flat(rho), inv_rho=_flat(irho))
    w_ric = dr.riccati_optimum(pm, x0, f["ws"], f["ys"], f["zs"], f["inv_rho"], f["rho"], sigma)
    P, p = dr.standard_riccati(pm, f["ws"], f["ys"], f["zs"], f["inv_rho"], f["rho"], sigma)
    out = dict(n=pm.n, m=pm.m, N=pm.N, ncs=pm.ncs, E=pm.E, c=pm.c, H=pm.H, h=pm.h, D=pm.D, x0=x0,
               sigma=np.float64(sigma), w_riccati=w_ric, P_k=np.array(pk_list, dtype=np.int32),
               P=np.stack([P[k] for k in pk_list]), p=np.stack([p[k] for k in pk_list]), **f)
    if qdldl:
        out["w_qdldl"] = dr.qdldl_equivalent(pm, x0, f["ws"], f["ys"], f["zs"], f["inv_rho"], sigma)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    print(f"{name}: n={pm.n} m={pm.m} N={pm.N} nc={int(pm.ncs.sum())} |u0|={np.linalg.norm(w_ric[:pm.m]):.6g}")


def main():
    # G1: the reference example, literally (lqr_example.cpp:53-190), rho = 0.01, sigma = 1e-6
    model, x0 = quadrotor_model(100)
    ws, ys, zs, rho, irho = initialize_vectors(model, 0.01)
    make_case("quadrotor_N100", model, x0, ws, ys, zs, rho, irho, 1e-6, [0, 25, 50, 75, 99, 100])

    # G2: BASELINE.json config 1 text: random unconstrained N=100 nx=4 nu=2
    model, x0 = random_model(4, 2, 100, seed=11)
    ws, ys, zs, rho, irho = initialize_vectors(model, 0.1)
    make_case("random_n4_m2_N100", model, x0, ws, ys, zs, rho, irho, 1e-6, [0, 33, 99, 100])

    # G3: constrained 12/4, dense random D, nonzero rho/sigma/y/z/w-bar
    model, x0 = random_model(12, 4, 64, seed=3, nc=4, D_kind="random")
    ws, ys, zs, rho, irho = random_admm_vectors(model, seed=5, rho=0.1)
    make_case("random_n12_m4_N64_nc4", model, x0, ws, ys, zs, rho, irho, 1e-3, [0, 17, 63, 64], qdldl=False)

    # G4: conic config C5 shape (u-box D = [I 0]), short horizon
    model, x0 = random_model(12, 4, 48, seed=7, nc=4, D_kind="ubox")
    ws, ys, zs, rho, irho = random_admm_vectors(model, seed=9, rho=0.1)
    make_case("ubox_n12_m4_N48_nc4", model, x0, ws, ys, zs, rho, irho, 1e-6, [0, 47, 48])

    # G5: config C4 shape (24/8), short horizon
    model, x0 = random_model(24, 8, 40, seed=13)
    ws, ys, zs, rho, irho = initialize_vectors(model, 0.1)
    make_case("random_n24_m8_N40", model, x0, ws, ys, zs, rho, irho, 1e-6, [0, 20, 40], qdldl=False)

    # G6: the example with its constraints enabled (u at k=0, [u;x] after, x at N)
    model, x0 = quadrotor_model(30, nc_on=True)
    ws, ys, zs, rho, irho = random_admm_vectors(model, seed=21, rho=0.1, scale=0.3)
    make_case("quadrotor_N30_constrained", model, x0, ws, ys, zs, rho, irho, 1e-6, [0, 15, 30])

    # G7: a short-segment case (ns = 8 gives Nseg ~ 3) so F, C, f matter
    model, x0 = random_model(6, 3, 26, seed=17)
    ws, ys, zs, rho, irho = initialize_vectors(model, 0.1)
    make_case("random_n6_m3_N26", model, x0, ws, ys, zs, rho, irho, 1e-6, [0, 13, 26])


if __name__ == "__main__":
    main()
