"""The facade's public KKT surface on the host (include/clqr/lqr/kkt.hpp:
KKTSystem::form_KKT_matrix / get_KKT_csc_matrix / form_rhs /
update_rhs_initial_stage and QDLDLSolver::create_workspace's elimination
tree; reference kkt.hpp:7-331, qdldl_solver.hpp:19,47-78) against the oracle's
restatement of the same assembly (orc_kkt_*: CSC pattern and values, the
right-hand side after one forward, QDLDL_etree's sum of column counts).
CPU only: g++ builds tests/cpp/kkt_check.cpp against the headers."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import ROOT, golden_names, load_golden


@pytest.fixture(scope="module")
def kkt_check(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ missing")
    exe = str(tmp_path_factory.mktemp("kkt") / "kkt_check")
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-DPDPLQR_NO_EIGEN", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "cpp", "kkt_check.cpp"), "-o", exe])
    return exe


def _run(exe, tmp, pm, ws, ys, zs, irho, x0, sigma, rho_dyn=1e-6, sigma_mat=1e-6):
    fin, fout = str(tmp / "in.bin"), str(tmp / "out.bin")
    with open(fin, "wb") as f:
        np.array([pm.n, pm.m, pm.N], dtype=np.int32).tofile(f)
        pm.ncs.astype(np.int32).tofile(f)
        for a in (pm.E, pm.c, pm.H, pm.h, pm.D, ws, ys, zs, irho, x0, np.array([sigma, rho_dyn, sigma_mat])):
            np.ascontiguousarray(a, dtype=np.float64).tofile(f)
    subprocess.check_call([exe, fin, fout])
    with open(fout, "rb") as f:
        dim, nnz, sumLnz = np.fromfile(f, dtype=np.int64, count=3)
        Ap = np.fromfile(f, dtype=np.int64, count=dim + 1)
        Ai = np.fromfile(f, dtype=np.int64, count=nnz)
        Ax = np.fromfile(f, dtype=np.float64, count=nnz)
        rhs = np.fromfile(f, dtype=np.float64, count=dim)
        Lnz = np.fromfile(f, dtype=np.int64, count=dim)
        etree = np.fromfile(f, dtype=np.int64, count=dim)
    return int(dim), Ap, Ai, Ax, rhs, int(sumLnz), Lnz, etree


@pytest.mark.parametrize("name", golden_names())
def test_kkt_csc_rhs_and_etree_match_oracle(name, kkt_check, tmp_path):
    from oracle.oracle import OracleKKT

    pm, d = load_golden(name)
    ny = int(np.sum(pm.ncs))
    g = np.random.default_rng(3)
    ws = d["ws"] if "ws" in d else g.standard_normal(pm.N * (pm.n + pm.m) + pm.n)
    ys = d["ys"] if ny else np.zeros(0)
    zs = d["zs"] if ny else np.zeros(0)
    irho = d["inv_rho"] if ny else np.zeros(0)
    sigma = float(d["sigma"])
    dim, Ap, Ai, Ax, rhs, sumLnz, Lnz, etree = _run(kkt_check, tmp_path, pm, ws, ys, zs, irho, d["x0"], sigma)
    o = OracleKKT(pm)
    assert dim == o.dim and Ai.size == o.nnz and sumLnz == o.sumLnz
    oAp, oAi, oAx = o.csc()
    assert np.array_equal(Ap, oAp) and np.array_equal(Ai, oAi)
    assert np.array_equal(Ax, oAx)
    assert np.all(Ai <= np.repeat(np.arange(dim), np.diff(Ap)))  # upper triangle
    par = etree[etree >= 0]
    assert np.all(par > np.nonzero(etree >= 0)[0])  # an elimination tree points to later columns
    assert int(Lnz.sum()) == sumLnz
    o.update_problem_data(ws, ys if ny else None, zs if ny else None, irho if ny else None, sigma)
    o.backward(irho if ny else None)
    o.forward(d["x0"])
    assert np.allclose(rhs, o.rhs(), rtol=0, atol=1e-14 * max(1.0, float(np.abs(rhs).max())))
