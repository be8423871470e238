"""CMake package parity (reference CMakeLists.txt:80-133):
the top-level CMakeLists.txt builds libpdplqr.so as HIP for gfx950, installs
headers, library, pdpLQRTargets.cmake, pdpLQRConfig.cmake (find_dependency(hip))
and an ExactVersion 1.0.0 version file; a downstream project then finds the
INSTALLED package with find_package(pdpLQR 1.0.0) and links pdpLQR::pdpLQR.
Compile-only (CPU): hipcc cross-compiles for gfx950 here."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


@pytest.mark.skipif(shutil.which("cmake") is None or not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="cmake / ROCm missing")
def test_install_and_consume(tmp_path):
    bd, pre, cons = tmp_path / "build", tmp_path / "prefix", tmp_path / "consumer"
    run = lambda *a: subprocess.run(list(a), capture_output=True, text=True, timeout=900)
    r = run("cmake", "-S", ROOT, "-B", str(bd), "-DCMAKE_PREFIX_PATH=/opt/rocm", "-DBUILD_EXAMPLES=ON")
    assert r.returncode == 0, r.stdout + r.stderr
    r = run("cmake", "--build", str(bd), f"-j{min(8, os.cpu_count() or 2)}")
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    r = run("cmake", "--install", str(bd), "--prefix", str(pre))
    assert r.returncode == 0, r.stdout + r.stderr
    cfgdir = pre / "lib" / "cmake" / "pdpLQR"
    for f in ("pdpLQRConfig.cmake", "pdpLQRConfigVersion.cmake", "pdpLQRTargets.cmake"):
        assert (cfgdir / f).exists(), f
    assert "find_dependency(hip" in (cfgdir / "pdpLQRConfig.cmake").read_text()
    assert "ExactVersion" in (cfgdir / "pdpLQRConfigVersion.cmake").read_text() or \
        "PACKAGE_VERSION_EXACT" in (cfgdir / "pdpLQRConfigVersion.cmake").read_text()
    assert (pre / "include" / "pdplqr.h").exists() and (pre / "include" / "clqr" / "lqr_model.hpp").exists()
    assert (pre / "lib" / "libpdplqr.so").exists()
    # gfx950 code object inside the installed library
    r = run("strings", str(pre / "lib" / "libpdplqr.so"))
    assert "gfx950" in r.stdout
    # a downstream project against the installed tree
    r = run("cmake", "-S", os.path.join(ROOT, "tests", "cpp"), "-B", str(cons),
            f"-DCMAKE_PREFIX_PATH={pre};/opt/rocm")
    assert r.returncode == 0, r.stdout + r.stderr
    r = run("cmake", "--build", str(cons), "-j4")
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert (cons / "facade_check").exists() and (cons / "lqr_example").exists()
    # a version other than 1.0.0 is refused (ExactVersion, as the reference)
    (tmp_path / "v" ).mkdir()
    (tmp_path / "v" / "CMakeLists.txt").write_text(
        "cmake_minimum_required(VERSION 3.21)\nproject(v CXX)\nfind_package(pdpLQR 1.1.0 REQUIRED)\n")
    r = run("cmake", "-S", str(tmp_path / "v"), "-B", str(tmp_path / "vb"), f"-DCMAKE_PREFIX_PATH={pre};/opt/rocm")
    assert r.returncode != 0
