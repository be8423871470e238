"""Static (CPU) check of the register-staged value-form backward
(kernels_schur.hip): compiles it to gfx950 assembly and verifies that no
instruction touches a staging register set while its loads are in flight,
and that the stage loop drains the vector-memory counter before it exits
(round 1 shipped a kernel where the loop exit copied an in-flight set and
reused its registers: stage 0 of ~2 % of the bench problems was wrong)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="hipcc not installed")
@pytest.mark.parametrize("src", ["kernels_schur.hip", "kkt_riccati.hip"])
def test_schur_staging_has_no_inflight_hazard(tmp_path, src):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "asm_inflight_check.py"),
                        os.path.join(ROOT, "pdp-lqr_amd", "csrc", src), str(tmp_path / "k.s")],
                       cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 hazards" in r.stdout


@pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="hipcc not installed")
def test_kkt_linear_pass_vmcnt_waits(tmp_path):
    """k_kkt_ric_nofact keeps PDPLQR_KKT_NF_DEPTH register sets in flight with
    hand-counted vmcnt waits: no instruction touches a set before the wait that
    retires it (scripts/asm_vmcnt_check.py models the counter in issue order)."""
    asm = str(tmp_path / "kkt.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-Iinclude",
                    "--cuda-device-only", "-S", os.path.join(ROOT, "pdp-lqr_amd", "csrc", "kkt_riccati.hip"), "-o",
                    asm], cwd=ROOT, check=True, capture_output=True, timeout=600)
    for sym in ("k_kkt_ric_nofactILi4E", "k_kkt_ric_nofactILi0E"):
        r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "asm_vmcnt_check.py"), asm, sym],
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0 and "0 hazards" in r.stdout, r.stdout + r.stderr


def test_runtime_switches_are_the_documented_seven():
    """The library reads exactly these environment switches (DESIGN.md section
    6a, each with a GPU test), nothing that selects a retired A/B variant."""
    import glob
    import re

    found = set()
    for p in glob.glob(os.path.join(ROOT, "pdp-lqr_amd", "csrc", "*.hip")) + \
            glob.glob(os.path.join(ROOT, "pdp-lqr_amd", "csrc", "*.hpp")):
        found |= set(re.findall(r'getenv\("(PDPLQR_[A-Z0-9_]+)"\)', open(p).read()))
    expected = {"PDPLQR_GRAPH", "PDPLQR_KKT_LDL", "PDPLQR_KKT_NO_LINEAR", "PDPLQR_MD_P2P", "PDPLQR_NO_ADMM_FUSE",
                "PDPLQR_NO_X1", "PDPLQR_SHARD_FOLD"}
    assert found == expected, found ^ expected
    design = open(os.path.join(ROOT, "DESIGN.md")).read()
    for v in expected:
        assert v in design, v
