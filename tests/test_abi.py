"""CPU-side checks of the C ABI boundary: libpdplqr.so loads, exports every
symbol include/pdplqr.h declares, and the config defaults match the
reference's constructor defaults.  No compute calls (no GPU here)."""
import ctypes as C
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "pdplqr.h")


def declared_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(pdplqr_[a-z_]+)\s*\(", txt)))


def test_header_declares_protocol():
    syms = declared_symbols()
    for s in ["pdplqr_create", "pdplqr_set_model", "pdplqr_update_problem_data", "pdplqr_backward",
              "pdplqr_backward_without_factorization", "pdplqr_forward", "pdplqr_destroy"]:
        assert s in syms


def test_library_exports_every_declared_symbol():
    from pdplqr import _lib

    L = _lib.lib()
    syms = declared_symbols()
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert sorted(_lib.EXPORTS) == syms


def test_bench_probe_library_loads():
    """bench.py's pattern-ceiling probe (csrc/probe_pattern.hip) is its own
    library, outside the C ABI: it loads, exports its one entry point, and
    rejects bad sizes before any launch."""
    path = os.path.join(ROOT, "pdp-lqr_amd", "pdplqr", "libpdplqr_probe.so")
    if not os.path.exists(path):
        pytest.skip("probe library not built")
    L = C.CDLL(path)
    fn = L.pdplqr_probe_pattern
    fn.restype = C.c_int
    fn.argtypes = [C.c_void_p, C.c_int] * 3 + [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
    assert fn(None, 0, None, 1, None, 1, None, 0, 1, 1, None, None) != 0  # r0 = 0: invalid
    assert fn(None, 1, None, 1, None, 129, None, 0, 1, 1, None, None) != 0  # r2 > 128: invalid
    assert not any(s.startswith("pdplqr_probe") for s in declared_symbols())


def test_config_defaults_match_reference():
    from pdplqr import _lib

    cfg = _lib.Config()
    _lib.lib().pdplqr_config_init(C.byref(cfg))
    assert cfg.load_balancing == 1  # lqr_solver_parallel.hpp:24 load_balancing=true
    assert cfg.condensed_type == _lib.PDPLQR_CONDENSED_CHOLESKY  # :25 default CHOLESKY
    assert cfg.rho_dyn == 1e-6 and cfg.kkt_sigma == 1e-6  # qdldl_solver.hpp:38-39
    assert cfg.keep_factors == 1 and cfg.batch == 1


def test_create_rejects_bad_horizon_without_touching_gpu():
    """lqr_model.hpp:75-77: N < 1 throws; the ABI returns INVALID before any HIP call."""
    from pdplqr import _lib

    L = _lib.lib()
    cfg = _lib.Config()
    L.pdplqr_config_init(C.byref(cfg))
    cfg.nx, cfg.nu, cfg.N = 4, 2, 0
    h = C.c_void_p()
    assert L.pdplqr_create(C.byref(cfg), C.byref(h)) == -1
    assert b"Horizon" in L.pdplqr_last_error()


def test_product_path_does_not_import_oracle():
    """The product package must never route through the CPU oracle."""
    pkg = os.path.join(ROOT, "pdp-lqr_amd")
    bad = re.compile(r"(import\s+oracle|from\s+oracle|liborcpdplqr|\borc_[a-z_]+\()")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith((".py", ".hip", ".hpp", ".cpp", ".h", "Makefile")):
                txt = open(os.path.join(dp, f)).read()
                assert not bad.search(txt), os.path.join(dp, f)
