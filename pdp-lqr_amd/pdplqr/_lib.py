"""ctypes binding of libpdplqr.so (the C ABI declared in include/pdplqr.h).

The library is built in-tree (``pdp-lqr_amd/pdplqr/libpdplqr.so``) by
``__graft_entry__.build()`` / ``make -C pdp-lqr_amd/csrc``.  There is no CPU
fallback: if the library is missing or a call fails, this module raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PDPLQR_LIB") or os.path.join(_HERE, "libpdplqr.so")  # override: diagnostics only

PDPLQR_OK = 0
PDPLQR_MEM_HOST = 0
PDPLQR_MEM_DEVICE = 1
PDPLQR_SOLVER_SERIAL = 0
PDPLQR_SOLVER_PARALLEL = 1
PDPLQR_SOLVER_KKT = 2
PDPLQR_CONDENSED_LU = 0
PDPLQR_CONDENSED_CHOLESKY = 1

ERRORS = {-1: "INVALID", -2: "HIP", -3: "ALLOC", -4: "STATE", -5: "UNSUPPORTED", -6: "NUMERIC"}

# Every symbol include/pdplqr.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "pdplqr_config_init", "pdplqr_create", "pdplqr_destroy", "pdplqr_last_error", "pdplqr_set_stream",
    "pdplqr_get_stream", "pdplqr_synchronize", "pdplqr_set_model", "pdplqr_set_model_arrays",
    "pdplqr_get_model_upload_bytes", "pdplqr_update_problem_data",
    "pdplqr_backward", "pdplqr_backward_without_factorization", "pdplqr_forward", "pdplqr_clear_workspace",
    "pdplqr_get_value_function", "pdplqr_get_status", "pdplqr_get_segments", "pdplqr_shard_element_size",
    "pdplqr_shard_backward", "pdplqr_shard_backward_without_factorization", "pdplqr_shard_forward",
    "pdplqr_device_count",
    "pdplqr_admm_settings_init", "pdplqr_admm_solve", "pdplqr_admm_info", "pdplqr_multidev_plan",
]


class PdplqrError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"pdplqr error {code} ({ERRORS.get(code, '?')}): {msg}")
        self.code = code


class Config(C.Structure):
    _fields_ = [
        ("nx", C.c_int32), ("nu", C.c_int32), ("N", C.c_int32), ("batch", C.c_int32),
        ("solver", C.c_int32), ("num_segments", C.c_int32), ("load_balancing", C.c_int32),
        ("condensed_type", C.c_int32), ("device", C.c_int32), ("keep_factors", C.c_int32),
        ("ncs", C.POINTER(C.c_int32)), ("rho_dyn", C.c_double), ("kkt_sigma", C.c_double),
        ("segment_len", C.c_int32), ("num_devices", C.c_int32), ("devices", C.POINTER(C.c_int32)),
    ]


class AdmmSettings(C.Structure):
    _fields_ = [
        ("sigma", C.c_double), ("alpha", C.c_double), ("max_iter", C.c_int32), ("check_every", C.c_int32),
        ("eps_abs", C.c_double), ("eps_rel", C.c_double), ("adaptive_rho", C.c_int32),
        ("adaptive_rho_tolerance", C.c_double),
    ]


_lib = None


def lib() -> C.CDLL:
    """Load libpdplqr.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process: torch bundles its own libamdhip64.so.7 (same
    # soname as /opt/rocm's).  Load torch first when it is installed so that
    # libpdplqr.so binds to the runtime torch's tensors and streams live in.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libpdplqr.so not built at {LIB_PATH}: run `make -C pdp-lqr_amd/csrc` "
                          "or __graft_entry__.build() (no CPU fallback exists)")
    L = C.CDLL(LIB_PATH)
    vp, dp, ip, i32 = C.c_void_p, C.c_void_p, C.POINTER(C.c_int32), C.c_int32
    L.pdplqr_config_init.argtypes = [C.POINTER(Config)]
    L.pdplqr_config_init.restype = None
    L.pdplqr_create.argtypes = [C.POINTER(Config), C.POINTER(vp)]
    L.pdplqr_destroy.argtypes = [vp]
    L.pdplqr_last_error.argtypes = []
    L.pdplqr_last_error.restype = C.c_char_p
    L.pdplqr_set_stream.argtypes = [vp, vp]
    L.pdplqr_get_stream.argtypes = [vp]
    L.pdplqr_get_stream.restype = vp
    L.pdplqr_synchronize.argtypes = [vp]
    L.pdplqr_set_model.argtypes = [vp, dp, dp, dp, dp, dp, C.c_int]
    L.pdplqr_set_model_arrays.argtypes = [vp, C.c_int, dp, dp, dp, dp, dp, C.c_int]
    L.pdplqr_get_model_upload_bytes.argtypes = [vp, C.POINTER(C.c_int64)]
    L.pdplqr_update_problem_data.argtypes = [vp, dp, dp, dp, dp, C.c_double, C.c_int]
    L.pdplqr_backward.argtypes = [vp, dp, C.c_int]
    L.pdplqr_backward_without_factorization.argtypes = [vp, dp, C.c_int]
    L.pdplqr_forward.argtypes = [vp, dp, dp, C.c_int]
    L.pdplqr_clear_workspace.argtypes = [vp]
    L.pdplqr_get_value_function.argtypes = [vp, i32, i32, dp, dp]
    L.pdplqr_get_status.argtypes = [vp, ip]
    L.pdplqr_get_segments.argtypes = [vp, ip, ip]
    L.pdplqr_shard_element_size.argtypes = [vp]
    L.pdplqr_shard_backward.argtypes = [vp, dp, C.c_int, dp, C.c_int]
    if hasattr(L, "pdplqr_shard_backward_without_factorization"):  # (absent from pre-round-5 A/B variants)
        L.pdplqr_shard_backward_without_factorization.argtypes = [vp, dp, C.c_int, dp, C.c_int]
    L.pdplqr_shard_forward.argtypes = [vp, dp, dp, i32, i32, dp, C.c_int]
    L.pdplqr_device_count.argtypes = [ip]
    L.pdplqr_admm_settings_init.argtypes = [C.POINTER(AdmmSettings)]
    L.pdplqr_admm_settings_init.restype = None
    L.pdplqr_admm_solve.argtypes = [vp, C.POINTER(AdmmSettings), dp, dp, dp, dp, dp, dp, dp, C.c_int]
    L.pdplqr_admm_info.argtypes = [vp, ip, ip, dp, dp, dp]
    if hasattr(L, "pdplqr_multidev_plan"):  # (absent from pre-round-4 A/B variants)
        L.pdplqr_multidev_plan.argtypes = [i32, i32, ip, i32, i32, C.POINTER(C.c_int64)]
    for nm in EXPORTS:
        if LIB_PATH != os.path.join(_HERE, "libpdplqr.so") and not hasattr(L, nm):
            continue  # an older A/B variant (PDPLQR_LIB) may predate a symbol
        f = getattr(L, nm)
        if nm not in ("pdplqr_config_init", "pdplqr_last_error", "pdplqr_get_stream", "pdplqr_admm_settings_init"):
            f.restype = C.c_int
    _lib = L
    return L


def check(rc: int) -> int:
    if rc < 0:
        raise PdplqrError(rc, lib().pdplqr_last_error().decode(errors="replace"))
    return rc


def device_count() -> int:
    n = C.c_int32(0)
    rc = lib().pdplqr_device_count(C.byref(n))
    return int(n.value) if rc == 0 else 0
