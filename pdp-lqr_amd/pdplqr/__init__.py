"""pdplqr -- MI355X-native parallel-DP LQR solver (host-side mirror).

Python mirror of the reference's ``namespace lqr`` (Luyao787/PDP-LQR) over the
C ABI of libpdplqr.so (include/pdplqr.h).  See DESIGN.md.
"""
from .model import LQR_INFTY, LQRModel, Node, PackedModel, initialize_vectors, pack_model, unpack_ws  # noqa: F401
from .solvers import (  # noqa: F401
    BatchedLQRSolver,
    CondensedSystemSolverType,
    LQRParallelSolver,
    LQRSolver,
    QDLDLSolver,
)
from ._lib import LIB_PATH, PdplqrError, device_count, lib  # noqa: F401

__version__ = "0.1.0"
