"""Dump a PARALLEL handle's internal segment buffers (diagnostics only)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pdp-lqr_amd"), os.path.join(ROOT, "tests")]
from conftest import load_golden  # noqa: E402
from pdplqr import CondensedSystemSolverType, LQRParallelSolver, lib  # noqa: E402
from pdplqr.model import unpack_model, unpack_ws  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "quadrotor_N100"
pm, d = load_golden(name)
model = unpack_model(pm)
n, m, N = pm.n, pm.m, pm.N
ws = unpack_ws(d["ws"], n, m, N)
sol = LQRParallelSolver(model, 4, True, CondensedSystemSolverType.CHOLESKY)
sol.update_problem_data(ws, [np.zeros(0)] * (N + 1), [np.zeros(0)] * (N + 1), [np.zeros(0)] * (N + 1), float(d["sigma"]))
sol.backward([np.zeros(0)] * (N + 1))
out = [w.copy() for w in ws]
sol.forward(d["x0"], out)
L = lib()
L.pdplqr_debug_parallel.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_longlong]
seg = np.zeros(2 * 256, dtype=np.int32)
S = L.pdplqr_debug_parallel(sol._hd.h, 5, seg.ctypes.data, seg.nbytes)
print("S", S, seg[:2 * S].reshape(S, 2).tolist())
es = 3 * n * n + 2 * n
for which, nm in [(0, "elem"), (1, "pre"), (2, "suf")]:
    a = np.zeros(S * es)
    L.pdplqr_debug_parallel(sol._hd.h, which, a.ctypes.data, a.nbytes)
    a = a.reshape(S, es)
    print(nm, "finite per seg:", [bool(np.all(np.isfinite(r))) for r in a])
    print(nm, "P trace:", [round(float(np.trace(r[2 * n * n + n:3 * n * n + n].reshape(n, n))), 4) for r in a])
for which, nm in [(3, "xhat"), (4, "lam")]:
    a = np.zeros((S + 1) * n)
    L.pdplqr_debug_parallel(sol._hd.h, which, a.ctypes.data, a.nbytes)
    print(nm, a.reshape(S + 1, n)[:, :3].round(5).tolist())
w = np.concatenate(out)
print("nan stages:", sorted(set(int(i) // (n + m) for i in np.where(~np.isfinite(w))[0]))[:20])
print("status", sol.status())
