"""Diagnostic: device internals of the wide parallel solver (kernels_wide.hip)
against the numpy restatement (tests/seg_ref.py) on one problem -- segment
elements, the suffix scan, boundary states and costates -- to locate where a
parity gap opens.  usage: python scripts/diag_wide.py [n m N ns seglen nc LU|CHOLESKY]"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pdp-lqr_amd"), os.path.join(ROOT, "tests")]

from seg_ref import boundary_state, combine, combine_lu, slice_element  # noqa: E402
from test_gpu_wide import _pm, _problem  # noqa: E402


def rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def main():
    a = sys.argv[1:]
    n, m, N, ns, seglen, nc = (int(x) for x in (a[:6] if len(a) >= 6 else [50, 10, 24, 3, 2, 4]))
    cond = a[6] if len(a) > 6 else "CHOLESKY"
    from oracle.oracle import OracleSerial
    from pdplqr import BatchedLQRSolver, _lib

    s = n + m
    p = _problem(n, m, N, 2, nc, 5 * n + m + nc + ns)
    bs = BatchedLQRSolver(n, m, N, 2, solver="parallel", num_segments=ns, keep_factors=True, condensed=cond,
                          segment_len=seglen, ncs=p["ncs"])
    bs.set_model(p["E"], p["c"], p["H"], p["h"], p["D"] if nc else None)
    bs.update_problem_data(p["ws"], p["ys"] if nc else None, p["zs"] if nc else None, p["irho"] if nc else None,
                           sigma=1e-6)
    bs.backward((1.0 / p["irho"]) if nc else None)
    out = np.zeros_like(p["ws"])
    bs.forward(p["x0"], out)
    L = _lib.lib()
    L.pdplqr_debug_parallel.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_longlong]
    L.pdplqr_debug_parallel.restype = C.c_int
    h = bs.handle.h
    segbuf = np.zeros(2 * 4096, dtype=np.int32)
    S = L.pdplqr_debug_parallel(h, 5, segbuf.ctypes.data, segbuf.nbytes)
    segs = [(int(segbuf[2 * i]), int(segbuf[2 * i] + segbuf[2 * i + 1])) for i in range(S)]
    es = 3 * n * n + 2 * n
    B = 2

    def fetch(which, count):
        v = np.zeros(B * count)
        L.pdplqr_debug_parallel(h, which, v.ctypes.data, v.nbytes)
        return v.reshape(B, -1)

    elem, suf = fetch(0, S * es), fetch(2, S * es)
    xhat, lam = fetch(3, (S + 1) * n), fetch(4, (S + 1) * n)
    b = 0
    # numpy restatement of the same data
    E = [p["E"][b][k * n * s:(k + 1) * n * s].reshape(n, s, order="F") for k in range(N)]
    c = [p["c"][b][k * n:(k + 1) * n] for k in range(N)]
    Ht, ht, doff, yoff = [], [], 0, 0
    for k in range(N + 1):
        d = s if k < N else n
        H = p["H"][b][k * s * s:k * s * s + d * d].reshape(d, d, order="F") + 1e-6 * np.eye(d)
        hh = p["h"][b][k * s:k * s + d] - 1e-6 * p["ws"][b][k * s:k * s + d]
        if nc:
            Dk = p["D"][b][doff:doff + nc * d].reshape(nc, d, order="F")
            rho = 1 / p["irho"][b][yoff:yoff + nc]
            g = p["zs"][b][yoff:yoff + nc] - p["irho"][b][yoff:yoff + nc] * p["ys"][b][yoff:yoff + nc]
            H = H + Dk.T @ np.diag(rho) @ Dk
            hh = hh - Dk.T @ (rho * g)
            doff += nc * d
            yoff += nc
        Ht.append(H)
        ht.append(hh)
    els = [slice_element(E, c, Ht, ht, k0, k1, (Ht[N], ht[N]) if k1 == N else None) for (k0, k1) in segs]
    comb = combine if cond == "CHOLESKY" else combine_lu
    cur, d = list(els), 1
    while d < S:
        cur = [comb(cur[i], cur[i + d]) if i + d < S else cur[i] for i in range(S)]
        d *= 2
    names = "FCfPp"
    for i in range(S):
        ge = [elem[b][i * es:(i + 1) * es]]
        from seg_ref import unpack
        g5, r5 = unpack(ge[0], n), els[i]
        g5s, r5s = unpack(suf[b][i * es:(i + 1) * es], n), cur[i]
        print(f"seg {i} {segs[i]} elem", " ".join(f"{nm}:{rel(x, y):.1e}" for nm, x, y in zip(names, g5, r5)),
              "| suf", " ".join(f"{nm}:{rel(x, y):.1e}" for nm, x, y in zip(names, g5s, r5s)))
    # boundary states: x_j = state at the start of segment j (j = 0..S), prefix (x) suffix
    x0 = p["x0"][b]
    pre = None
    for j in range(S + 1):
        if j == 0:
            xr = x0
        else:
            pre = els[0] if pre is None else comb(pre, els[j - 1])
            xr = boundary_state(pre, cur[j], x0) if j < S else (pre[0] @ x0 + pre[2])
        print(f"boundary {j} x err {rel(xhat[b][j * n:(j + 1) * n], xr):.2e}")
    o = OracleSerial(_pm(p, b, n, m, N))
    o.update_problem_data(p["ws"][b], p["ys"][b] if nc else None, p["zs"][b] if nc else None,
                          p["irho"][b] if nc else None, 1e-6)
    o.backward((1.0 / p["irho"][b]) if nc else None)
    ref = o.forward(x0)
    print("w err", rel(out[b], ref))
    # boundary states and costates against the serial oracle's trajectory
    for j, (k0, k1) in enumerate(segs):
        xt = ref[k0 * s + (m if k0 < N else 0):k0 * s + (m if k0 < N else 0) + n]
        Pt, pt = o.value_function(k0)
        lt = Pt @ xt + pt
        print(f"boundary {j} (stage {k0}) x vs oracle {rel(xhat[b][j * n:(j + 1) * n], xt):.2e}"
              f"  lambda vs oracle {rel(lam[b][j * n:(j + 1) * n], lt):.2e}  |lambda| {np.linalg.norm(lt):.2e}")
    for k0, k1 in segs:
        print(f"  stages {k0}..{k1} err", rel(out[b][k0 * s:k1 * s], ref[k0 * s:k1 * s]))


if __name__ == "__main__":
    main()
