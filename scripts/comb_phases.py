"""Phase breakdown of the segment combine (debug build libpdplqr_combprof.so,
-DPDPLQR_COMB_PROFILE): runs one horizon-slice backward (segments + scans) and
prints the median duration of each combine phase over the recorded blocks.
usage: python scripts/comb_phases.py [N] [n] [m]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("PDPLQR_LIB", os.path.join(ROOT, "pdp-lqr_amd", "build", "variants", "libpdplqr_combprof.so"))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pdp-lqr_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from pdplqr import _lib  # noqa: E402
from pdplqr.horizon import HorizonShard  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
n = int(sys.argv[2]) if len(sys.argv) > 2 else 24
m = int(sys.argv[3]) if len(sys.argv) > 3 else 8
dev = torch.device("cuda", 0)
E, c, H, h, x0 = bench.gen_batch_device(n, m, N, 1, seed=1, device=dev)
sh = HorizonShard(n, m, N, 1, device=0)
sh.set_model(E, c, H, h)
sh.update_problem_data(torch.zeros(1, N * (n + m) + n, dtype=torch.float64, device=dev), sigma=1e-6)
elem = torch.empty(1, sh.es, dtype=torch.float64, device=dev)
sh.backward(elem, True)
sh.synchronize()
sh.backward(elem, True)
sh.synchronize()
L = _lib.lib()
buf = np.zeros(1024 * 32, dtype=np.uint64)
L.pdplqr_debug_comb_times.argtypes = [C.c_void_p]
assert L.pdplqr_debug_comb_times(C.c_void_p(buf.ctypes.data)) == 0
tall = buf.reshape(1024, 32).astype(np.int64)
t = tall
ok = (t[:, 0] > 0) & (t[:, 9] > t[:, 0])
for k in range(1, 10):
    ok &= t[:, k] >= t[:, k - 1]
t = t[ok]
mw = os.environ.get("COMB_MW", "1") != "0"  # the 4-wave combine (combine_mw.hpp) marks
names = (["A: chol R (w0)", "B: S products (w0)", "B: wait slowest wave", "C: chol S carrying (w0)",
          "C: wait + store", "D: P (w0)", "D: wait slowest wave", "-", "-"] if mw else
         ["load Ca", "load Pb+chol R", "T1,S products", "chol Q", "U solve (LDS)", "Y,Z,Zt products", "P path",
          "F,C path", "vectors"])
d = np.diff(t[:, :10], axis=1)
print(f"blocks={len(t)}  wall_clock64 ticks (100 MHz): total median {np.median(t[:, 9] - t[:, 0]):.0f}")
for k, nm in enumerate(names):
    print(f"  {nm:18s} {np.median(d[:, k]):8.0f}")
ka = tall[ok]
if len(ka) and (ka[:, 16] > 0).all():  # kernel-level marks of k_seg_scan_mw
    med = lambda v: float(np.median(v))
    print(f"  scan kernel: entry -> staged {med(ka[:, 17] - ka[:, 16]):.0f}, staged -> combine "
          f"{med(ka[:, 0] - ka[:, 17]):.0f}, combine end -> stores done {med(ka[:, 18] - ka[:, 9]):.0f}, "
          f"entry -> stores done {med(ka[:, 18] - ka[:, 16]):.0f}")
    print(f"  chol R: load P_b {med(ka[:, 19] - ka[:, 0]):.0f}, chol_blk4 {med(ka[:, 20] - ka[:, 19]):.0f}, "
          f"transpose {med(ka[:, 1] - ka[:, 20]):.0f}")
    for fl, nm in ((1, "full combines (F, C, f, P, p)"), (0, "P-only combines (right operand at the terminal)")):
        sel = ka[:, 22] == fl
        if sel.any():
            dd = np.diff(ka[sel][:, :10], axis=1)
            print(f"  {nm}: {sel.sum()} blocks, total {med(ka[sel][:, 9] - ka[sel][:, 0]):.0f}; " +
                  ", ".join(f"{names[k].split(':')[-1].strip()} {np.median(dd[:, k]):.0f}" for k in range(6)))
    # blocks of the last recorded round of each distance: entry spread and end spread
    for dist in sorted(set(ka[:, 21].tolist()))[-3:]:
        r = ka[ka[:, 21] == dist]
        e0 = r[:, 16].min()
        print(f"  round d={dist}: {len(r)} blocks, entry first -> median {med(r[:, 16] - e0):.0f} -> last "
              f"{(r[:, 16] - e0).max()}, stores done median {med(r[:, 18] - e0):.0f} last {(r[:, 18] - e0).max()}")
seg = buf.reshape(1024, 32).astype(np.int64)
seg = seg[seg[:, 12] > 0]
if len(seg):
    st = seg[:, 12]
    print(f"segment backward ({len(seg)} waves, median {np.median(st):.0f} stages): ticks per stage "
          f"riccati {np.median(seg[:, 10] / st):.0f}  element {np.median(seg[:, 11] / st):.0f}")
# stage phases of the 4-wave segment backward (k_seg_bwd_aug_mw, second stage of each segment)
if hasattr(L, "pdplqr_debug_aug_times"):
    ab = np.zeros(1024 * 16, dtype=np.uint64)
    L.pdplqr_debug_aug_times.argtypes = [C.c_void_p]
    if L.pdplqr_debug_aug_times(C.c_void_p(ab.ctypes.data)) == 0:
        a16 = ab.reshape(1024, 16).astype(np.int64)
        a = a16[:, :8]
        ok = (a[:, 0] > 0) & np.all(np.diff(a, axis=1) >= 0, axis=1)
        a = a[ok]
        a16 = a16[ok]
        if len(a):
            an = ["B1 (publish, barrier)", "G = P E~", "rows [u;x] + aug", "B2", "u-pivot blocks", "checks, cache",
                  "inputs, B_end"]
            da = np.diff(a, axis=1)
            print(f"aug stage ({len(a)} blocks): total median {np.median(a[:, 7] - a[:, 0]):.0f} ticks")
            for k, nm in enumerate(an):
                print(f"  {nm:24s} {np.median(da[:, k]):8.0f}")
            # inside the two u-pivot blocks: barrier passed, factor + update issued, records issued
            two = len(a16) and (a16[:, 11] > 0).all()  # 4-pivot blocks (else one 8-pivot block)
            pb = a16[:, [4, 8, 9, 10, 11, 12, 13, 5] if two else [4, 8, 9, 10, 5]]
            if len(pb) and (np.diff(pb, axis=1) >= 0).all():
                dp = np.diff(pb, axis=1)
                nms = ["blk0: publish + barrier", "blk0: factor, X, MFMA issue", "blk0: records"]
                nms += ["blk1: publish + barrier", "blk1: factor, X, MFMA issue", "blk1: records"] if two else []
                for k, nm in enumerate(nms + ["-> end of pivots"]):
                    print(f"    {nm:30s} {np.median(dp[:, k]):8.0f}")
            wt, ct = a16[:, 7] - a16[:, 0], a16[:, 15] - a16[:, 14]
            if (wt > 0).all():
                print(f"  shader clock over the stage: {np.median(ct / wt) * 100:.0f} MHz")
