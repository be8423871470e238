"""Phase breakdown of the n = 24 blocked-LDL^T combine (combine_qd.hpp) in a
diagnostic build (-DPDPLQR_COMB_PROFILE, libpdplqr_combprof.so): one C4 slice
backward (segments + suffix scan); per scan-combine block the wall-clock marks
(100 MHz ticks)
(entry, staged, assembled, eliminated, end).
usage: python scripts/qd_phases.py [N=8192]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("PDPLQR_LIB", os.path.join(ROOT, "pdp-lqr_amd", "build", "abv", "libpdplqr_combprof.so"))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pdp-lqr_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from pdplqr import _lib  # noqa: E402
from pdplqr.horizon import HorizonShard  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
n, m = 24, 8
dev = torch.device("cuda", 0)
E, c, H, h, x0 = bench.gen_batch_device(n, m, N, 1, seed=1, device=dev)
sh = HorizonShard(n, m, N, 1, device=0)
sh.set_model(E, c, H, h)
sh.update_problem_data(torch.zeros(1, N * (n + m) + n, dtype=torch.float64, device=dev), sigma=1e-6)
elem = torch.empty(1, sh.es, dtype=torch.float64, device=dev)
for _ in range(3):
    sh.backward(elem, True)
    sh.synchronize()
L = _lib.lib()
buf = np.zeros(1024 * 32, dtype=np.uint64)
L.pdplqr_debug_comb_times.argtypes = [C.c_void_p]
assert L.pdplqr_debug_comb_times(C.c_void_p(buf.ctypes.data)) == 0
t = buf.reshape(1024, 32).astype(np.int64)
t = t[(t[:, 0] > 0) & (t[:, 8] > t[:, 0]) & (t[:, 16] > 0) & (t[:, 7] > 0)]
med = lambda v: float(np.median(v))
print(f"blocks {len(t)}; wall ticks (10 ns): entry->staged {med(t[:, 17] - t[:, 16]):.0f}, "
      f"staged->assembled {med(t[:, 1] - t[:, 17]):.0f}, elimination {med(t[:, 7] - t[:, 1]):.0f}, "
      f"outputs {med(t[:, 8] - t[:, 7]):.0f}, total combine {med(t[:, 8] - t[:, 0]):.0f}, "
      f"entry->stores done {med(t[:, 18] - t[:, 16]):.0f}")
for fl in (1, 0):
    sel = t[:, 22] == fl
    if sel.any():
        print(f"  fcf={fl}: {sel.sum()} blocks, combine {med(t[sel][:, 8] - t[sel][:, 0]):.0f} ticks")
for nm, off in (("wave 0 (diagonal tiles, LDL^T)", 27), ("wave 1 (tiles)", 23)):
    print(f"  {nm}, shader cycles over the 6 blocks: after B (updates, publish, LDL^T) {med(t[:, off]):.0f}, "
          f"wait at A {med(t[:, off + 1]):.0f}, V/W {med(t[:, off + 2]):.0f}, wait at B {med(t[:, off + 3]):.0f}")
