"""C4 horizon solve (24/8) at N = 65536 (1 GPU) and N = 8192 (one rank's slice
as a whole solve): device segment count S and ms per backward + forward for
the 4-wave kernels and their one-wave alternatives (PDPLQR_SCAN_1WAVE,
PDPLQR_AUG_1WAVE, read at launch).  python scripts/c4_variants.py [N ...]"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pdp-lqr_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from pdplqr import BatchedLQRSolver, _lib  # noqa: E402


def main():
    Ns = [int(x) for x in sys.argv[1:]] or [65536, 8192]
    n, m = 24, 8
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    L = _lib.lib()
    L.pdplqr_debug_parallel.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_longlong]
    L.pdplqr_debug_parallel.restype = C.c_int
    for N in Ns:
        E, c, H, h, x0 = bench.gen_batch_device(n, m, N, 1, seed=77, device=dev)
        ws0 = torch.zeros(1, N * (n + m) + n, dtype=torch.float64, device=dev)
        out = torch.empty_like(ws0)
        for scan1, aug1 in ((0, 0), (1, 0), (0, 1), (1, 1), (0, 0)):
            for k, v in (("PDPLQR_SCAN_1WAVE", scan1), ("PDPLQR_AUG_1WAVE", aug1)):
                if v:
                    os.environ[k] = "1"
                else:
                    os.environ.pop(k, None)
            bs = BatchedLQRSolver(n, m, N, 1, solver="parallel", num_segments=8, keep_factors=True, device=0)
            bs.set_model(E, c, H, h)
            bs.update_problem_data(ws0, sigma=1e-6)
            segbuf = np.zeros(2 * 65536, dtype=np.int32)
            S = L.pdplqr_debug_parallel(bs.handle.h, 5, segbuf.ctypes.data, segbuf.nbytes)

            def step():
                bs.backward()
                bs.forward(x0, out)

            t = bench._timed(step, 10, 3, dev, None)
            print(json.dumps({"N": N, "scan_1wave": scan1, "aug_1wave": aug1, "S": S, "ms": round(t * 1e3, 4),
                              "finite": bool(torch.isfinite(out).all().item())}), flush=True)
            bs.close()


if __name__ == "__main__":
    main()
