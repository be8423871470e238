"""Phase cycles of the block-wide value-form backward (k_seg_bwd_wide, serial
mode) on block 0: needs the diagnostic build -DPDPLQR_SEGW_PROFILE=1 loaded
through PDPLQR_LIB.  usage: PDPLQR_LIB=... python scripts/prof_segw.py n m"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pdp-lqr_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from pdplqr import BatchedLQRSolver  # noqa: E402
from pdplqr import _lib  # noqa: E402


def main():
    n, m = int(sys.argv[1]), int(sys.argv[2])
    N, batch = 256, 1024
    dev = torch.device("cuda", 0)
    s = n + m
    E, c, H, h, x0 = bench.gen_batch_device(n, m, N, batch, seed=91, device=dev)
    ws0 = torch.zeros(batch, N * s + n, dtype=torch.float64, device=dev)
    bs = BatchedLQRSolver(n, m, N, batch, keep_factors=False, device=0)
    bs.set_model(E, c, H, h)
    bs.update_problem_data(ws0, sigma=1e-6)
    torch.cuda.synchronize()
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    bs.backward()
    t1.record()
    torch.cuda.synchronize()
    out = (ctypes.c_ulonglong * 16)()
    _lib.lib().pdplqr_debug_segw(out)
    # g_segw[i]: the time up to marker i (kernels_wide.hip SEGW_T)
    names = ["blk_mv pc", "blk_mm PE", "blk_mv lp", "blk_mm M", "issue next loads", "pivots", "P_k out",
             "store next + tail", "loop head"]
    tot = sum(out[i] for i in range(9))
    print(f"{n}/{m}: backward {t0.elapsed_time(t1):.3f} ms; block 0 stage-loop s_memtime ticks {tot} "
          f"({tot / N:.0f} per stage)")
    for i, nm in enumerate(names):
        print(f"  {nm:18s} {out[i]:10d}  {100.0 * out[i] / tot:5.1f} %")


if __name__ == "__main__":
    main()
