"""Where and when the waves of the C5 backward kernels run (diagnostic).

Needs the probe variant: scripts/build_variant.sh hwid -DPDPLQR_HWID_PROBE=1 and
PDPLQR_LIB=pdp-lqr_amd/build/variants/libpdplqr_hwid.so.  Every block's lane 0
records (XCC, SE, SH, CU, SIMD) and its start / end on the 100 MHz constant
clock (device_common.hpp, PDPLQR_PROBE_*).  For the protocol order (update,
backward, forward), back-to-back (backward, forward), after 2 ms of idle and
after a read-only sweep of 1 GiB (evicts the dirty lines update leaves in the
caches) this prints, per call: kernel span from the waves, wave durations (min / median / max), how many
waves shared a SIMD / a CU, the per-XCC spread of the start times and the
waves' core clock (MHz, min / median / max).
usage: python scripts/c5_placement.py [kkt|serial|head]"""
import ctypes as C
import json
import os
import sys
import time
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pdp-lqr_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from pdplqr import BatchedLQRSolver  # noqa: E402
from pdplqr._lib import lib  # noqa: E402

SLOTS = 16384
FIELDS = 5


def read_probe(tu, nblk):
    buf = (C.c_longlong * (FIELDS * SLOTS))()
    fn = getattr(lib(), "pdplqr_probe_read_" + tu)
    fn.argtypes = [C.c_void_p]
    assert fn(C.cast(buf, C.c_void_p)) == 0
    a = np.frombuffer(buf, dtype=np.int64).reshape(SLOTS, FIELDS)[:nblk].copy()
    return a


def summarize(a):
    place, t0, t1, c0, c1 = a[:, 0], a[:, 1], a[:, 2], a[:, 3], a[:, 4]
    mhz = (c1 - c0) / np.maximum(t1 - t0, 1) * 100.0
    xcc = place >> 16
    cu_key = place >> 2  # (xcc, se, sh, cu)
    simd_cnt = Counter(place.tolist())
    cu_cnt = Counter(cu_key.tolist())
    dur = (t1 - t0) * 0.01  # us (100 MHz)
    span = (t1.max() - t0.min()) * 0.01
    start_rel = (t0 - t0.min()) * 0.01
    per_xcc = {}
    for x in sorted(set(xcc.tolist())):
        sel = xcc == x
        per_xcc[int(x)] = {"waves": int(sel.sum()), "start_max_us": round(float(start_rel[sel].max()), 1),
                           "dur_med_us": round(float(np.median(dur[sel])), 1),
                           "dur_max_us": round(float(dur[sel].max()), 1)}
    return {
        "span_us": round(float(span), 1),
        "clock_mhz": [round(float(mhz.min())), round(float(np.median(mhz))), round(float(mhz.max()))],
        "dur_us": [round(float(dur.min()), 1), round(float(np.median(dur)), 1), round(float(dur.max()), 1)],
        "start_spread_us": round(float(start_rel.max()), 1),
        "simds_used": len(simd_cnt), "waves_per_simd_hist": dict(Counter(simd_cnt.values())),
        "cus_used": len(cu_cnt), "waves_per_cu_hist": dict(Counter(cu_cnt.values())),
        "dur_by_waves_on_simd": {int(k): round(float(np.median(dur[[simd_cnt[p] == k for p in place.tolist()]])), 1)
                                 for k in sorted(set(simd_cnt.values()))},
        "per_xcc": per_xcc,
    }


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "kkt"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    n, m, s = 12, 4, 16
    if which == "head":
        N, batch, nc = 1024, 4096, 0
    else:
        N, batch, nc = 512, 1024, 4
    E, c, H, h, x0 = bench.gen_batch_device(n, m, N, batch, seed=555, device=dev)
    out = torch.empty(batch, N * s + n, dtype=torch.float64, device=dev)
    if nc:
        ncs = np.array([nc] * N + [0], dtype=np.int32)
        Dk = torch.zeros(nc, s, dtype=torch.float64, device=dev)
        Dk[:, :m] = torch.eye(m, dtype=torch.float64, device=dev)
        D = Dk.t().contiguous().reshape(-1).repeat(batch, N)
        g = torch.Generator(device=dev)
        g.manual_seed(556)
        ny = nc * N
        ws = torch.randn(batch, N * s + n, dtype=torch.float64, device=dev, generator=g)
        ys = torch.randn(batch, ny, dtype=torch.float64, device=dev, generator=g)
        zs = torch.randn(batch, ny, dtype=torch.float64, device=dev, generator=g)
        rho = torch.full((batch, ny), 0.1, dtype=torch.float64, device=dev)
        irho = 1.0 / rho
        solver = "kkt" if which == "kkt" else "serial"
        bs = BatchedLQRSolver(n, m, N, batch, solver=solver, ncs=ncs, device=0)
        bs.set_model(E, c, H, h, D)
        upd = lambda: bs.update_problem_data(ws, ys, zs, irho, sigma=1e-6)  # noqa: E731
        r = irho if solver == "kkt" else rho
        tu = "kkt" if solver == "kkt" else "schur"
    else:
        ws = torch.zeros(batch, N * s + n, dtype=torch.float64, device=dev)
        bs = BatchedLQRSolver(n, m, N, batch, device=0)
        bs.set_model(E, c, H, h)
        upd = lambda: bs.update_problem_data(ws, sigma=1e-6)  # noqa: E731
        r = None
        tu = "schur"
    upd()
    bs.synchronize()
    side = torch.cuda.Stream(device=dev)
    bs.handle.set_stream(side.cuda_stream)
    res = []
    with torch.cuda.stream(side):
        sweep = torch.ones(1 << 27, dtype=torch.float64, device=dev)  # 1 GiB
        for mode in ["repeat"] * 3 + ["update"] * 3 + ["repeat"] * 2 + ["update_idle", "update_sweep"] * 2:
            if mode.startswith("update"):
                upd()
            if mode == "update_idle":
                torch.cuda.synchronize()
                time.sleep(0.002)
            elif mode == "update_sweep":
                float(sweep.sum())  # read-only pass: update's dirty lines leave the caches
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(side)
            if r is None:
                bs.backward()
            else:
                bs.backward(r)
            e1.record(side)
            torch.cuda.synchronize()
            a = read_probe(tu, batch)
            bs.forward(x0, out)
            torch.cuda.synchronize()
            d = summarize(a)
            d["mode"] = mode
            d["event_ms"] = round(e0.elapsed_time(e1), 4)
            res.append(d)
            print(json.dumps(d), flush=True)
    bs.close()


if __name__ == "__main__":
    main()
