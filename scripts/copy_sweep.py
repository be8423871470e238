"""Achievable HBM copy rate on this box: the probe library's
16-byte copy variants (csrc/probe_pattern.hip pdplqr_probe_copy_mode: grid-stride
with a block sweep, one element per thread, 64 B per thread, 64 B per thread
non-temporal) and torch's blit, at 1 and 4 GiB; read + write bytes / time,
best of 5 launches after one warm-up.  usage: python scripts/copy_sweep.py"""
import ctypes
import json
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = ctypes.CDLL(os.path.join(ROOT, "pdp-lqr_amd", "pdplqr", "libpdplqr_probe.so"))
fn = lib.pdplqr_probe_copy_mode
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
dev = torch.device("cuda", 0)
res = []
for gib in (1, 4):
    nbytes = gib << 30
    a = torch.ones(nbytes // 8, dtype=torch.float64, device=dev)
    b = torch.empty_like(a)
    st = torch.cuda.current_stream()

    def rate(launch, reps=5):
        launch()
        best = 0.0
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            launch()
            e1.record(st)
            torch.cuda.synchronize()
            best = max(best, 2 * nbytes / (e0.elapsed_time(e1) * 1e-3) / 1e12)
        return best

    def probe(mode, blocks=0):
        def go():
            rc = fn(a.data_ptr(), b.data_ptr(), nbytes, mode, blocks, ctypes.c_void_p(st.cuda_stream))
            assert rc == 0, rc
        return go

    row = {"GiB": gib, "blit": rate(lambda: b.copy_(a))}
    for bl in (1024, 2048, 4096, 8192, 16384, 32768):
        row[f"gridstride_{bl}"] = rate(probe(0, bl))
    for mode, nm in ((1, "one_per_thread"), (2, "64B_per_thread"), (3, "64B_per_thread_nt")):
        row[nm] = rate(probe(mode))
    assert torch.equal(a, b)
    print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in row.items()}), flush=True)
    res.append(row)
    del a, b
    torch.cuda.empty_cache()
print(json.dumps({"best_TBps": max(v for r in res for k, v in r.items() if k not in ("GiB",))}))
