"""C2 (one N = 1024 12/4 problem, LQRParallelSolver path) host-issue study:
per-solve wall time of backward + forward with
  own      the handle's own stream, torch stream joins per call (bench.py)
  shared   the handle on torch's current stream (no joins)
  raw      shared + the C ABI called directly through ctypes (no wrapper)
and the host-only issue time of the raw calls (no synchronisation inside the
loop).  PDPLQR_GRAPH=1 in the environment replays captured graphs."""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pdp-lqr_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from pdplqr import BatchedLQRSolver  # noqa: E402
from pdplqr._lib import lib  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    n, m, N = 12, 4, 1024
    E, c, H, h, x0 = bench.gen_batch_device(n, m, N, 1, seed=77, device=dev)
    ws0 = torch.zeros(1, N * (n + m) + n, dtype=torch.float64, device=dev)
    out = torch.empty_like(ws0)
    bs = BatchedLQRSolver(n, m, N, 1, solver="parallel", num_segments=8, keep_factors=True, device=0)
    bs.set_model(E, c, H, h)
    bs.update_problem_data(ws0, sigma=1e-6)
    res = {"graph": os.environ.get("PDPLQR_GRAPH", "0")}

    def wrapped():
        bs.backward(None)
        bs.forward(x0, out)

    L = lib()
    hx, ho = C.c_void_p(x0.data_ptr()), C.c_void_p(out.data_ptr())

    def raw():
        L.pdplqr_backward(bs.handle.h, None, 1)
        L.pdplqr_forward(bs.handle.h, hx, ho, 1)

    def timed(fn, steps=200, warm=20):
        for _ in range(warm):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3

    def raw_hostmem():  # backward with mem = HOST (no rho), as the wrapper passes it
        L.pdplqr_backward(bs.handle.h, None, 0)
        L.pdplqr_forward(bs.handle.h, hx, ho, 1)

    def wb_rf():
        bs.backward(None)
        L.pdplqr_forward(bs.handle.h, hx, ho, 1)

    def rb_wf():
        L.pdplqr_backward(bs.handle.h, None, 1)
        bs.forward(x0, out)

    res["raw_first_ms"] = timed(raw)
    res["own_ms"] = timed(wrapped)
    bs.handle.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    res["shared_ms"] = timed(wrapped)
    res["raw_ms"] = timed(raw)
    res["raw_hostmem_ms"] = timed(raw_hostmem)
    res["wrapped_bwd_raw_fwd_ms"] = timed(wb_rf)
    res["raw_bwd_wrapped_fwd_ms"] = timed(rb_wf)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        wrapped()
    res["wrapped_issue_ms"] = (time.perf_counter() - t0) / 50 * 1e3

    def spin(us):
        t = time.perf_counter() + us * 1e-6
        while time.perf_counter() < t:
            pass

    def raw_spin_fwd():  # host time before the forward call (no Python API work)
        L.pdplqr_backward(bs.handle.h, None, 1)
        spin(25)
        L.pdplqr_forward(bs.handle.h, hx, ho, 1)

    def raw_spin_bwd():  # host time before the backward call
        spin(25)
        L.pdplqr_backward(bs.handle.h, None, 1)
        L.pdplqr_forward(bs.handle.h, hx, ho, 1)

    def raw_curstream():
        L.pdplqr_backward(bs.handle.h, None, 1)
        torch.cuda.current_stream(dev)
        L.pdplqr_forward(bs.handle.h, hx, ho, 1)

    from pdplqr.solvers import _ptr, _mem_of

    def raw_ptr():  # the wrapper's pointer conversion, then the raw call
        L.pdplqr_backward(bs.handle.h, None, 1)
        ps = [_ptr(x0, "x0"), _ptr(out, "ws")]
        L.pdplqr_forward(bs.handle.h, ps[0][0], ps[1][0], _mem_of(*ps))

    def raw_enter():  # the wrapper's stream join check, then the raw call
        L.pdplqr_backward(bs.handle.h, None, 1)
        cur = bs.handle._enter(x0, out)
        L.pdplqr_forward(bs.handle.h, hx, ho, 1)
        bs.handle._leave(cur)

    def handle_fwd():  # _Handle.forward directly
        L.pdplqr_backward(bs.handle.h, None, 1)
        bs.handle.forward(x0, out)

    def fresh_ptr():  # new c_void_p objects from data_ptr() every call
        L.pdplqr_backward(bs.handle.h, None, 1)
        L.pdplqr_forward(bs.handle.h, C.c_void_p(x0.data_ptr()), C.c_void_p(out.data_ptr()), 1)

    res["raw_ptr_ms"] = timed(raw_ptr)
    res["raw_enter_ms"] = timed(raw_enter)
    res["handle_fwd_ms"] = timed(handle_fwd)
    res["fresh_ptr_ms"] = timed(fresh_ptr)
    side = torch.cuda.Stream(device=dev)
    torch.cuda.synchronize()
    bs.handle.set_stream(side.cuda_stream)
    with torch.cuda.stream(side):
        res["wrapped_on_callers_stream_ms"] = timed(wrapped)
    torch.cuda.synchronize()
    res["raw_spin25_before_fwd_ms"] = timed(raw_spin_fwd)
    res["raw_spin25_before_bwd_ms"] = timed(raw_spin_bwd)
    res["raw_current_stream_ms"] = timed(raw_curstream)
    # host issue time alone (the queue absorbs 50 solves)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        raw()
    res["raw_issue_ms"] = (time.perf_counter() - t0) / 50 * 1e3
    torch.cuda.synchronize()
    res["status_ok"] = bool((bs.status() == 0).all())
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
