#!/usr/bin/env python3
"""bench.py -- LQR stages/sec on MI355X (driver contract).

Workload (north_star target): batch = 4096 independent
synthetic LQRs per GPU, N = 1024, nx = 12, nu = 4, fp64, model resident in HBM.
One step = backward + forward of the batched serial Riccati (the reference's
timed region, examples/lqr_example.cpp:197-202).  value = N * batch * n_gpus /
(time per step, max over ranks): weak scaling, no data-path collective (the
problems are independent; a barrier and a max-reduce of the clock only).

Roofline: the dominant kernel (k_riccati_bwd) timed with HIP events on the
handle's stream; algorithmic bytes per stage = SURVEY.md 8(d)'s compulsory
reads of E, c, H, h = 8 (n s + n + s^2 + s) (3,808 B at 12/4); the forward
kernel owns the w write (128 B), 3,936 B per stage in all.  `traffic` comes
from the committed rocprofv3 PMC summary (profiles/) when it matches.

cpu_baseline: the Eigen-free C restatement (oracle/, "port"), batched serial
solves with OpenMP on the host cores, rank 0 only, bounded sample.

Run:  python bench.py [--gpus N --steps K --warmup W]
 N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pdp-lqr_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "LQR stages/sec (N*batch) at nx=12,nu=4; wall-clock/solve; 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_PEAK_TF = 78.6    # MI355X fp64 (vector = matrix)


def gen_batch_device(n, m, N, batch, seed, device):
    """Synthetic LQR batch (BASELINE.md section 3 distribution) generated on the
    GPU directly in the boundary layout (include/pdplqr.h)."""
    f64 = torch.float64
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    s = n + m
    E = torch.empty(batch, N, s, n, dtype=f64, device=device)  # column-major n x s blocks
    E[:, :, :m, :] = torch.randn(batch, N, m, n, dtype=f64, device=device, generator=g)
    E[:, :, m:, :] = 0.1 * torch.randn(batch, N, n, n, dtype=f64, device=device, generator=g)
    E[:, :, m:, :] += torch.eye(n, dtype=f64, device=device)
    c = torch.randn(batch, N, n, dtype=f64, device=device, generator=g)
    H = torch.empty(batch, N * s * s + n * n, dtype=f64, device=device)
    chunk = max(1, (1 << 27) // (N * s * s))
    for b0 in range(0, batch, chunk):
        b1 = min(batch, b0 + chunk)
        M = torch.randn(b1 - b0, N, s, s, dtype=f64, device=device, generator=g)
        Hk = M @ M.transpose(-1, -2) / s + torch.eye(s, dtype=f64, device=device)
        H[b0:b1, :N * s * s] = Hk.reshape(b1 - b0, N * s * s)
        del M, Hk
    MN = torch.randn(batch, n, n, dtype=f64, device=device, generator=g)
    H[:, N * s * s:] = (MN @ MN.transpose(-1, -2) / n + torch.eye(n, dtype=f64, device=device)).reshape(batch, n * n)
    h = torch.randn(batch, N * s + n, dtype=f64, device=device, generator=g)
    x0 = torch.randn(batch, n, dtype=f64, device=device, generator=g)
    return E.reshape(batch, -1).contiguous(), c.reshape(batch, -1).contiguous(), H, h, x0


def _pmc_summaries():
    """Every committed rocprofv3 PMC summary (profiles/**/*_pmc.json), oldest
    first: top-level files (rounds 1-2), then profiles/rNN/ in round order, so
    the last match for a workload is the newest."""
    pdir = os.path.join(ROOT, "profiles")
    out = []
    for dp, dns, fs in os.walk(pdir):
        dns.sort()
        for f in sorted(fs):
            if f.endswith("_pmc.json"):
                try:
                    d = json.load(open(os.path.join(dp, f)))
                except Exception:
                    continue
                d["_path"] = os.path.relpath(os.path.join(dp, f), ROOT)
                out.append(d)
    return out


def load_pmc_traffic(workload_tag, kernel=None):
    """Per-launch HBM bytes of the dominant kernel from the newest committed
    rocprofv3 PMC summary, or None.  Only a summary collected on the same
    workload AND the same backward kernel counts."""
    best = None
    names = [kernel] if kernel else []
    if kernel and kernel.endswith(", 0>"):  # pre-round-4 name of the same kernel
        names.append(kernel[:-4] + ">")
    if kernel and kernel.endswith(">"):  # round-5+ name: the one-wave-per-SIMD flag appended (false here)
        names.append(kernel[:-1] + ", false>")
    for d in _pmc_summaries():
        if (d.get("workload") == workload_tag and "bytes_per_launch" in d
                and (kernel is None or any(d.get("dominant_kernel", "").endswith(k) for k in names))):
            best = d
    return best


def pmc_traffic(workload_tag, kernels):
    """HBM bytes per solve of a secondary workload from the newest committed PMC
    summary with this workload tag: the sum over the solve's kernels (name
    substrings) of FETCH_SIZE x 2 + WRITE_SIZE (KB; gfx950 correction of
    MI355X_MICROARCH.md), or None."""
    found = None
    for d in _pmc_summaries():
        if d.get("workload") == workload_tag:
            found = d
    if not found:
        return None
    tot, seen = 0.0, []
    for sub in kernels:
        opt = sub.startswith("?")  # "?name": counted when that kernel ran in the profile
        sub = sub.lstrip("?")
        ks = [k for k in found.get("kernels", {}) if sub in k]
        if not ks:
            if opt:
                continue
            return None
        c = found["kernels"][ks[0]]
        if "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
            return None
        # dispatches per solve: counted when the profile made only this workload's
        # solves (PMC_SOLVES), else one per solve
        mult = c.get("dispatches", 1) / found["solves"] if found.get("solves") else 1.0
        tot += (c["FETCH_SIZE"] * 1024 * 2 + c["WRITE_SIZE"] * 1024) * mult
        seen.append(ks[0])
    return {"bytes": tot, "kernels": seen, "path": found.get("_path", "profiles/")}


def roofline_block(bytes_stage, stages, ms, workload_tag=None, kernels=(), flops_stage=None, kernel_desc=None):
    """roofline of a secondary line: SURVEY.md 8(d) algorithmic bytes per stage x
    stages over the measured solve time, against the 8 TB/s HBM spec; traffic =
    counter bytes of the same workload from a committed profile (profiles/),
    frac_moved = traffic / time / peak; flops (if given) against fp64 peak."""
    achieved = bytes_stage * stages / (ms * 1e-3) / 1e9
    r = {"kernel": kernel_desc, "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": achieved / HBM_PEAK_GBS, "bytes_per_stage_algorithmic": bytes_stage, "ms": ms}
    t = pmc_traffic(workload_tag, kernels) if workload_tag else None
    r["traffic"] = t["bytes"] if t else None
    r["traffic_source"] = (f"committed PMC summary {t['path']}, workload {workload_tag}: {', '.join(t['kernels'])}"
                           if t else "no committed PMC summary for this workload")
    if t:
        r["frac_moved"] = t["bytes"] / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS
        r["traffic_over_algorithmic"] = t["bytes"] / (bytes_stage * stages)
    if flops_stage:
        tf = flops_stage * stages / (ms * 1e-3) / 1e12
        r["fp64_tflops"] = tf
        r["fp64_frac"] = tf / FP64_PEAK_TF
    return r


def cpu_baseline(n, m, N, seconds=12.0, sample_batch=64, threads=None):
    """Oracle ("port") batched serial solves on host cores; bounded sample."""
    sys.path.insert(0, ROOT)
    from oracle.oracle import batched_serial_solve
    from pdplqr.problems import random_batch_arrays

    if threads is None:
        try:
            threads = len(os.sched_getaffinity(0))
        except Exception:
            threads = os.cpu_count() or 1
        threads = max(1, min(16, threads))  # the GPU box grants a 16-CPU share per GPU
    E, c, H, h, x0 = random_batch_arrays(n, m, N, sample_batch, 7)
    batched_serial_solve(n, m, N, E[:threads], c[:threads], H[:threads], h[:threads], x0[:threads],
                         threads=threads)  # warm-up
    reps, t0 = 0, time.perf_counter()
    while True:
        batched_serial_solve(n, m, N, E, c, H, h, x0, threads=threads)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    stages = reps * sample_batch * N
    return {"value": stages / el, "unit": "stages/s", "cores": threads, "kind": "port",
            "sample": f"{reps} x {sample_batch} problems of N={N} nx={n} nu={m} (batched serial Riccati, "
                      f"OpenMP over problems, {el:.1f} s)",
            "cpu_model": cpu_model(),
            "variants": {"C2_serial_1core": cpu_single_problem(n, m, N),
                         "C2_parallel_all_cores": cpu_parallel_problem(n, m, N, threads)}}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_parallel_problem(n, m, N, threads, seconds=2.0):
    """SURVEY.md 8(d) baseline (ii): one problem, the LQRParallelSolver
    restatement with num_segments = the host cores granted (an OpenMP team of
    that many threads, pinned one per CPU as lqr_solver_parallel.hpp:102-112
    does), load balancing (alpha = 1.55), CHOLESKY condensed system; bounded
    to ~2 s.  Run last: the pinning stays on the OpenMP pool's threads."""
    from oracle.oracle import OracleParallel
    from pdplqr.model import PackedModel
    from pdplqr.problems import random_batch_arrays

    E, c, H, h, x0 = random_batch_arrays(n, m, N, 1, 77)
    pm = PackedModel(n, m, N, np.zeros(N + 1, dtype=np.int32), E[0], c[0], H[0], h[0], np.zeros(0))
    saved = os.sched_getaffinity(0)
    o = OracleParallel(pm, threads, load_balancing=True, condensed="CHOLESKY")
    pinned = o.set_threads(True, True)
    o.update_problem_data(np.zeros(N * (n + m) + n), None, None, None, 1e-6)
    o.backward(None)
    o.forward(x0[0])  # warm-up
    reps, t0 = 0, time.perf_counter()
    while True:
        o.backward(None)
        o.forward(x0[0])
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    os.sched_setaffinity(0, saved)  # the calling thread was team thread 0
    return {"ms_per_solve": el / reps * 1e3, "stages_per_s": N * reps / el, "cores": threads,
            "threads_pinned": pinned, "num_segments": threads,
            "sample": f"{reps} solves of one N={N} nx={n} nu={m} problem"}


def cpu_single_problem(n, m, N, seconds=2.0):
    """SURVEY.md 8(d) baseline (i): one problem, the serial LQRSolver
    restatement on one core (backward + forward), the CPU counterpart of the
    C2 line; bounded to ~2 s."""
    from oracle.oracle import OracleSerial
    from pdplqr.model import PackedModel
    from pdplqr.problems import random_batch_arrays

    E, c, H, h, x0 = random_batch_arrays(n, m, N, 1, 77)
    pm = PackedModel(n, m, N, np.zeros(N + 1, dtype=np.int32), E[0], c[0], H[0], h[0], np.zeros(0))
    o = OracleSerial(pm)
    o.update_problem_data(np.zeros(N * (n + m) + n), None, None, None, 1e-6)
    o.backward(None)
    o.forward(x0[0])  # warm-up
    reps, t0 = 0, time.perf_counter()
    while True:
        o.backward(None)
        o.forward(x0[0])
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"ms_per_solve": el / reps * 1e3, "stages_per_s": N * reps / el, "cores": 1,
            "sample": f"{reps} solves of one N={N} nx={n} nu={m} problem"}


BACKEND = os.environ.get("PDPLQR_BENCH_BACKEND", "nccl")


def _max_over_ranks(dist, value, dev):
    t = torch.tensor([value], dtype=torch.float64, device=dev if BACKEND == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _timed(fn, steps, warmup, dev, dist):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    if dist:
        el = _max_over_ranks(dist, el, dev)
    return el / steps


def _timed_local(fn, steps, warmup, dev):
    """This rank alone (no barrier, no max over ranks): seconds per call."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) / steps


def measured_copy_gbs(dev, nbytes=1 << 32, reps=5):
    """Achievable HBM rate, read + write bytes / time of a 4 GiB device copy:
    {"float4": the 16-byte copy kernels (csrc/probe_pattern.hip, the guide's
    6.29 TB/s probe shape: best of one element per thread and a short
    grid-stride sweep), "blit":
    torch's copy_ (the runtime's blit kernel)}.  float4 is None without the
    probe library."""
    import ctypes

    a = torch.empty(nbytes // 8, dtype=torch.float64, device=dev)
    b = torch.empty_like(a)
    a.fill_(1.0)
    b.copy_(a)
    torch.cuda.synchronize(dev)
    stream = torch.cuda.current_stream(dev)

    def rate(launch):
        launch()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            launch()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        return 2 * nbytes / (e0.elapsed_time(e1) / reps * 1e-3) / 1e9

    out = {"blit": rate(lambda: b.copy_(a)), "float4": None}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "pdp-lqr_amd", "pdplqr", "libpdplqr_probe.so")
    if os.path.exists(path):
        fn = ctypes.CDLL(path).pdplqr_probe_copy_mode
        fn.restype = ctypes.c_int
        fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]

        def launcher(mode, blocks=0):
            def go():
                rc = fn(a.data_ptr(), b.data_ptr(), nbytes, mode, blocks, ctypes.c_void_p(stream.cuda_stream))
                if rc != 0:
                    raise RuntimeError(f"pdplqr_probe_copy_mode: hip error {rc}")
            return go

        # mode 1: one 16-byte element per thread over a grid covering the
        # buffer once -- the guide's float4 copy shape (6.21 TB/s against the
        # guide's 6.29, scripts/copy_sweep.py, profiles/r06/copy_sweep.log);
        # the grid-stride form (mode 0) peaks near 5.2
        out["float4"] = max([rate(launcher(1))] + [rate(launcher(0, bl)) for bl in (8192, 32768)])
    del a, b
    torch.cuda.empty_cache()
    return out


def pattern_ceiling_ms(dev, n, m, N, batch, reps=5):
    """Time of the serial kernels' own HBM access pattern with no arithmetic
    (libpdplqr_probe.so, csrc/probe_pattern.hip): one wave per problem streams
    the stage records the kernel reads and writes its per-stage output.
    Returns {"backward": ms, "forward": ms}, or None when the probe library
    is absent.  Backward: E | packed H~ + h~ | c in, rollout record out;
    forward: E | c | record in, w_k out (all 16-byte chunks per stage; the record
    in the form the backward leaves it)."""
    import ctypes

    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "pdp-lqr_amd", "pdplqr",
                        "libpdplqr_probe.so")
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    fn = lib.pdplqr_probe_pattern
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int] * 3 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                         ctypes.c_void_p, ctypes.c_void_p]
    s = n + m
    ch = lambda doubles: (doubles + 1) // 2  # noqa: E731
    # rollout record: gain form [K~ | k~] on the 12/4 value-form path, else [L(:, 0:m) | lu']
    gain = (n, m) == (12, 4)
    rE, rH, rc, rR, rw = ch(n * s), ch(s * (s + 1) // 2 + s), ch(n), ch(n * m + m if gain else s * m + m), ch(s)
    st = N * batch
    bufs = [torch.zeros(st * r * 2, dtype=torch.float64, device=dev) for r in (rE, rH, rc, rR)]
    out = torch.empty(st * max(rR, rw) * 2, dtype=torch.float64, device=dev)
    sink = torch.zeros(1, dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev)
    res = {}
    for name, (a0, r0), (a1, r1), (a2, r2), r_out in (
            ("backward", (bufs[0], rE), (bufs[1], rH), (bufs[2], rc), rR),
            ("forward", (bufs[0], rE), (bufs[2], rc), (bufs[3], rR), rw)):
        def launch():
            rc_ = fn(a0.data_ptr(), r0, a1.data_ptr(), r1, a2.data_ptr(), r2, out.data_ptr(), r_out, batch, N,
                     sink.data_ptr(), ctypes.c_void_p(stream.cuda_stream))
            if rc_ != 0:
                raise RuntimeError(f"pdplqr_probe_pattern: hip error {rc_}")
        launch()
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps)]
        for i in range(reps):
            e[2 * i].record(stream)
            launch()
            e[2 * i + 1].record(stream)
        torch.cuda.synchronize(dev)
        res[name] = min(e[2 * i].elapsed_time(e[2 * i + 1]) for i in range(reps))
    del bufs, out, sink
    torch.cuda.empty_cache()
    return res


def bench_batched_c3(local, dev, dist, steps=10, warmup=3, N=256, batch=4096, n=12, m=4):
    """C3: batch 4096 independent LQRs, N = 256, 12/4 (MPC-style batched solve):
    backward + forward of the serial solver, as the headline line, plus an
    oracle check of two problems.  Also the wide-shape line (VERDICT r2 item 5:
    24/16, batch 1024 -- kernels_wide.hip's value-form backward on 256-thread
    blocks and k_riccati_fwd_big)."""
    from oracle.oracle import OracleSerial
    from pdplqr import BatchedLQRSolver
    from pdplqr.model import PackedModel

    E, c, H, h, x0 = gen_batch_device(n, m, N, batch, seed=4321, device=dev)
    ws0 = torch.zeros(batch, N * (n + m) + n, dtype=torch.float64, device=dev)
    out = torch.empty_like(ws0)
    bs = BatchedLQRSolver(n, m, N, batch, keep_factors=False, device=local)
    bs.set_model(E, c, H, h)
    bs.update_problem_data(ws0, sigma=1e-6)

    def step():
        bs.backward()
        bs.forward(x0, out)

    t = _timed(step, steps, warmup, dev, dist)
    ok = bool(np.all(bs.status() == 0)) and bool(torch.isfinite(out).all().item())
    bs.close()
    err = 0.0
    for b in (0, batch - 1):
        pm = PackedModel(n, m, N, np.zeros(N + 1, dtype=np.int32), *(a[b].cpu().numpy() for a in (E, c, H, h)),
                         np.zeros(0))
        o = OracleSerial(pm)
        o.update_problem_data(np.zeros(N * (n + m) + n), None, None, None, 1e-6)
        o.backward(None)
        ref = o.forward(x0[b].cpu().numpy())
        err = max(err, float(np.linalg.norm(out[b].cpu().numpy() - ref) / np.linalg.norm(ref)))
    del E, c, H, h
    torch.cuda.empty_cache()
    bst = 8 * (n * (n + m) + n + (n + m) ** 2 + (n + m)) + 8 * (n + m)  # 3,936 B at 12/4
    wide = n + m > 32
    if (n, m) == (24, 16):  # the 3 x 3 register-tile backward and rollout (kernels_riccati.hip)
        kern = ("k_riccati_bwd_vf3", "k_rollout_dma3")
    else:
        kern = ("k_seg_bwd_wide", "k_riccati_fwd_big") if wide else ("k_riccati_bwd_schur", "k_rollout_dma")
    tag = f"C3_N{N}_b{batch}" if (n, m) == (12, 4) else f"W_n{n}_m{m}_N{N}_b{batch}"
    s_ = n + m
    # value-form stage flops: P E (2 n^2 s), E^T (P E) lower (n s (s + 1)), u-pivots (~m s^2)
    fl = 2 * n * n * s_ + n * s_ * (s_ + 1) + m * s_ * s_
    return {"N": N, "nx": n, "nu": m, "batch": batch, "ms_per_solve": t * 1e3, "stages_per_s": N * batch / t,
            "status_ok": ok, "oracle_rel_err": err,
            "roofline": roofline_block(bst, N * batch, t * 1e3, tag, kern, flops_stage=fl if wide else None,
                                       kernel_desc="backward + forward")}


def bench_factor_reuse(local, dev, dist, steps=10, warmup=3, N=1024, batch=4096):
    """SURVEY.md 8(f) rank 1 at the headline config: backward_without_factorization
    + forward (lqr_solver.hpp:65-77) on factors cached by one factorising
    backward, the per-iteration cost of an ADMM loop.  The right-hand side
    changes between the factorisation and the timed calls (new w-bar), so the
    oracle check (two problems, factorising OracleSerial on the new data) sees
    the reused factors applied to new linear terms.  Roofline of the streamed
    k_nofact_dma: it reads the per-stage record [E | c | h~ | L packed] and
    writes lp (8 (n s + n + s + s(s+1)/2) + 8 s bytes per stage)."""
    from oracle.oracle import OracleSerial
    from pdplqr import BatchedLQRSolver
    from pdplqr.model import PackedModel

    n, m = 12, 4
    s = n + m
    E, c, H, h, x0 = gen_batch_device(n, m, N, batch, seed=2468, device=dev)
    ws0 = torch.zeros(batch, N * s + n, dtype=torch.float64, device=dev)
    ws1 = torch.randn(batch, N * s + n, dtype=torch.float64, device=dev,
                      generator=torch.Generator(device=dev).manual_seed(5))
    out = torch.empty_like(ws0)
    sigma = 1e-3
    bs = BatchedLQRSolver(n, m, N, batch, keep_factors=True, device=local)
    bs.set_model(E, c, H, h)
    bs.update_problem_data(ws0, sigma=sigma)
    bs.backward()
    bs.update_problem_data(ws1, sigma=sigma)  # same H~, new h~ = h - sigma w-bar
    stream = torch.cuda.ExternalStream(bs.handle.stream(), device=dev)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    it = iter(evs)

    def step():
        e = next(it, None)
        if e:
            e[0].record(stream)
        bs.backward_without_factorization()
        if e:
            e[1].record(stream)
        bs.forward(x0, out)
        if e:
            e[2].record(stream)

    for _ in range(warmup):
        bs.backward_without_factorization()
        bs.forward(x0, out)
    t = _timed(step, steps, 0, dev, dist)
    bs.synchronize()
    ms_bwd = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    ms_fwd = float(np.mean([e[1].elapsed_time(e[2]) for e in evs]))
    ok = bool(np.all(bs.status() == 0)) and bool(torch.isfinite(out).all().item())
    bs.close()
    err = 0.0
    for b in (0, batch - 1):
        pm = PackedModel(n, m, N, np.zeros(N + 1, dtype=np.int32), *(a[b].cpu().numpy() for a in (E, c, H, h)),
                         np.zeros(0))
        o = OracleSerial(pm)
        o.update_problem_data(ws1[b].cpu().numpy(), None, None, None, sigma)
        o.backward(None)
        ref = o.forward(x0[b].cpu().numpy())
        err = max(err, float(np.linalg.norm(out[b].cpu().numpy() - ref) / np.linalg.norm(ref)))
    del E, c, H, h, ws0, ws1, out
    torch.cuda.empty_cache()
    stages = N * batch
    bytes_stage = 8 * (n * s + n + s + s * (s + 1) // 2) + 8 * s
    achieved = bytes_stage * stages / (ms_bwd * 1e-3) / 1e9
    kern = "k_nofact_dma<12, 4, 4>"
    pmc = load_pmc_traffic(f"nofact_N{N}_n{n}_m{m}_b{batch}", kern)
    return {"N": N, "nx": n, "nu": m, "batch": batch, "ms_per_iteration": t * 1e3, "stages_per_s": stages / t,
            "kernels_ms": {"backward_without_factorization": ms_bwd, "forward": ms_fwd},
            "roofline": {"kernel": kern, "bound": "hbm", "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": (pmc["bytes_per_launch"] if pmc else None),
                         "bytes_per_stage_algorithmic": bytes_stage},
            "status_ok": ok, "oracle_rel_err": err}


def bench_single(local, dev, dist, steps=10, warmup=3):
    """C2: one N = 1024, 12/4 problem, LQRParallelSolver path (segments + scans).
    Latency-bound; stages/s = N / time of backward + forward (every rank runs a
    replica)."""
    from pdplqr import BatchedLQRSolver

    n, m, N = 12, 4, 1024
    E, c, H, h, x0 = gen_batch_device(n, m, N, 1, seed=77, device=dev)
    ws0 = torch.zeros(1, N * (n + m) + n, dtype=torch.float64, device=dev)
    out = torch.empty_like(ws0)
    res = {}
    for solver in ("parallel", "serial"):
        bs = BatchedLQRSolver(n, m, N, 1, solver=solver, num_segments=8, keep_factors=(solver == "parallel"),
                              device=local)
        bs.set_model(E, c, H, h)
        bs.update_problem_data(ws0, sigma=1e-6)
        bs.synchronize()
        # the caller's stream is the solver's stream (a latency-bound caller's
        # setup): no cross-stream event joins per call -- they
        # cost ~19 us of the GPU timeline per forward here (profiles/r04/c2_host.log)
        side = torch.cuda.Stream(device=dev)
        bs.handle.set_stream(side.cuda_stream)

        def step():
            bs.backward()
            bs.forward(x0, out)

        with torch.cuda.stream(side):
            t = _timed(step, steps, warmup, dev, dist)
        res[solver] = {"ms_per_solve": t * 1e3, "stages_per_s": N / t, "status_ok": bool(np.all(bs.status() == 0)),
                       "stream": "caller's stream = solver stream"}
        bs.close()
    return res


def bench_conic(local, dev, dist, steps=5, warmup=2, N=512, batch=1024, admm=True):
    """C5: conic (box-constrained u) LQ, N = 512, 12/4, nc = 4 (D = [I 0]) on
    every stage but the terminal, batch 1024, rho = 0.1, random y, z, w-bar.
    One ADMM inner solve = backward + forward, timed for the KKT path
    (QDLDLSolver semantics, kkt.hip) and for the Riccati path on the same data.
    KKT matrix formation (the QDLDLSolver constructor) is outside the timed region."""
    from pdplqr import BatchedLQRSolver

    n, m, nc = 12, 4, 4
    s = n + m
    E, c, H, h, x0 = gen_batch_device(n, m, N, batch, seed=555, device=dev)
    ncs = np.array([nc] * N + [0], dtype=np.int32)
    Dk = torch.zeros(nc, s, dtype=torch.float64, device=dev)
    Dk[:, :m] = torch.eye(m, dtype=torch.float64, device=dev)
    D = Dk.t().contiguous().reshape(-1).repeat(batch, N)  # column-major nc x s blocks
    g = torch.Generator(device=dev)
    g.manual_seed(556)
    ny = nc * N
    ws = torch.randn(batch, N * s + n, dtype=torch.float64, device=dev, generator=g)
    ys = torch.randn(batch, ny, dtype=torch.float64, device=dev, generator=g)
    zs = torch.randn(batch, ny, dtype=torch.float64, device=dev, generator=g)
    rho = torch.full((batch, ny), 0.1, dtype=torch.float64, device=dev)
    irho = 1.0 / rho
    out = torch.empty(batch, N * s + n, dtype=torch.float64, device=dev)
    res = {"N": N, "nx": n, "nu": m, "nc": nc, "batch": batch}
    for solver in ("kkt", "serial"):
        bs = BatchedLQRSolver(n, m, N, batch, solver=solver, ncs=ncs, device=local)
        bs.set_model(E, c, H, h, D)
        bs.update_problem_data(ws, ys, zs, irho, sigma=1e-6)
        r = irho if solver == "kkt" else rho
        # the solver on the caller's stream, as the C2 line (no per-call event joins)
        bs.synchronize()
        torch.cuda.synchronize(dev)
        side = torch.cuda.Stream(device=dev)
        bs.handle.set_stream(side.cuda_stream)

        def step():
            bs.backward(r)
            bs.forward(x0, out)

        # the reference's protocol (lqr_example.cpp:176-183): update_problem_data,
        # untimed, before every timed backward + forward; events on the solver's
        # stream bracket the backward + forward only
        nrep = steps + warmup
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(nrep)]
        with torch.cuda.stream(side):
            for e0, e1 in evs:
                bs.update_problem_data(ws, ys, zs, irho, sigma=1e-6)
                e0.record(side)
                step()
                e1.record(side)
            torch.cuda.synchronize(dev)
            t_proto = float(np.mean([e0.elapsed_time(e1) for e0, e1 in evs[warmup:]])) * 1e-3
            if dist:
                t_proto = _max_over_ranks(dist, t_proto, dev)
            # back to back (no update in between): a state the reference's timed
            # region never has, kept as an extra key
            t_b2b = _timed(step, steps, warmup, dev, dist)
            # one fresh protocol round for the check: the KKT forward accumulates the
            # x0 terms of its rhs on every call (kkt.hpp:207-222, as the reference)
            bs.update_problem_data(ws, ys, zs, irho, sigma=1e-6)
            step()
        torch.cuda.synchronize(dev)
        t = t_proto
        ok = bool(np.all(bs.status() == 0)) and bool(torch.isfinite(out).all().item())
        # C5 = 4,704 B per stage (E, c, H, h, w + D, y, z, inv_rho, rho, w-bar)
        bst = 8 * (n * s + n + s * s + s) + 8 * s + 8 * (nc * s + 4 * nc + s)
        # the serial path's rho penalty is fused into the streamed backward
        # (k_riccati_bwd_schur<12, 4, true, 4>); k_penalty runs where it is not
        kern = ("k_kkt_ric_bwd", "k_kkt_ric_fwd") if solver == "kkt" else ("?k_penalty", "k_riccati_bwd_schur",
                                                                              "k_rollout_dma")
        res["kkt" if solver == "kkt" else "riccati"] = {
            "ms_per_solve": t * 1e3, "stages_per_s": N * batch / t, "status_ok": ok,
            "timing": "update_problem_data (untimed) before every timed backward + forward, lqr_example.cpp:176-183",
            "ms_per_solve_back_to_back": t_b2b * 1e3,
            "oracle_rel_err": _conic_oracle_err(solver, n, m, N, ncs, E, c, H, h, D, x0, ws, ys, zs, irho, rho, out),
            "roofline": roofline_block(bst, N * batch, t * 1e3, f"C5_N{N}_b{batch}", kern,
                                       kernel_desc="backward + forward")}
        bs.close()
    if not admm:  # (scripts/prof_secondary.py c5solve: PMC passes of the solves alone)
        del E, H, D
        torch.cuda.empty_cache()
        return res
    # the ADMM outer loop on the same data (pdplqr_admm_solve): |u| <= 0.5,
    # rho = 1, from a cold start.  (a) 100 fixed iterations (eps = 0, one
    # termination test at the end): iterations/s of the batch; (b) a run to
    # OSQP's default tolerances (1e-3, test every 25 iterations, at most 500).
    lb = torch.full((batch, ny), -0.5, dtype=torch.float64, device=dev)
    ub = torch.full((batch, ny), 0.5, dtype=torch.float64, device=dev)
    rho1 = torch.full((batch, ny), 1.0, dtype=torch.float64, device=dev)
    w0 = torch.zeros(batch, N * s + n, dtype=torch.float64, device=dev)
    y0 = torch.zeros(batch, ny, dtype=torch.float64, device=dev)
    wa, ya, za = w0.clone(), y0.clone(), y0.clone()
    for solver in ("serial", "kkt"):
        bs = BatchedLQRSolver(n, m, N, batch, solver=solver, ncs=ncs, keep_factors=(solver == "serial"),
                              device=local)
        bs.set_model(E, c, H, h, D)
        iters = 100 if solver == "serial" else 30

        def step():
            wa.copy_(w0)
            ya.zero_()
            za.zero_()
            bs.admm_solve(x0, lb, ub, rho1, wa, ya, za, max_iter=iters, check_every=iters, eps_abs=0.0, eps_rel=0.0)

        t = _timed(step, max(1, steps // 2), 1, dev, dist)
        ok = bool(np.all(bs.status() == 0)) and bool(torch.isfinite(wa).all().item())
        wa.copy_(w0)
        ya.zero_()
        za.zero_()
        t0 = time.perf_counter()
        info = bs.admm_solve(x0, lb, ub, rho1, wa, ya, za, max_iter=500)
        torch.cuda.synchronize(dev)
        t_conv = time.perf_counter() - t0
        res[f"admm_{'riccati' if solver == 'serial' else 'kkt'}"] = {
            "iterations": iters, "ms_per_iteration": t * 1e3 / iters, "iterations_per_s": iters / t,
            "stages_per_s": N * batch * iters / t, "status_ok": ok,
            "to_tolerance": {"eps": 1e-3, "iterations": info["iterations"],
                             "converged_frac": float(np.mean(info["converged"])), "ms": t_conv * 1e3}}
        bs.close()
    del E, H, D
    torch.cuda.empty_cache()
    return res


def _conic_oracle_err(solver, n, m, N, ncs, E, c, H, h, D, x0, ws, ys, zs, irho, rho, out, probs=(0, -1)):
    """Max relative error of the timed output against the CPU oracle on two
    sampled problems (test infrastructure, outside the timed region)."""
    from oracle.oracle import OracleKKT, OracleSerial
    from pdplqr.model import PackedModel

    err = 0.0
    for b in probs:
        a = [t[b].cpu().numpy() for t in (E, c, H, h, D, x0, ws, ys, zs, irho, rho, out)]
        pm = PackedModel(n, m, N, ncs, *a[:5])
        o = OracleKKT(pm) if solver == "kkt" else OracleSerial(pm)
        o.update_problem_data(a[6], a[7], a[8], a[9], 1e-6)
        o.backward(a[9] if solver == "kkt" else a[10])
        ref = o.forward(a[5])
        err = max(err, float(np.linalg.norm(a[11] - ref) / np.linalg.norm(ref)))
    return err


def bench_horizon(local, dev, dist, world, rank, Ntot, steps=3, warmup=1):
    """C4: one N = Ntot, 24/8 problem, horizon-sharded over the ranks (strong
    scaling): shard backward -> all-gather of slice elements (RCCL when nccl)
    -> shard forward.  value = Ntot / time per solve (max over ranks)."""
    from pdplqr.horizon import HorizonShard, solve_distributed, split_horizon

    n, m = 24, 8
    s = n + m
    N0, N1 = split_horizon(Ntot, world)[rank]
    Nl = N1 - N0
    last = rank == world - 1
    E, c, H, h, x0 = gen_batch_device(n, m, Nl, 1, seed=4242 + rank, device=dev)
    if not last:
        H[:, Nl * s * s:] = 0.0
        h[:, Nl * s:] = 0.0
    x0 = gen_batch_device(n, m, 1, 1, seed=4242, device=dev)[4]  # the same x0 on every rank
    sh = HorizonShard(n, m, Nl, 1, device=local)
    sh.set_model(E, c, H, h)
    ws0 = torch.zeros(1, Nl * s + n, dtype=torch.float64, device=dev)
    out = torch.empty_like(ws0)
    sh.update_problem_data(ws0, sigma=1e-6)
    E0, H0 = E, H  # kept for the oracle check of the 1-GPU line
    del E, H
    if dist:
        step = lambda: solve_distributed(sh, x0, out)
    else:
        elem = torch.empty(1, 1, sh.es, dtype=torch.float64, device=dev)

        def step():
            sh.backward(elem[0], True)
            sh.forward(x0, elem, 1, 0, out)
    # the shard on the caller's (side) stream: backward, all-gather and forward
    # in stream order, no cross-stream event joins (solve_distributed fast path)
    sh.synchronize()
    side = torch.cuda.Stream(device=dev)
    sh.set_stream(side.cuda_stream)
    with torch.cuda.stream(side):
        t = _timed(step, steps, warmup, dev, dist)
    torch.cuda.synchronize(dev)
    ok = bool(torch.isfinite(out).all().item())
    # the parts of the strong-scaling ratio, measured in this run (VERDICT r5
    # item 6): every rank's own solve without the exchange (backward + forward
    # on the gather of the timed solves), the exchange alone (the same
    # all-gather of 3n^2+2n doubles per rank), and rank 0 solving the whole
    # horizon alone on its GPU while the others wait
    scal = {"rank_ms": [t * 1e3], "max_rank_ms": t * 1e3, "exchange_ms": 0.0}
    if dist:
        gat = sh._gathered.to(dev).contiguous()  # the last timed solve's gather
        el1 = torch.empty(1, sh.es, dtype=torch.float64, device=dev)
        with torch.cuda.stream(side):
            def solve_local():
                sh.backward(el1, last)
                sh.forward(x0, gat, world, rank, out)
            tl = _timed_local(solve_local, steps, warmup, dev)
        per = [None] * world
        dist.all_gather_object(per, tl * 1e3)
        ex_in = torch.zeros(1, sh.es, dtype=torch.float64, device=dev if BACKEND == "nccl" else "cpu")
        ex_out = torch.empty(world, 1, sh.es, dtype=ex_in.dtype, device=ex_in.device)

        def exch():
            if BACKEND == "nccl":
                dist.all_gather_into_tensor(ex_out, ex_in)
            else:
                dist.all_gather(list(ex_out.unbind(0)), ex_in)
        scal = {"rank_ms": per, "max_rank_ms": max(per),
                "exchange_ms": _timed(exch, max(steps, 5), warmup, dev, dist) * 1e3}
    sh.close()
    ref_ms = t * 1e3
    if dist:
        ref_ms = None
        if rank == 0:  # the 1-GPU reference of the same horizon, same run
            Ef, cf, Hf, hf, _ = gen_batch_device(n, m, Ntot, 1, seed=4242, device=dev)
            sh1 = HorizonShard(n, m, Ntot, 1, device=local)
            sh1.set_model(Ef, cf, Hf, hf)
            del Ef, Hf
            w1 = torch.zeros(1, Ntot * s + n, dtype=torch.float64, device=dev)
            sh1.update_problem_data(w1, sigma=1e-6)
            e1 = torch.empty(1, 1, sh1.es, dtype=torch.float64, device=dev)
            sh1.synchronize()
            sh1.set_stream(side.cuda_stream)
            with torch.cuda.stream(side):
                def one():
                    sh1.backward(e1[0], True)
                    sh1.forward(x0, e1, 1, 0, w1)
                ref_ms = _timed_local(one, steps, warmup, dev) * 1e3
            sh1.close()
            del w1, e1, cf, hf
            torch.cuda.empty_cache()
        dist.barrier()
    scal["ref_1rank_ms"] = ref_ms
    scal["strong_scaling_ratio"] = (ref_ms / (t * 1e3)) if ref_ms else None
    if not dist:
        scal["rehearsal_R8"] = _horizon_rehearsal(local, dev, Ntot, 8, x0)
    oerr = None
    if world == 1:  # the whole horizon is this rank's: check it against the serial oracle
        oerr = _horizon_oracle_err([(E0[0], c[0], H0[0], h[0])], [out[0].cpu().numpy()], x0[0], n, m, Ntot)
    else:
        # every rank's slice of the trajectory to rank 0, which regenerates the
        # other ranks' model slices (same device generator and seeds) and checks
        # the assembled horizon against the serial oracle
        outs = [None] * world
        dist.all_gather_object(outs, out[0].cpu().numpy())
        if rank == 0:
            parts = []
            for r, (a0, a1) in enumerate(split_horizon(Ntot, world)):
                Er, cr, Hr, hr, _ = gen_batch_device(n, m, a1 - a0, 1, seed=4242 + r, device=dev)
                parts.append((Er[0], cr[0], Hr[0], hr[0]))
                del Er, Hr
            oerr = _horizon_oracle_err(parts, outs, x0[0], n, m, Ntot)
    del E0, H0
    bst = 8 * (n * s + n + s * s + s) + 8 * s  # 15,040 B per stage at 24/8
    # SURVEY 8(d) flop model: 103,235 per stage (backward + forward) + 59,968 for the segment element
    return {"N": Ntot, "nx": n, "nu": m, "n_gpus": world, "ms_per_solve": t * 1e3, "stages_per_s": Ntot / t,
            "scaling": "strong", "finite": ok, "oracle_rel_err": oerr,
            "exchange": "all-gather of 3n^2+2n doubles per rank",
            "parts": dict(scal, note="rank_ms: each rank's backward + forward without the exchange; exchange_ms: "
                                      "the all-gather alone; ref_1rank_ms: rank 0 solving the whole horizon alone "
                                      "in this run; strong_scaling_ratio = ref_1rank_ms / ms_per_solve"),
            "roofline": roofline_block(bst, Ntot, t * 1e3, f"C4_N{Ntot}_R{world}",
                                       ("k_seg_bwd_aug", "k_seg_scan", "k_seg_maps", "k_map_scan", "k_seg_fwd_dma"),
                                       flops_stage=103235 + 59968,
                                       kernel_desc="whole horizon solve (latency-bound: see DESIGN.md section 6)")}


def _horizon_rehearsal(local, dev, Ntot, R, x0, reps=10):
    """The R-GPU split rehearsed on this one GPU (scripts/prof_shards.py's
    method): the R slices solved in turn as R virtual ranks, each rank's
    backward + forward issued `reps` times back to back on its stream (the
    rank's own critical path, as an R-GPU run would see it less the all-gather;
    the gather is the slices' elements of one untimed pass).  Not a multi-GPU
    measurement: the per-rank kernels run alone on the device here."""
    from pdplqr.horizon import HorizonShard, split_horizon

    n, m = 24, 8
    s = n + m
    side = torch.cuda.Stream(device=dev)
    shards, elems, outs = [], [], []
    for r, (N0, N1) in enumerate(split_horizon(Ntot, R)):
        Nl = N1 - N0
        E, c, H, h, _ = gen_batch_device(n, m, Nl, 1, seed=4242 + r, device=dev)
        if r < R - 1:
            H[:, Nl * s * s:] = 0.0
            h[:, Nl * s:] = 0.0
        sh = HorizonShard(n, m, Nl, 1, device=local)
        sh.set_model(E, c, H, h)
        sh.update_problem_data(torch.zeros(1, Nl * s + n, dtype=torch.float64, device=dev), sigma=1e-6)
        sh.synchronize()
        sh.set_stream(side.cuda_stream)
        shards.append(sh)
        elems.append(torch.empty(1, sh.es, dtype=torch.float64, device=dev))
        outs.append(torch.empty(1, Nl * s + n, dtype=torch.float64, device=dev))
        del E, H
    gathered = torch.empty(R, 1, shards[0].es, dtype=torch.float64, device=dev)
    with torch.cuda.stream(side):
        for r, sh in enumerate(shards):
            sh.backward(elems[r], r == R - 1)
            gathered[r].copy_(elems[r])
        per = []
        for r, sh in enumerate(shards):
            def one():
                sh.backward(elems[r], r == R - 1)
                sh.forward(x0, gathered, R, r, outs[r])
            per.append(_timed_local(one, reps, 2, dev) * 1e3)
    ok = all(bool(torch.isfinite(o).all().item()) for o in outs)
    for sh in shards:
        sh.close()
    return {"R": R, "rank_ms": per, "max_rank_ms": max(per), "finite": ok,
            "note": "one-GPU rehearsal of the R-rank split (virtual ranks solved in turn, each rank's calls "
                    "back to back): the per-rank critical path less the all-gather"}


def _horizon_oracle_err(parts, outs, x0, n, m, Ntot):
    """Relative error of a horizon-sharded trajectory against the serial oracle
    over the whole horizon (test infrastructure, outside the timed region).
    parts: per rank (E, c, H, h) of its slice (the last carries the terminal);
    outs: per rank its w slice (stages, then the slice's end state)."""
    from oracle.oracle import OracleSerial
    from pdplqr.model import PackedModel

    s = n + m
    R = len(parts)
    Ls = [p[1].numel() // n for p in parts]
    E = np.concatenate([p[0].cpu().numpy()[:L * n * s] for p, L in zip(parts, Ls)])
    c = np.concatenate([p[1].cpu().numpy() for p in parts])
    H = np.concatenate([p[2].cpu().numpy()[:L * s * s] for p, L in zip(parts, Ls)] +
                       [parts[-1][2].cpu().numpy()[Ls[-1] * s * s:]])
    h = np.concatenate([p[3].cpu().numpy()[:L * s] for p, L in zip(parts, Ls)] +
                       [parts[-1][3].cpu().numpy()[Ls[-1] * s:]])
    w = np.concatenate([o[:L * s] for o, L in zip(outs, Ls)] + [outs[R - 1][Ls[-1] * s:]])
    pm = PackedModel(n, m, Ntot, np.zeros(Ntot + 1, dtype=np.int32), E, c, H, h, np.zeros(0))
    o = OracleSerial(pm)
    o.update_problem_data(np.zeros(Ntot * s + n), None, None, None, 1e-6)
    o.backward(None)
    ref = o.forward(x0.cpu().numpy())
    return float(np.linalg.norm(w - ref) / np.linalg.norm(ref))


def headline_oracle_err(E, c, Hs, h, x0, out, n, m, N, probs):
    """Max relative error of the timed output against the CPU oracle on a few
    problems of the headline batch (test infrastructure, outside the timed
    region).  Hs: the sampled problems' H (the handle keeps its own copy)."""
    from oracle.oracle import OracleSerial
    from pdplqr.model import PackedModel

    err = 0.0
    for b in probs:
        pm = PackedModel(n, m, N, np.zeros(N + 1, dtype=np.int32), E[b].cpu().numpy(), c[b].cpu().numpy(), Hs[b],
                         h[b].cpu().numpy(), np.zeros(0))
        o = OracleSerial(pm)
        o.update_problem_data(np.zeros(N * (n + m) + n), None, None, None, 1e-6)
        o.backward(None)
        ref = o.forward(x0[b].cpu().numpy())
        err = max(err, float(np.linalg.norm(out[b].cpu().numpy() - ref) / np.linalg.norm(ref)))
    return err


def bench_end_to_end(bs, E, c, H, h, x0, ws0, out, dev, dist, local, steps=3, warmup=1, host_batch=256):
    """the solve with what the timed step leaves out.
    device_resident: update_problem_data + backward + forward on the bench
    workload (model resident in HBM).  host_pcie: a host-memory caller on a
    sub-batch of the same problems -- set_model from pageable host arrays (H2D of
    E, c, H, h), update_problem_data from host ws, backward, forward into host
    ws (D2H): the PCIe-inclusive rate (never the headline value)."""
    from pdplqr import BatchedLQRSolver

    B, N = ws0.shape[0], bs.N
    n, m = bs.n, bs.m

    def dev_step():
        bs.update_problem_data(ws0, sigma=1e-6)
        bs.backward()
        bs.forward(x0, out)

    t_dev = _timed(dev_step, steps, warmup, dev, dist)
    Bh = min(host_batch, B)
    Eh, ch, Hh, hh, x0h = (t[:Bh].cpu().numpy() for t in (E, c, H, h, x0))
    wsh = np.zeros((Bh, ws0.shape[1]))
    outh = np.empty_like(wsh)
    hs = BatchedLQRSolver(n, m, N, Bh, keep_factors=False, device=local)

    def host_step():
        hs.set_model(Eh, ch, Hh, hh)
        hs.update_problem_data(wsh, sigma=1e-6)
        hs.backward()
        hs.forward(x0h, outh)

    t_host = _timed(host_step, steps, warmup, dev, dist)
    hs.close()
    return {"device_resident": {"ms_per_solve": t_dev * 1e3, "stages_per_s": N * B / t_dev,
                                "includes": "update_problem_data + backward + forward"},
            "host_pcie": {"batch": Bh, "ms_per_solve": t_host * 1e3, "stages_per_s": N * Bh / t_host,
                          "includes": "set_model H2D + update_problem_data + backward + forward + ws D2H"}}


def bwd_kernel_name(n, m, keep):
    """The backward kernel the C ABI dispatches for this shape (kernels_schur.hip /
    kernels_riccati.hip launch_riccati_backward)."""
    s = n + m
    if not keep and s <= 16:
        if (n, m) == (12, 4):  # the record form rides in the template (kernels_schur.hip GAIN; NC = 0:
            # no fused penalty rows -- summaries before round 4 name it without that argument)
            return "k_riccati_bwd_schur<12, 4, true, 0>"
        return "k_riccati_bwd_schur<0, 0, false>"
    if (n, m) == (12, 4):
        return f"k_riccati_bwd_fast<1, 12, 4, {str(bool(keep)).lower()}>"
    return "k_riccati_bwd<1>" if s <= 16 else "k_riccati_bwd<2>"


def _spawn_ranks(n):
    """One child process per rank (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in
    its environment, rendezvous on 127.0.0.1), as torch.distributed.run would
    start them; returns the first non-zero exit status.  A rank that fails ends
    the others (they would wait in a collective): the exact PIDs started here."""
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r and not rc:
                rc = r
                for q in live:
                    q.terminate()
        time.sleep(0.2)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)  # ~2 s timed at the headline config (visible to a busy sampler)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--N", type=int, default=1024)
    ap.add_argument("--nx", type=int, default=12)
    ap.add_argument("--nu", type=int, default=4)
    ap.add_argument("--batch", type=int, default=4096, help="problems per GPU")
    ap.add_argument("--keep-factors", action="store_true", help="also cache L_k (factor-reuse path)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-secondary", action="store_true", help="skip the C2 / C4 secondary lines")
    ap.add_argument("--c4-N", type=int, default=65536)
    ap.add_argument("--secondary", default="all",
                    help="comma list of secondary lines (C2,C3,wide,reuse,C5,C4) or 'all'")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `python bench.py --gpus N` without a launcher: start the N ranks here
        # (this process has not touched the GPU: nothing before this line does)
        sys.exit(_spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if BACKEND != "nccl":  # rehearsal: more ranks than GPUs share the devices
        local %= max(1, torch.cuda.device_count())
    dist = None
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        # nccl = RCCL over xGMI; PDPLQR_BENCH_BACKEND=gloo rehearses the
        # multi-rank flow on a box with fewer GPUs than ranks
        if BACKEND == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(BACKEND, rank=rank, world_size=world)
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from pdplqr import BatchedLQRSolver

    n, m, N, B = args.nx, args.nu, args.N, args.batch
    s = n + m
    E, c, H, h, x0 = gen_batch_device(n, m, N, B, seed=1234 + rank, device=dev)
    ws0 = torch.zeros(B, N * s + n, dtype=torch.float64, device=dev)
    out = torch.empty_like(ws0)
    bs = BatchedLQRSolver(n, m, N, B, keep_factors=args.keep_factors, device=local)
    bs.set_model(E, c, H, h)
    # the handle holds its own copy; a sub-batch is kept for the host-memory (PCIe) line
    Hk = H[:256].clone() if not args.no_secondary else None
    Hk_full_sample = {b: H[b].cpu().numpy() for b in (0, B // 2, B - 1)}  # the oracle check's problems
    del H
    bs.update_problem_data(ws0, sigma=1e-6)
    bs.synchronize()
    stream = torch.cuda.ExternalStream(bs.handle.stream(), device=dev)

    def step(evs=None):
        if evs:
            evs[0].record(stream)
        bs.backward()
        if evs:
            evs[1].record(stream)
        bs.forward(x0, out)
        if evs:
            evs[2].record(stream)

    for _ in range(args.warmup):
        step()
    bs.synchronize()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
    bs.synchronize()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    st = bs.status()
    # outside the timed region: the timed batch's output is finite and agrees
    # with the CPU oracle on sampled problems (a wrong-but-finite answer would
    # pass the status flags alone)
    finite = bool(torch.isfinite(out).all().item())
    oracle_err = headline_oracle_err(E, c, Hk_full_sample, h, x0, out, n, m, N, (0, B // 2, B - 1))
    status_ok = bool(np.all(st == 0)) and finite and oracle_err < 1e-9
    if dist:
        el = _max_over_ranks(dist, el, dev)
        status_ok = _max_over_ranks(dist, 0.0 if status_ok else 1.0, dev) == 0.0  # every rank's batch
    ms_bwd = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    ms_fwd = float(np.mean([e[1].elapsed_time(e[2]) for e in evs]))
    stages = N * B
    value = stages * world * args.steps / el
    bytes_bwd_stage = 8 * (n * s + n + s * s + s)  # SURVEY.md 8(d) compulsory reads
    bytes_stage = bytes_bwd_stage + 8 * s  # + the w write = B of BASELINE.md section 2
    achieved = bytes_bwd_stage * stages / (ms_bwd * 1e-3) / 1e9
    tag = f"N{N}_n{n}_m{m}_b{B}_kf{int(args.keep_factors)}"
    pmc = load_pmc_traffic(tag, bwd_kernel_name(n, m, args.keep_factors))
    res = {
        "metric": METRIC,
        "value": value,
        "unit": "stages/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (BASELINE.md section 3 distribution, generated on device)",
        "config": {"workload": f"batched serial Riccati backward+forward, N={N} nx={n} nu={m} batch={B} per GPU "
                               "(north_star target config)",
                   "N": N, "nx": n, "nu": m, "batch_per_gpu": B, "solver": "LQRSolver (batched)",
                   "keep_factors": bool(args.keep_factors), "parallelism": f"batch-sharded x{world}"},
        "roofline": {"kernel": bwd_kernel_name(n, m, args.keep_factors), "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": (pmc["bytes_per_launch"] if pmc else None),
                     "bytes_per_stage_algorithmic": bytes_bwd_stage, "ms_per_launch": ms_bwd},
        "kernels_ms": {"backward": ms_bwd, "forward": ms_fwd},
        "solve_hbm_frac": bytes_stage * stages / ((ms_bwd + ms_fwd) * 1e-3) / 1e9 / HBM_PEAK_GBS,
        "status_ok": status_ok,
        "checks": {"factor_status_clean": bool(np.all(st == 0)), "finite": finite,
                   "oracle_rel_err_sampled": oracle_err, "sampled_problems": [0, B // 2, B - 1],
                   "all_ranks": bool(dist)},
    }
    if BACKEND != "nccl":
        # a gloo rehearsal of the multi-rank flow: the ranks share the visible
        # GPU(s), so value / n_gpus are NOT an N-GPU measurement
        res["rehearsal"] = {"backend": BACKEND, "ranks": world, "physical_devices": torch.cuda.device_count(),
                            "note": "ranks share the devices; timings are not a multi-GPU measurement"}
    if pmc:
        # bytes the kernel actually moves (counter bytes of the committed profile
        # of this workload) over the same time: the value-form backward reads
        # the PACKED H~ that update_problem_data writes (136 of 256 doubles at
        # 12/4), so it moves fewer bytes than the 3,808 B algorithmic figure and
        # `frac_of_measured_copy` (algorithmic bytes) can exceed 1
        res["roofline"]["frac_moved"] = pmc["bytes_per_launch"] / (ms_bwd * 1e-3) / 1e9 / HBM_PEAK_GBS
        res["roofline"]["traffic_source"] = (f"committed PMC summary {pmc.get('_path', 'profiles/')}, same workload "
                                             "and kernel; not this run")
    copy = measured_copy_gbs(dev)
    copy_gbs = copy["float4"] or copy["blit"]
    res["roofline"]["peak_measured_copy"] = copy_gbs
    res["roofline"]["peak_measured_copy_blit"] = copy["blit"]
    # fraction of the box's achievable copy rate the kernel uses: its moved
    # (counter) bytes when a committed PMC summary exists, else algorithmic
    moved = pmc["bytes_per_launch"] / (ms_bwd * 1e-3) / 1e9 if pmc else achieved
    res["roofline"]["frac_of_measured_copy"] = moved / copy_gbs
    res["roofline"]["frac_algorithmic_of_measured_copy"] = achieved / copy_gbs
    res["roofline"]["note"] = ("achieved/frac count the SURVEY 8(d) algorithmic bytes (dense s x s H~); the kernel "
                               "reads the packed H~ (s(s+1)/2 doubles), so it moves fewer bytes than that figure; "
                               "frac_moved and frac_of_measured_copy use the counter bytes (peak_measured_copy: the "
                               "16-byte streaming copy kernel, csrc/probe_pattern.hip; _blit: torch copy_)")
    pat = pattern_ceiling_ms(dev, n, m, N, B)
    if pat is not None:
        # the kernels' own access pattern with nothing on the chain: the time
        # their data flow needs on this box (1.0 = at that ceiling)
        res["roofline"]["pattern_ceiling"] = {
            "backward_ms": pat["backward"], "forward_ms": pat["forward"],
            "backward_frac": pat["backward"] / ms_bwd, "forward_frac": pat["forward"] / ms_fwd,
            "solve_frac": (pat["backward"] + pat["forward"]) / (ms_bwd + ms_fwd),
            "probe": "csrc/probe_pattern.hip"}
    if not args.no_secondary:
        res["end_to_end"] = bench_end_to_end(bs, E, c, Hk, h, x0, ws0, out, dev, dist, local)
    bs.close()
    del E, c, h, x0, ws0, out, Hk
    torch.cuda.empty_cache()
    if not args.no_secondary:
        lines = [("C2", "C2_single_N1024_parallel", lambda: bench_single(local, dev, dist, steps=50, warmup=5)),
                 ("C3", "C3_batched_N256", lambda: bench_batched_c3(local, dev, dist)),
                 ("wide", "wide_24x16_N256_b1024", lambda: bench_batched_c3(local, dev, dist, steps=5, warmup=2,
                                                                             N=256, batch=1024, n=24, m=16)),
                 ("reuse", "factor_reuse", lambda: bench_factor_reuse(local, dev, dist, N=N, batch=B)),
                 ("C5", "C5_conic_kkt", lambda: bench_conic(local, dev, dist)),
                 ("C4", "C4_horizon_sharded", lambda: bench_horizon(local, dev, dist, world, rank, args.c4_N, steps=10, warmup=2))]
        pick = None if args.secondary == "all" else set(args.secondary.split(","))
        res["secondary"] = {key: fn() for tag, key, fn in lines if pick is None or tag in pick}
    if rank == 0 and not args.no_cpu:
        # rank 0 only, after every timed region (the other ranks are done)
        res["cpu_baseline"] = cpu_baseline(n, m, N, seconds=args.cpu_seconds)
    elif rank == 0:
        res["cpu_baseline"] = None
    assert res["n_gpus"] == args.gpus
    if rank == 0:
        print(json.dumps(res), flush=True)
    if dist:
        dist.destroy_process_group()
    if not res["status_ok"]:
        # a solve that flagged a failed factorisation, a non-finite output or an
        # oracle mismatch on any rank's timed batch does not back its number:
        # report it, then fail the run
        print("bench: status_ok is false (factor status, finiteness or oracle check on the timed batch)",
              file=sys.stderr)
        sys.exit(3)


if __name__ == "__main__":
    main()
