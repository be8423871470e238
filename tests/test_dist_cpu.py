"""world_size-2 gloo test (CPU) of the horizon-sharding exchange protocol
(DESIGN.md section 6): each rank computes its slice element, the elements are
all-gathered, each rank folds the global prefix/suffix and derives its
boundary state.  The per-rank math is the numpy restatement in seg_ref.py
(the HIP kernels cannot run here; tests/test_gpu_horizon.py covers them)."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import load_golden

import dense_ref as dr
import seg_ref as sr


def _worker(rank, world, port, name, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pdplqr.horizon import split_horizon

        pm, d = load_golden(name)
        n, m, N = pm.n, pm.m, pm.N
        E, c, Ht, ht = dr.effective_cost(pm, d["ws"], d["ys"], d["zs"], d["inv_rho"], d["rho"], float(d["sigma"]))
        N0, N1 = split_horizon(N, world)[rank]
        last = rank == world - 1
        e = sr.slice_element(E, c, Ht, ht, N0, N1, (Ht[N], ht[N]) if last else None)
        mine = torch.from_numpy(sr.pack(e))
        parts = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(parts, mine)
        elems = [sr.unpack(p.numpy(), n) for p in parts]
        # global prefix (ranks < r) and suffix (ranks >= r)
        if rank == 0:
            pre = (np.eye(n), np.zeros((n, n)), np.zeros(n), np.zeros((n, n)), np.zeros(n))
        else:
            pre = elems[0]
            for j in range(1, rank):
                pre = sr.combine(pre, elems[j])
        suf = elems[world - 1]
        for j in range(world - 2, rank - 1, -1):
            suf = sr.combine(elems[j], suf)
        x = sr.boundary_state(pre, suf, d["x0"])
        out_q.put((rank, N0, x))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name", ["random_n12_m4_N64_nc4", "quadrotor_N100"])
def test_gloo_two_rank_boundary_states(name):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_worker, args=(r, 2, port, name, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    pm, d = load_golden(name)
    s = pm.n + pm.m
    ref = d["w_riccati"]
    for rank, N0, x in res:
        want = ref[N0 * s + pm.m:(N0 + 1) * s] if N0 < pm.N else ref[pm.N * s:]
        assert np.linalg.norm(x - want) <= 1e-9 * max(1.0, np.linalg.norm(want))


def _worker_nofact(rank, world, port, name, out_q):
    """The backward_without_factorization exchange (horizon.py solve_distributed
    factorize=False): after a full all-gather, new linear data changes only
    every slice element's (f, p); the ranks all-gather those 2n doubles, write
    them into the kept gather and fold it.  F, C, P of the new elements are
    checked equal to the kept ones (what makes the short exchange valid)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pdplqr.horizon import split_horizon

        pm, d = load_golden(name)
        n, N = pm.n, pm.N
        N0, N1 = split_horizon(N, world)[rank]
        last = rank == world - 1

        def element(ws):
            E, c, Ht, ht = dr.effective_cost(pm, ws, d["ys"], d["zs"], d["inv_rho"], d["rho"], float(d["sigma"]))
            return sr.pack(sr.slice_element(E, c, Ht, ht, N0, N1, (Ht[N], ht[N]) if last else None))

        full = torch.from_numpy(element(d["ws"]))
        parts = [torch.empty_like(full) for _ in range(world)]
        dist.all_gather(parts, full)
        kept = torch.stack(parts)
        ws2 = d["ws"] + 0.1 * np.random.default_rng(11).standard_normal(d["ws"].shape)
        new = element(ws2)
        fs, ps = slice(2 * n * n, 2 * n * n + n), slice(3 * n * n + n, 3 * n * n + 2 * n)
        rest = np.ones(new.size, dtype=bool)
        rest[fs] = rest[ps] = False
        same = bool(np.allclose(new[rest], full.numpy()[rest], rtol=1e-13, atol=1e-13))
        fp = torch.from_numpy(np.concatenate([new[fs], new[ps]]))
        fparts = [torch.empty_like(fp) for _ in range(world)]
        dist.all_gather(fparts, fp)
        for q in range(world):
            kept[q, fs] = fparts[q][:n]
            kept[q, ps] = fparts[q][n:]
        elems = [sr.unpack(kept[q].numpy(), n) for q in range(world)]
        if rank == 0:
            pre = (np.eye(n), np.zeros((n, n)), np.zeros(n), np.zeros((n, n)), np.zeros(n))
        else:
            pre = elems[0]
            for j in range(1, rank):
                pre = sr.combine(pre, elems[j])
        suf = elems[world - 1]
        for j in range(world - 2, rank - 1, -1):
            suf = sr.combine(elems[j], suf)
        out_q.put((rank, N0, sr.boundary_state(pre, suf, d["x0"]), same, ws2))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name", ["random_n12_m4_N64_nc4", "quadrotor_N100"])
def test_gloo_two_rank_nofact_exchange(name):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_worker_nofact, args=(r, 2, port, name, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    pm, d = load_golden(name)
    s = pm.n + pm.m
    for rank, N0, x, same, ws2 in res:
        assert same, rank
        ref = dr.riccati_optimum(pm, d["x0"], ws2, d["ys"], d["zs"], d["inv_rho"], d["rho"], float(d["sigma"]))
        want = ref[N0 * s + pm.m:(N0 + 1) * s] if N0 < pm.N else ref[pm.N * s:]
        assert np.linalg.norm(x - want) <= 1e-9 * max(1.0, np.linalg.norm(want))
