"""GPU tests of horizon sharding (pdplqr_shard_backward / pdplqr_shard_forward):
R virtual ranks in one process (host-side all-gather), and 2 real processes
exchanging elements with torch.distributed (gloo) on one GPU.  Compared with
the serial oracle on the full horizon; tolerance 1e-9 relative."""
import os

import numpy as np
import pytest

from conftest import load_golden, rel_err

pytestmark = pytest.mark.gpu
TOL = 1e-9


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    from pdplqr import device_count

    assert device_count() > 0


def _full(n, m, N, batch, seed):
    from pdplqr.problems import random_batch_arrays

    return random_batch_arrays(n, m, N, batch, seed)


def _oracle(n, m, N, E, c, H, h, x0):
    from oracle.oracle import OracleSerial
    from pdplqr.model import PackedModel

    outs = []
    for b in range(E.shape[0]):
        pm = PackedModel(n, m, N, np.zeros(N + 1, dtype=np.int32), E[b], c[b], H[b], h[b], np.zeros(0))
        o = OracleSerial(pm)
        o.update_problem_data(np.zeros(N * (n + m) + n), None, None, None, 1e-6)
        o.backward(None)
        outs.append(o.forward(x0[b]))
    return np.stack(outs)


def _run_virtual(n, m, N, batch, R, seglen, seed=3):
    from pdplqr.horizon import HorizonShard, slice_arrays, split_horizon

    E, c, H, h, x0 = _full(n, m, N, batch, seed)
    s = n + m
    sl = split_horizon(N, R)
    shards, elems = [], []
    for r, (N0, N1) in enumerate(sl):
        last = r == R - 1
        Nl = N1 - N0
        sh = HorizonShard(n, m, Nl, batch, segment_len=seglen)
        sh.set_model(*slice_arrays(E, c, H, h, n, m, N, N0, N1, last))
        sh.update_problem_data(np.zeros((batch, Nl * s + n)), sigma=1e-6)
        e = np.zeros((batch, 3 * n * n + 2 * n))
        sh.backward(e, last)
        shards.append(sh)
        elems.append(e)
    gathered = np.ascontiguousarray(np.stack(elems))
    full = np.zeros((batch, N * s + n))
    ends = []
    for r, (N0, N1) in enumerate(sl):
        Nl = N1 - N0
        loc = np.zeros((batch, Nl * s + n))
        shards[r].forward(x0, gathered, R, r, loc)
        full[:, N0 * s:N1 * s] = loc[:, :Nl * s]
        if r == R - 1:
            full[:, N * s:] = loc[:, Nl * s:]
        else:
            ends.append((N1, loc[:, Nl * s:].copy()))
    for N1, xe in ends:  # each slice-end state is the next slice's first state
        assert rel_err(xe, full[:, N1 * s + m:(N1 + 1) * s]) < TOL
    return full, _oracle(n, m, N, E, c, H, h, x0)


@pytest.mark.parametrize("n,m,N,batch,R,seglen", [(12, 4, 256, 1, 1, 0), (12, 4, 256, 1, 2, 0),
                                                  (12, 4, 200, 2, 3, 7), (24, 8, 96, 1, 4, 8),
                                                  (4, 2, 50, 3, 5, 2)])
def test_virtual_ranks_match_oracle(n, m, N, batch, R, seglen):
    got, ref = _run_virtual(n, m, N, batch, R, seglen)
    for b in range(batch):
        assert rel_err(got[b], ref[b]) < TOL, b


@pytest.mark.parametrize("fold", ["scan", "chain", "tree"])
@pytest.mark.parametrize("n,m,N,batch,R,seglen", [(12, 4, 200, 2, 3, 7), (12, 4, 320, 3, 8, 8),
                                                  (24, 8, 128, 1, 8, 4), (24, 8, 150, 2, 5, 6),
                                                  (20, 6, 133, 2, 7, 5), (24, 8, 96, 3, 2, 6),
                                                  (4, 2, 60, 2, 6, 3)])
def test_virtual_ranks_fold_variants(n, m, N, batch, R, seglen, fold, monkeypatch):
    """The folds of the gathered rank elements (PDPLQR_SHARD_FOLD): the
    sequential prefix / suffix chains, the log-depth rank suffix scan with
    rank boundary maps, and the pairwise prefix / suffix trees (4-wave
    combines, 16 < n <= 32; the chain form elsewhere).  Rank-major strides are
    exercised by batch > 1; R = 5, 7, 8 give carried odd partials and one-
    element lists."""
    monkeypatch.setenv("PDPLQR_SHARD_FOLD", fold)
    got, ref = _run_virtual(n, m, N, batch, R, seglen, seed=5)
    for b in range(batch):
        assert rel_err(got[b], ref[b]) < TOL, b


def _dist_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pdplqr.horizon import HorizonShard, slice_arrays, solve_distributed, split_horizon

        n, m, N = 12, 4, 160
        E, c, H, h, x0 = _full(n, m, N, 1, 11)
        N0, N1 = split_horizon(N, world)[rank]
        last = rank == world - 1
        sh = HorizonShard(n, m, N1 - N0, 1, segment_len=8)
        sh.set_model(*slice_arrays(E, c, H, h, n, m, N, N0, N1, last))
        sh.update_problem_data(np.zeros((1, (N1 - N0) * (n + m) + n)), sigma=1e-6)
        loc = np.zeros((1, (N1 - N0) * (n + m) + n))
        solve_distributed(sh, x0, loc)
        # the gather kept for factorize=False is invalidated by a new
        # model and by a factorising backward outside solve_distributed
        loc2 = np.zeros_like(loc)
        solve_distributed(sh, x0, loc2, factorize=False)  # same data: same answer
        stale = []
        sh.set_model(*slice_arrays(E, c, H, h, n, m, N, N0, N1, last))
        sh.update_problem_data(np.zeros((1, (N1 - N0) * (n + m) + n)), sigma=1e-6)
        for act in ("set_model", "backward"):
            if act == "backward":
                solve_distributed(sh, x0, loc2)
                sh.backward(np.zeros((1, sh.es)), last)
            try:
                solve_distributed(sh, x0, loc2, factorize=False)
                stale.append(act)
            except RuntimeError:
                pass
        q.put((rank, N0, N1, loc, bool(np.allclose(loc, loc2, rtol=1e-12, atol=1e-12)), stale))
    except Exception as e:  # report instead of leaving the parent waiting on the queue
        import traceback

        q.put((rank, -1, -1, None, False, [traceback.format_exc()]))
        raise
    finally:
        dist.destroy_process_group()


def test_two_process_gloo_exchange():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + (os.getpid() % 500)
    ps = [ctx.Process(target=_dist_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(2)], key=lambda r: r[0])
    for r in res:
        assert r[1] >= 0, r[5]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    n, m, N = 12, 4, 160
    s = n + m
    E, c, H, h, x0 = _full(n, m, N, 1, 11)
    ref = _oracle(n, m, N, E, c, H, h, x0)[0]
    full = np.zeros(N * s + n)
    for rank, N0, N1, loc, same, stale in res:
        full[N0 * s:N1 * s] = loc[0, :(N1 - N0) * s]
        if N1 == N:
            full[N * s:] = loc[0, (N1 - N0) * s:]
        assert same and stale == [], (rank, same, stale)
    assert rel_err(full, ref) < TOL


def _nccl_worker(port, q):
    """One rank on the RCCL backend: exercises solve_distributed's device path
    (event ordering between the handle's stream and torch's current stream, no
    host synchronisation), from the default stream and from a side stream."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        from pdplqr.horizon import HorizonShard

        n, m, N = 12, 4, 96
        E, c, H, h, x0 = _full(n, m, N, 2, 13)
        dev = torch.device("cuda", 0)
        sh = HorizonShard(n, m, N, 2, segment_len=8)
        sh.set_model(*[torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (E, c, H, h)])
        sh.update_problem_data(torch.zeros(2, N * (n + m) + n, dtype=torch.float64, device=dev), sigma=1e-6)
        outs = []
        from pdplqr.horizon import solve_distributed

        for it in range(3):  # torch's default stream, a side stream, the shard on that side stream
            if it == 1:
                torch.cuda.set_stream(torch.cuda.Stream())
            if it == 2:  # solve_distributed's no-join path
                sh.synchronize()
                sh.set_stream(torch.cuda.current_stream().cuda_stream)
            out = torch.full((2, N * (n + m) + n), float("nan"), dtype=torch.float64, device=dev)
            solve_distributed(sh, torch.from_numpy(x0).to(dev), out)
            torch.cuda.synchronize()
            outs.append(out.cpu().numpy())
        q.put(outs)
        sh.close()
    finally:
        dist.destroy_process_group()


def test_single_rank_nccl_device_path():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_worker, args=(29300 + (os.getpid() % 400), q))
    p.start()
    outs = q.get(timeout=300)
    p.join(timeout=60)
    assert p.exitcode == 0
    n, m, N = 12, 4, 96
    E, c, H, h, x0 = _full(n, m, N, 2, 13)
    ref = _oracle(n, m, N, E, c, H, h, x0)
    for got in outs:
        for b in range(2):
            assert rel_err(got[b], ref[b]) < TOL, b
    assert len(outs) == 3 and np.array_equal(outs[0], outs[1]) and np.array_equal(outs[0], outs[2])
