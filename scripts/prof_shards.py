"""Per-rank cost of the horizon-sharded C4 solve, rehearsed on one GPU with R
virtual ranks (each rank's slice solved in turn on the same device): prints,
per rank, the slice backward and the shard forward (fold of the gathered
elements + boundary maps + rollout) in ms, and the slowest rank's total -- what
an R-GPU run takes per solve, less the all-gather.  bwd_ms / fwd_ms are event
times of single calls on an idle GPU (they include the host's launch latency);
pipelined_ms is the rank's backward + forward issued back to back, wall clock
per solve (bench.py's per-rank figure).
usage: python scripts/prof_shards.py [Ntot=65536] [R=8] [reps=5] [segment_len=0 (automatic)]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pdp-lqr_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from pdplqr.horizon import HorizonShard, split_horizon  # noqa: E402


def main():
    Ntot = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    seglen = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    n, m = 24, 8
    s = n + m
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    st = torch.cuda.Stream()  # one non-default stream for every handle and the events
    torch.cuda.set_stream(st)
    x0 = bench.gen_batch_device(n, m, 1, 1, seed=4242, device=dev)[4]
    shards, elems, outs = [], [], []
    for r, (N0, N1) in enumerate(split_horizon(Ntot, R)):
        Nl = N1 - N0
        E, c, H, h, _ = bench.gen_batch_device(n, m, Nl, 1, seed=4242 + r, device=dev)
        if r < R - 1:
            H[:, Nl * s * s:] = 0.0
            h[:, Nl * s:] = 0.0
        sh = HorizonShard(n, m, Nl, 1, segment_len=seglen, device=0)
        sh.set_model(E, c, H, h)
        sh.update_problem_data(torch.zeros(1, Nl * s + n, dtype=torch.float64, device=dev), sigma=1e-6)
        sh.handle.set_stream(st.cuda_stream)
        shards.append(sh)
        elems.append(torch.empty(1, sh.es, dtype=torch.float64, device=dev))
        outs.append(torch.empty(1, Nl * s + n, dtype=torch.float64, device=dev))
    gathered = torch.empty(R, 1, shards[0].es, dtype=torch.float64, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    res = {"bwd": [[] for _ in range(R)], "fwd": [[] for _ in range(R)]}
    for it in range(reps + 1):
        for r, sh in enumerate(shards):
            ev[0].record()
            sh.backward(elems[r], r == R - 1)
            ev[1].record()
            gathered[r].copy_(elems[r])
        for r, sh in enumerate(shards):
            ev[1].record()
            sh.forward(x0, gathered, R, r, outs[r])
            ev[2].record()
            torch.cuda.synchronize()
            if it:
                res["fwd"][r].append(ev[1].elapsed_time(ev[2]))
        for r, sh in enumerate(shards):  # backward alone, timed
            ev[0].record()
            sh.backward(elems[r], r == R - 1)
            ev[1].record()
            torch.cuda.synchronize()
            if it:
                res["bwd"][r].append(ev[0].elapsed_time(ev[1]))
    # pipelined: each rank's backward + forward issued `reps` times back to back
    # on its stream and timed by the wall clock around them (as bench.py's C4
    # line times a rank): the host's launch latency overlaps the GPU work, as in
    # a distributed solve where the forward is queued behind the all-gather
    import time
    pipe = []
    for r, sh in enumerate(shards):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps * 4):
            sh.backward(elems[r], r == R - 1)
            sh.forward(x0, gathered, R, r, outs[r])
        torch.cuda.synchronize()
        pipe.append((time.perf_counter() - t0) / (reps * 4) * 1e3)
    med = lambda v: sorted(v)[len(v) // 2]
    per = [{"rank": r, "bwd_ms": med(res["bwd"][r]), "fwd_ms": med(res["fwd"][r])} for r in range(R)]
    ok = all(bool(torch.isfinite(o).all().item()) for o in outs)
    for r, p in enumerate(per):
        p["pipelined_ms"] = pipe[r]
    print(json.dumps({"Ntot": Ntot, "R": R, "ranks": per, "max_rank_ms": max(p["bwd_ms"] + p["fwd_ms"] for p in per),
                      "max_rank_ms_pipelined": max(pipe),
                      "finite": ok, "segment_len": seglen, "fold": os.environ.get("PDPLQR_SHARD_FOLD", "auto"), "lib": os.environ.get("PDPLQR_LIB", "in-tree")}), flush=True)
    for sh in shards:
        sh.close()


if __name__ == "__main__":
    main()
