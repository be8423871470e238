"""Diagnostic: the value-form backward's status flag on the bench batch
(N = 1024, 12/4, batch 4096, bench.py's gen_batch_device, seed 1234).

For the library in PDPLQR_LIB (default: in-tree), runs backward + forward
REPS times and reports per run: the failing problems and stages (status =
stage + 1), whether the failure set repeats (numerics) or moves (a race), and
the largest per-problem difference to the full-factor path (PDPLQR_NO_SCHUR,
toggled in-process).  Failing problems and a few random ones are re-solved by
the oracle (OracleSerial) on the host.  JSON to stdout."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pdp-lqr_amd")]

import torch  # noqa: E402

from bench import gen_batch_device  # noqa: E402


def main():
    from oracle.oracle import OracleSerial
    from pdplqr import BatchedLQRSolver
    from pdplqr.model import PackedModel

    n, m, N, B = 12, 4, int(os.environ.get("DIAG_N", 1024)), int(os.environ.get("DIAG_B", 4096))
    reps = int(os.environ.get("DIAG_REPS", 3))
    s = n + m
    dev = torch.device("cuda", 0)
    E, c, H, h, x0 = gen_batch_device(n, m, N, B, seed=1234, device=dev)
    ws0 = torch.zeros(B, N * s + n, dtype=torch.float64, device=dev)
    bs = BatchedLQRSolver(n, m, N, B, keep_factors=False)
    bs.set_model(E, c, H, h)
    bs.update_problem_data(ws0, sigma=1e-6)
    outs, sts = [], []
    for r in range(reps):
        out = torch.empty_like(ws0)
        bs.backward()
        bs.forward(x0, out)
        bs.synchronize()
        outs.append(out.cpu().numpy())
        sts.append(bs.status().copy())
    os.environ["PDPLQR_NO_SCHUR"] = "1"
    out = torch.empty_like(ws0)
    bs.backward()
    bs.forward(x0, out)
    bs.synchronize()
    del os.environ["PDPLQR_NO_SCHUR"]
    ref_ff = out.cpu().numpy()
    st_ff = bs.status().copy()
    bs.close()
    res = {"N": N, "batch": B, "lib": os.environ.get("PDPLQR_LIB", "in-tree"), "runs": []}
    nrm = np.linalg.norm(ref_ff, axis=1)
    for r in range(reps):
        bad = np.nonzero(sts[r])[0]
        d = np.linalg.norm(outs[r] - ref_ff, axis=1) / nrm
        fin = np.isfinite(outs[r]).all(axis=1)
        worst = np.argsort(-np.nan_to_num(d, nan=np.inf))[:8]
        res["runs"].append({"n_fail": int(bad.size), "fail": [[int(b), int(sts[r][b]) - 1] for b in bad[:32]],
                            "n_nonfinite": int((~fin).sum()),
                            "max_rel_vs_fullfactor": float(np.nanmax(np.where(fin, d, np.nan))) if fin.any() else None,
                            "worst": [[int(b), float(d[b])] for b in worst],
                            "n_rel_gt_1e9": int(np.sum(~(d <= 1e-9)))})
    res["same_fail_set"] = all(np.array_equal(np.nonzero(sts[0])[0], np.nonzero(x)[0]) for x in sts)
    res["fullfactor_n_fail"] = int(np.count_nonzero(st_ff))
    # oracle on failing / worst / random problems
    cand = set(int(b) for r in range(reps) for b in np.nonzero(sts[r])[0][:6])
    cand |= set(int(w[0]) for w in res["runs"][0]["worst"][:3])
    cand |= set(int(b) for b in np.random.default_rng(0).choice(B, 3, replace=False))
    Eh, ch, Hh, hh, xh = (t.cpu().numpy() for t in (E, c, H, h, x0))
    orc = {}
    for b in sorted(cand):
        pm = PackedModel(n, m, N, np.zeros(N + 1, dtype=np.int32), Eh[b], ch[b], Hh[b], hh[b], np.zeros(0))
        o = OracleSerial(pm)
        o.update_problem_data(np.zeros(N * s + n), None, None, None, 1e-6)
        o.backward(None)
        wo = o.forward(xh[b])
        on = np.linalg.norm(wo)
        orc[b] = {"fullfactor": float(np.linalg.norm(ref_ff[b] - wo) / on),
                  "schur": [float(np.linalg.norm(outs[r][b] - wo) / on) for r in range(reps)],
                  "status": [int(sts[r][b]) for r in range(reps)], "norm_w": float(on),
                  "max_abs_x": float(np.abs(wo).max())}
    res["oracle"] = orc
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
