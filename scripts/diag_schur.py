"""Diagnostic: value-form backward (kernels_schur.hip) vs the oracle across
horizons and variants.  Variant chosen by env (PDPLQR_NO_DMA / PDPLQR_NO_SCHUR)
in a fresh process per variant."""
import os, sys, subprocess, json
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pdp-lqr_amd"), ROOT]


def run_one():
    from pdplqr import BatchedLQRSolver
    from pdplqr.model import PackedModel
    from pdplqr.problems import random_batch_arrays
    from oracle.oracle import OracleSerial
    n, m = 12, 4
    out = {}
    for N in [2, 8, 64, 200, 1024]:
        batch = 3
        E, c, H, h, x0 = random_batch_arrays(n, m, N, batch, 117)
        s = n + m
        ws0 = np.zeros((batch, N * s + n))
        bs = BatchedLQRSolver(n, m, N, batch, keep_factors=False)
        bs.set_model(E, c, H, h)
        bs.update_problem_data(ws0, sigma=1e-6)
        bs.backward()
        w = np.zeros_like(ws0)
        bs.forward(x0, w)
        errs = []
        for b in range(batch):
            pm = PackedModel(n, m, N, np.zeros(N + 1, dtype=np.int32), E[b], c[b], H[b], h[b], np.zeros(0))
            o = OracleSerial(pm)
            o.update_problem_data(ws0[b], None, None, None, 1e-6)
            o.backward(None)
            wo = o.forward(x0[b])
            d = np.abs(w[b] - wo)
            first = int(np.argmax(d > 1e-12 * (1 + np.abs(wo)))) if np.any(d > 1e-12 * (1 + np.abs(wo))) else -1
            errs.append([float(np.linalg.norm(w[b] - wo) / np.linalg.norm(wo)), first])
        out[N] = {"status": bs.status().tolist(), "errs": errs}
        bs.close()
    print(json.dumps(out))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        run_one()
    else:
        for tag, env in [("dma", {}), ("runtime", {"PDPLQR_NO_DMA": "1"}), ("fullfactor", {"PDPLQR_NO_SCHUR": "1"})]:
            e = dict(os.environ, **env)
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "child"], env=e, capture_output=True,
                               text=True, timeout=300)
            print(tag, r.stdout.strip(), r.stderr[-500:] if r.returncode else "")
