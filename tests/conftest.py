"""Shared pytest setup: path wiring, the ``gpu`` marker and fixture loaders."""
import glob
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "pdp-lqr_amd"), os.path.dirname(os.path.abspath(__file__))):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def load_golden(name):
    """Load a golden fixture (allow_pickle=False) into (PackedModel, dict)."""
    from pdplqr.model import PackedModel

    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    d = {k: z[k] for k in z.files}
    pm = PackedModel(int(d["n"]), int(d["m"]), int(d["N"]), d["ncs"].astype(np.int32), d["E"], d["c"], d["H"],
                     d["h"], d["D"])
    return pm, d


def golden_names():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "*.npz")))


def rel_err(a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def u_parts(w, n, m, N):
    s = n + m
    return np.concatenate([w[k * s:k * s + m] for k in range(N)])


def x_parts(w, n, m, N):
    s = n + m
    return np.concatenate([w[k * s + m:(k + 1) * s] for k in range(N)] + [w[N * s:N * s + n]])
