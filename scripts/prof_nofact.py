"""Factor-reuse pass at the headline config for rocprofv3 (kernel trace / PMC):
one factorising backward, then backward_without_factorization + forward
(bench.bench_factor_reuse, 3 timed iterations).  Prints its bench dict.

usage: python scripts/prof_nofact.py [N] [batch]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pdp-lqr_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
torch.cuda.set_device(0)
print(json.dumps(bench.bench_factor_reuse(0, torch.device("cuda", 0), None, steps=3, warmup=1, N=N, batch=B)))
