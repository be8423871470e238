"""C2 (one N = 1024, 12/4 problem, parallel solver) for rocprofv3 kernel traces."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pdp-lqr_amd")]

import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5  # more for an A/B timing
    print(json.dumps(bench.bench_single(0, dev, None, steps=steps, warmup=2)), flush=True)
