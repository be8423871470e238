"""C5 (conic LQ, N = 512, 12/4, nc = 4, batch 1024): KKT path and Riccati path
on the same data, for rocprofv3 kernel traces.  Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pdp-lqr_amd")]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    print(json.dumps(bench.bench_conic(0, dev, None, steps=3, warmup=1)), flush=True)


if __name__ == "__main__":
    main()
