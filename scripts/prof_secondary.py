"""One secondary bench workload on its own (for rocprofv3 kernel traces and PMC
passes of exactly that workload): c2 | c3 | c5 | c5solve | c4 [N] | wide.
Prints the bench's JSON for it."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pdp-lqr_amd")]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "c5"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    if which == "c2":
        r = bench.bench_single(0, dev, None, steps=5, warmup=2)
    elif which == "c3":
        r = bench.bench_batched_c3(0, dev, None, steps=5, warmup=2)
    elif which == "c5":
        r = bench.bench_conic(0, dev, None, steps=3, warmup=1)
    elif which == "c5solve":  # the KKT and Riccati solves only (no ADMM runs through the same kernels)
        r = bench.bench_conic(0, dev, None, steps=3, warmup=1, admm=False)
    elif which == "c4":
        r = bench.bench_horizon(0, dev, None, 1, 0, int(sys.argv[2]) if len(sys.argv) > 2 else 65536, steps=3,
                                warmup=1)
    elif which == "c4one":  # exactly one solve (PMC passes with PMC_SOLVES=1)
        r = bench.bench_horizon(0, dev, None, 1, 0, int(sys.argv[2]) if len(sys.argv) > 2 else 65536, steps=1,
                                warmup=0)
    elif which == "wide":
        r = bench.bench_batched_c3(0, dev, None, steps=3, warmup=1, N=256, batch=1024, n=24, m=16)
    else:
        raise SystemExit(f"unknown workload {which}")
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
