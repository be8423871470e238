"""C4 (horizon-sharded 24/8) per-rank cost on one GPU for several slice
lengths: what each of R ranks would run for N = 65536 / R (plus a 14 KB
all-gather).  Prints one JSON line per N."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pdp-lqr_amd")]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    Ns = [int(x) for x in (sys.argv[1:] or ["65536", "32768", "16384", "8192"])]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    for N in Ns:
        r = bench.bench_horizon(0, dev, None, 1, 0, N, steps=3, warmup=1)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
