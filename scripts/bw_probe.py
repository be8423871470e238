"""Practical HBM ceilings on the box, for reading the roofline fractions:
read-only (sum of a large fp64 buffer), copy (read + write) and fill
(write-only) rates in GB/s, median of 5."""
import json
import sys

import torch


def rate(fn, nbytes, reps=5):
    fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        out.append(nbytes / (e0.elapsed_time(e1) * 1e-3) / 1e9)
    out.sort()
    return out[len(out) // 2]


n = (int(sys.argv[1]) if len(sys.argv) > 1 else 8) << 27  # GiB -> doubles
a = torch.ones(n, dtype=torch.float64, device="cuda")
b = torch.empty_like(a)
res = {"bytes": 8 * n,
       "read_sum_gbs": rate(lambda: a.sum(), 8 * n),
       "copy_gbs": rate(lambda: b.copy_(a), 16 * n),
       "fill_gbs": rate(lambda: b.fill_(2.0), 8 * n)}
print(json.dumps(res))
