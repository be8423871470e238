"""The bench.py driver contract: the JSON line's keys and types (GPU, one small
run through the C ABI) and the CPU baseline's fields (host only, the oracle
restatement timed on a bounded sample)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cpu_baseline_fields():
    sys.path[:0] = [ROOT, os.path.join(ROOT, "pdp-lqr_amd")]
    import bench

    cb = bench.cpu_baseline(4, 2, 32, seconds=0.2, sample_batch=4, threads=2)
    assert cb["kind"] == "port" and cb["unit"] == "stages/s" and cb["cores"] == 2
    assert cb["value"] > 0 and "problems of N=32" in cb["sample"]
    one = cb["variants"]["C2_serial_1core"]
    assert one["cores"] == 1 and one["stages_per_s"] > 0 and one["ms_per_solve"] > 0


@pytest.mark.gpu
def test_bench_json_line():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--N", "128", "--batch", "256", "--steps", "2",
                          "--warmup", "1", "--no-cpu", "--no-secondary"], capture_output=True, text=True, timeout=300,
                         env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    d = json.loads(out.stdout.strip().splitlines()[-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["value"] > 0 and d["unit"] == "stages/s" and d["n_gpus"] == 1 and d["steps"] == 2
    assert d["higher_is_better"] is True and d["scaling"] == "weak" and d["dtype"] == "f64"
    assert d["config"]["workload"] and d["status_ok"] is True
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert 0 < r["frac"] < 1 and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-12
    assert d["cpu_baseline"] is None  # --no-cpu
    # value = stages per second over the timed steps
    assert abs(d["value"] - 128 * 256 / (d["ms_per_step"] * 1e-3)) / d["value"] < 1e-6
