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


def test_world_size_mismatch_fails_before_gpu():
    """--gpus N under a launcher that started a different number of ranks is an
    error (exit 2), decided before any GPU call (runs on CPU)."""
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"], capture_output=True,
                         text=True, timeout=120, env=env, cwd=ROOT)
    assert out.returncode == 2 and "WORLD_SIZE=2" in out.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("gpus", [2])
def test_bench_spawns_ranks(gpus):
    """`bench.py --gpus N` without a launcher starts N ranks itself (gloo
    rehearsal on one GPU): the line says n_gpus = N, value counts every rank's
    batch, the C4 horizon is split over the N ranks and checked against the
    serial oracle across ranks, and the CPU baseline is on the line."""
    env = dict(os.environ, PDPLQR_BENCH_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--N", "128", "--batch",
                          "256", "--steps", "2", "--warmup", "1", "--cpu-seconds", "1", "--secondary", "C4",
                          "--c4-N", "2048"], capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [x for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == gpus and d["status_ok"] is True
    assert abs(d["value"] - gpus * 128 * 256 / (d["ms_per_step"] * 1e-3)) / d["value"] < 1e-6
    c4 = d["secondary"]["C4_horizon_sharded"]
    assert c4["n_gpus"] == gpus and c4["oracle_rel_err"] < 1e-9
    # the strong-scaling parts of the same run
    pt = c4["parts"]
    assert len(pt["rank_ms"]) == gpus and all(x > 0 for x in pt["rank_ms"])
    assert pt["max_rank_ms"] == max(pt["rank_ms"]) and pt["exchange_ms"] > 0
    assert pt["ref_1rank_ms"] > 0 and abs(pt["strong_scaling_ratio"] - pt["ref_1rank_ms"] / c4["ms_per_solve"]) < 1e-9
    assert d["rehearsal"]["backend"] == "gloo"
    assert d["cpu_baseline"] is not None and d["cpu_baseline"]["value"] > 0
