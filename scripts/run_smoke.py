"""Run __graft_entry__.smoke() from the repo root (GPU-box helper for scripts/gpu_run.sh py: steps)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as g  # noqa: E402

g.smoke()
print("smoke ok")
