"""bench.py's multi-GPU launch contract, on CPU: `--gpus N` without a distributed
environment starts N ranks itself, and refuses (non-zero exit, before any GPU work)
when fewer than N GPUs are visible."""
import os
import subprocess
import sys

from conftest import ROOT


def test_bench_refuses_more_gpus_than_visible():
    import torch
    if torch.cuda.device_count() >= 64:
        return
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "64", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "--gpus 64 but only" in r.stderr
