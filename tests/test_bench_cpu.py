"""bench.py plumbing on CPU: `--gpus N` outside torchrun launches N rank
processes itself (gloo here, --dry-run touches no GPU), they meet in a barrier
and rank 0 reports n_gpus = N with the max over ranks."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT


@pytest.mark.parametrize("n", [1, 2, 3])
def test_bench_self_launches_n_ranks(n):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--dry-run"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout            # only rank 0 prints
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["max_rank"] == n - 1
    assert out["backend"] == ("gloo" if n > 1 else None)


def test_cpu_threads_and_model():
    sys.path.insert(0, ROOT)
    import bench
    assert 1 <= bench.cpu_threads() <= (os.cpu_count() or 1)
    assert isinstance(bench.cpu_model(), str)
