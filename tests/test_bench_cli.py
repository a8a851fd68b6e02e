"""bench.py's multi-GPU entry: --gpus N without a launcher starts N ranks
itself, and refuses (non-zero exit, clear message) when the node has fewer than N GPUs --
never a 1-GPU number labelled as N GPUs."""
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


@pytest.mark.skipif(torch.cuda.device_count() >= 2, reason="node has >= 2 GPUs: the spawn would run the bench")
def test_bench_gpus2_refuses_without_two_gpus():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "--gpus 2 needs 2 visible GPUs" in r.stderr
    assert '"metric"' not in r.stdout


def test_bench_world_mismatch_is_an_error():
    """Launched by torchrun-like env with WORLD_SIZE=1 but --gpus 2: refuse."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "process group has 1 rank" in (r.stderr + r.stdout)
