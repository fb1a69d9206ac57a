"""bench.py's rank launcher (`--gpus N` without torchrun, bench.py
launch_ranks): it refuses more ranks than visible GPUs unless
--allow-shared-gpu, and the rehearsal with ranks sharing one GPU reports every
rank in its line (ranks, oversubscribed, distinct n_gpus).  The multi-rank
protocol itself is tests/test_dist.py's (gloo, world 2)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")
SMALL = ["--sites", "200000", "--steps", "1", "--warmup", "0", "--device-steps", "1", "--no-extras"]


def run_bench(args, timeout):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)   # the launcher path: no torchrun around it
    return subprocess.run([sys.executable, BENCH] + args, cwd=ROOT, env=env, capture_output=True, timeout=timeout)


def visible_gpus():
    import torch
    return torch.cuda.device_count()   # (counting does not initialise a device on this image)


def test_launcher_needs_a_device():
    if visible_gpus() > 0:
        pytest.skip("a GPU is visible: the refusal without one is the CPU container's case")
    r = run_bench(["--gpus", "2"] + SMALL, 120)
    assert r.returncode != 0
    assert b"no HIP device visible" in r.stderr


@pytest.mark.gpu
def test_launcher_refuses_more_ranks_than_gpus():
    n = visible_gpus()
    r = run_bench(["--gpus", str(n + 1)] + SMALL, 120)
    assert r.returncode != 0
    assert b"--allow-shared-gpu" in r.stderr
    assert b'{"metric"' not in r.stdout


@pytest.mark.gpu
def test_shared_gpu_rehearsal_reports_every_rank():
    if visible_gpus() != 1:
        pytest.skip("the rehearsal case: one visible GPU")
    r = run_bench(["--gpus", "2", "--allow-shared-gpu"] + SMALL, 300)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    lines = [ln for ln in r.stdout.decode().splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1   # rank 0's line only
    d = json.loads(lines[0])
    assert d["config"]["ranks"] == 2
    assert d["config"]["oversubscribed"] is True
    assert d["n_gpus"] == 1
    assert d["config"]["sites_total"] == 2 * 200000
    assert d["value"] > 0
