"""bench.py's rank launcher on CPU: `bench.py --gpus N` (no WORLD_SIZE) starts N rank processes
itself and the line reports n_gpus == N; a world/--gpus mismatch fails loudly.  The
--protocol-check mode runs the launch + barrier / max-time / summed-units protocol with no GPU
work (gloo), so this runs here."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(extra)
    return env


def _run(args, env=None, timeout=180):
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout,
                          env=env or _env(), cwd=ROOT)


def _line(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout  # ONE JSON line, from rank 0 only
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_spawns_n_ranks(n):
    r = _run(["--gpus", str(n), "--protocol-check"])
    assert r.returncode == 0, r.stderr[-2000:]
    out = _line(r.stdout)
    assert out["n_gpus"] == n and out["gpus_arg"] == n
    assert out["distinct_rank_pids"] == n          # N separate processes
    assert out["units"] == 1000 * n * (n + 1) / 2  # summed over ranks
    assert out["elapsed_max_s"] >= 0.01 * n        # the slowest rank's time


def test_single_rank_protocol():
    r = _run(["--protocol-check"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert _line(r.stdout)["n_gpus"] == 1


def test_world_mismatch_fails():
    r = _run(["--gpus", "2", "--protocol-check"], env=_env(WORLD_SIZE="1"))
    assert r.returncode != 0
    assert "WORLD_SIZE=1 but --gpus 2" in r.stderr


def test_launcher_refuses_missing_gpus():
    """With the RCCL backend, asking for more ranks than visible GPUs exits non-zero before
    starting anything (this container has no GPU)."""
    import torch
    if torch.cuda.device_count() >= 64:
        pytest.skip("enough GPUs")
    r = _run(["--gpus", "64"], env=_env(QFEC_BENCH_BACKEND="nccl"))
    assert r.returncode == 2
    assert "GPU(s) visible" in r.stderr
