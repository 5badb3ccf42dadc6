"""GPU box: bench.py's multi-GPU launcher is safe to run before the driver's 8-GPU scaling run.

* The launching parent counts devices from sysfs (quicknet_amd.topology) without importing
  torch and without opening /dev/kfd or /dev/dri/*, and its count equals what HIP reports in a
  separate process.
* Asking for more ranks than the box has exits 2 before any rank starts.
* The RCCL code path (init_process_group("nccl", device_id=...), all-reduce on device tensors,
  barrier, destroy) runs on hardware through --force-dist at one rank; the line names the
  backend and this rank's NUMA placement.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(extra)
    return env


def _line(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


def _hip_count():
    r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                       capture_output=True, text=True, timeout=120, env=_env())
    assert r.returncode == 0, r.stderr
    return int(r.stdout.strip().splitlines()[-1])


def test_launcher_parent_touches_no_gpu():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--launch-check"], capture_output=True, text=True,
                       timeout=120, env=_env(QFEC_BENCH_BACKEND="nccl"), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    out = _line(r.stdout)
    print("launch-check:", out)
    assert out["torch_imported"] is False
    assert out["gpu_fds"] == []
    if out["gpu_count"] is not None:  # sysfs readable: it must agree with HIP
        assert out["gpu_count"] == _hip_count()
        assert out["plan"][0] is not None and out["plan"][0]["bdf"]


def test_launcher_refuses_more_ranks_than_gpus():
    n = _hip_count() + 1
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--launch-check"], capture_output=True, text=True,
                       timeout=120, env=_env(QFEC_BENCH_BACKEND="nccl"), cwd=ROOT)
    out_ok = r.returncode == 2 and "GPU(s) visible" in r.stderr
    if not out_ok:  # sysfs unreadable: the launcher cannot count, the ranks check themselves
        assert r.returncode == 0 and _line(r.stdout)["gpu_count"] is None, (r.returncode, r.stderr[-2000:])


def test_rccl_path_one_rank():
    """The RCCL branch of dist_setup and the device-tensor reductions, on hardware, at 1 rank."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--force-dist", "--steps", "5", "--warmup", "2",
                        "--no-cpu", "--no-side", "--no-host", "--config4-groups", "20000"],
                       capture_output=True, text=True, timeout=300,
                       env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                                MASTER_PORT=str(29500 + os.getpid() % 1000), QFEC_BENCH_BACKEND="nccl"), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _line(r.stdout)
    assert out["process_group"] == "nccl"
    assert out["verified"] is True and out["n_gpus"] == 1
    assert len(out["per_rank_numa"]) == 1
    print("numa:", out["numa_binding_rank0"], out["host_cpus"])
