"""bench.py's rank launcher on CPU: `bench.py --gpus N` (no WORLD_SIZE) starts N rank processes
itself and the line reports n_gpus == N; a world/--gpus mismatch fails loudly.  The
--protocol-check mode runs the launch + barrier / max-time / summed-units protocol with no GPU
work (gloo), so this runs here."""
import json
import os
import subprocess
import sys
import time

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


def _fake_sysfs(root, gpus):
    """A KFD topology + PCI tree: node 0 is a CPU, then one node per (bdf, numa_node, cpulist)."""
    nodes = os.path.join(root, "sys/class/kfd/kfd/topology/nodes")
    os.makedirs(os.path.join(nodes, "0"))
    with open(os.path.join(nodes, "0", "properties"), "w") as f:
        f.write("cpu_cores_count 64\ngfx_target_version 0\n")
    for i, (bdf, numa, cpus) in enumerate(gpus, 1):
        dom, bus, devfn = bdf.split(":")[0], bdf.split(":")[1], bdf.split(":")[2]
        dev, fn = devfn.split(".")
        loc = int(bus, 16) << 8 | int(dev, 16) << 3 | int(fn)
        os.makedirs(os.path.join(nodes, str(i)))
        with open(os.path.join(nodes, str(i), "properties"), "w") as f:
            f.write(f"gfx_target_version 90500\nlocation_id {loc}\ndomain {int(dom, 16)}\nunique_id {0xABC0 + i}\n")
        pci = os.path.join(root, "sys/bus/pci/devices", bdf)
        os.makedirs(pci)
        with open(os.path.join(pci, "numa_node"), "w") as f:
            f.write(f"{numa}\n")
        with open(os.path.join(pci, "local_cpulist"), "w") as f:
            f.write(cpus + "\n")
    return root


GPUS = [("0000:05:00.0", 0, "0-3"), ("0000:65:00.0", 0, "0-3"), ("0000:85:00.0", 1, "4-7")]


def test_topology_counts_and_places(tmp_path):
    from quicknet_amd import topology as T
    root = _fake_sysfs(str(tmp_path), GPUS)
    assert T.gpu_count({}, root)[0] == 3
    assert [d["bdf"] for d in T.visible_gpus({}, root)] == [g[0] for g in GPUS]
    assert T.gpu_count({"HIP_VISIBLE_DEVICES": "2,0"}, root)[0] == 2
    assert T.gpu_numa(0, {"HIP_VISIBLE_DEVICES": "2,0"}, root)["numa_node"] == 1
    assert T.gpu_count({"ROCR_VISIBLE_DEVICES": "1,2", "HIP_VISIBLE_DEVICES": "1"}, root)[0] == 1
    assert T.gpu_numa(0, {"ROCR_VISIBLE_DEVICES": "1,2", "HIP_VISIBLE_DEVICES": "1"}, root)["bdf"] == "0000:85:00.0"
    assert T.gpu_count({"CUDA_VISIBLE_DEVICES": "0,9,1"}, root)[0] == 1   # the list ends at a bad entry
    assert T.gpu_count({"HIP_VISIBLE_DEVICES": ""}, root)[0] == 3     # empty = HIP's default, no filter
    assert T.gpu_count({"ROCR_VISIBLE_DEVICES": ""}, root)[0] == 0
    assert T.gpu_count({"ROCR_VISIBLE_DEVICES": "GPU-%016x" % (0xABC0 + 3)}, root)[0] == 1
    p = T.gpu_numa(2, {}, root)
    assert p["cpus"] == {4, 5, 6, 7} and p["numa_node"] == 1 and p["kfd_node"] == 3
    assert T.gpu_numa(3, {}, root) is None
    assert T.parse_cpulist("0-2,5,7-8") == {0, 1, 2, 5, 7, 8}
    assert T.gpu_count({}, str(tmp_path / "none"))[0] is None
    # a node the sandbox will not let us read (another job's GPU): the count is only a lower
    # bound, so the launcher does not refuse on it; placement still follows the readable nodes
    os.makedirs(os.path.join(root, "sys/class/kfd/kfd/topology/nodes", "9"))
    n, why = T.gpu_count({}, root)
    assert n is None and "unreadable" in why
    assert T.gpu_numa(2, {}, root)["bdf"] == "0000:85:00.0"


def test_bind_rank_dry_run(tmp_path):
    from quicknet_amd import topology as T
    root = _fake_sysfs(str(tmp_path), GPUS)
    mine = os.sched_getaffinity(0)
    rec = T.bind_rank(2, {}, root, apply=False)
    assert rec["numa_node"] == 1 and rec["bdf"] == "0000:85:00.0"
    if {4, 5, 6, 7} & mine:
        assert rec["bound"] and rec["cpus"] == len({4, 5, 6, 7} & mine)
    assert os.sched_getaffinity(0) == mine  # dry run changed nothing
    assert T.bind_rank(0, {}, str(tmp_path / "none"), apply=False)["bound"] is False


def test_launch_check_parent_is_gpu_free(tmp_path):
    """The launcher's pre-spawn state: torch never imported, no /dev/kfd or /dev/dri fd open,
    devices counted from sysfs, a NUMA plan per rank."""
    root = _fake_sysfs(str(tmp_path), GPUS)
    r = _run(["--gpus", "3", "--launch-check"], env=_env(QFEC_BENCH_BACKEND="nccl", QFEC_SYSFS_ROOT=root))
    assert r.returncode == 0, r.stderr[-2000:]
    out = _line(r.stdout)
    assert out["torch_imported"] is False and out["gpu_fds"] == []
    assert out["gpu_count"] == 3
    assert [p["numa_node"] for p in out["plan"]] == [0, 0, 1]


def test_launcher_refuses_missing_gpus(tmp_path):
    """Counted from sysfs: more ranks than visible GPUs exits 2 before starting anything."""
    root = _fake_sysfs(str(tmp_path), GPUS)
    t0 = time.time()
    r = _run(["--gpus", "4"], env=_env(QFEC_BENCH_BACKEND="nccl", QFEC_SYSFS_ROOT=root))
    assert r.returncode == 2
    assert "only 3 GPU(s) visible" in r.stderr
    assert time.time() - t0 < 30


def test_ranks_check_their_own_device_when_sysfs_is_silent(tmp_path):
    """No readable topology: the launcher starts the ranks and each checks its own index
    (this container has no GPU), so the job exits 2 instead of running on nothing."""
    r = _run(["--gpus", "2", "--no-cpu"], env=_env(QFEC_BENCH_BACKEND="nccl", QFEC_SYSFS_ROOT=str(tmp_path)))
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "GPU(s) are visible" in r.stderr


def test_rank_failure_ends_the_job():
    """Rank 1 fails before the rendezvous; rank 0 would wait in it forever.  The launcher ends
    it after the grace period and exits with rank 1's code."""
    t0 = time.time()
    r = _run(["--gpus", "2", "--protocol-check", "--fail-rank", "1", "--fail-grace-s", "2"])
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert time.time() - t0 < 60
    assert "rank 1 exited 3" in r.stderr


def test_launch_deadline_kills_hung_rank():
    t0 = time.time()
    r = _run(["--gpus", "2", "--protocol-check", "--hang-rank", "1", "--deadline-s", "6"])
    assert r.returncode == 124, (r.returncode, r.stderr[-2000:])
    assert time.time() - t0 < 60
    assert "deadline" in r.stderr
