"""The host thread pool (quicknet_amd/csrc/qfec_pool.cpp) on CPU: every part of a job runs
exactly once with the part count the caller asked for (capped by the pool's threads), jobs from
several caller threads are serialised, an exception in any part is rethrown after all parts are
done, and usable_cpus() honours the affinity mask (and a cgroup
CPU quota where one is set).  tests/pool_host/shim.cpp is compiled here with g++."""
import ctypes as C
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRCS = [os.path.join(ROOT, "tests", "pool_host", "shim.cpp"), os.path.join(ROOT, "quicknet_amd", "csrc", "qfec_pool.cpp")]
HDR = os.path.join(ROOT, "quicknet_amd", "csrc", "qfec_pool.hpp")
OUT = os.path.join(ROOT, "tests", "pool_host", "_build", "libpool_shim.so")


@pytest.fixture(scope="module")
def shim():
    if not os.path.exists(OUT) or os.path.getmtime(OUT) < max(os.path.getmtime(f) for f in SRCS + [HDR]):
        os.makedirs(os.path.dirname(OUT), exist_ok=True)
        subprocess.run(["g++", "-O1", "-std=c++17", "-fPIC", "-shared", "-o", OUT] + SRCS + ["-lpthread"], check=True)
    L = C.CDLL(OUT)
    L.pool_check.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_longlong)]
    return L


@pytest.mark.parametrize("threads,parts,jobs,callers", [(1, 5, 50, 1), (4, 1, 50, 1), (4, 3, 200, 1), (4, 64, 200, 1),
                                                         (8, 8, 100, 3), (16, 1 << 30, 50, 2), (3, 0, 20, 2)])
def test_pool_parts_run_once(shim, threads, parts, jobs, callers):
    calls = C.c_longlong()
    assert shim.pool_check(threads, parts, jobs, callers, C.byref(calls)) == 0
    per = min(threads, max(1, parts))
    assert calls.value == per * jobs * callers


@pytest.mark.parametrize("threads,thrower", [(4, 0), (4, 2), (8, 7), (1, 0)])
def test_pool_exception_waits_for_all_parts(shim, threads, thrower):
    """A part that throws (the caller's part or a worker's): run() rethrows once every other part
    has returned, and the pool runs the next job normally."""
    assert shim.pool_throw_check(threads, thrower, 20) == 0


def test_usable_cpus(shim):
    n = shim.pool_usable_cpus()
    assert 1 <= n <= len(os.sched_getaffinity(0))
