"""The module/rs.h host-pointer classifier's rules (quicknet_amd/csrc/qfec_maps.hpp) on CPU:
which mappings hold memory the CPU copies may use without asking the HIP runtime (anonymous,
heap, stack, regular files, /dev/shm, /dev/zero, memfd) and which send a pointer to the runtime
probe (GPU driver files -- the render node, /dev/kfd, dma-bufs -- inaccessible ranges, addresses
no mapping covers).  tests/maps_host/shim.cpp is compiled here with g++; the GPU side is
tests/test_gpu_rs_host.py::test_rs_host_memory_kinds."""
import ctypes as C
import mmap
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "maps_host", "shim.cpp")
HDR = os.path.join(ROOT, "quicknet_amd", "csrc", "qfec_maps.hpp")
OUT = os.path.join(ROOT, "tests", "maps_host", "_build", "libmaps_shim.so")

MAPS = b"""55d0c0000000-55d0c0021000 r--p 00000000 08:01 1234                       /usr/bin/python3.10
55d0c1000000-55d0c2000000 rw-p 00000000 00:00 0                          [heap]
7f0000000000-7f0000200000 rw-s 1a000000 00:05 77                         /dev/dri/renderD176
7f0000200000-7f0000400000 rw-p 00000000 00:00 0 
7f0000400000-7f0001400000 ---p 00000000 00:00 0 
7f0001400000-7f0001500000 rw-s 00000000 00:19 5                          /dev/shm/qfec x (deleted)
7f0001500000-7f0001600000 rw-s 00000000 00:01 6                          /dev/zero (deleted)
7f0001600000-7f0001700000 rw-s 00000000 00:0e 7                          anon_inode:dmabuf
7f0001700000-7f0001800000 rw-s 00000000 00:01 8                          /memfd:pool (deleted)
7f0001800000-7f0001900000 rw-s 00000000 00:0d 9                          /dmabuf:
7f0001900000-7f0001a00000 rw-s 00000000 00:06 10                         /dev/kfd
7f0001a00000-7f0001b00000 r--s 00000000 00:06 11                         /dev/dri/card0
7ffd00000000-7ffd00021000 rw-p 00000000 00:00 0                          [stack]
"""


@pytest.fixture(scope="module")
def shim():
    if not os.path.exists(OUT) or os.path.getmtime(OUT) < max(os.path.getmtime(SRC), os.path.getmtime(HDR)):
        os.makedirs(os.path.dirname(OUT), exist_ok=True)
        subprocess.run(["g++", "-O1", "-std=c++17", "-fPIC", "-shared", "-o", OUT, SRC], check=True)
    L = C.CDLL(OUT)
    L.maps_is_host.argtypes = [C.c_char_p, C.c_ulonglong]
    L.maps_count.argtypes = [C.c_char_p]
    L.maps_self_is_host.argtypes = [C.c_ulonglong]
    return L


@pytest.mark.parametrize("addr,want", [
    (0x55d0c0000010, 1),   # a regular file's pages (read-only text)
    (0x55d0c1800000, 1),   # [heap]
    (0x7f0000000000, 0),   # the render node: device memory mapped for the CPU
    (0x7f00001fffff, 0),   # ... its last byte
    (0x7f0000200000, 1),   # anonymous rw-p (malloc'd or hipHostMalloc'd)
    (0x7f00003fffff, 1),
    (0x7f0000400000, 0),   # PROT_NONE reservation: possibly device memory the CPU cannot see
    (0x7f0001400100, 1),   # /dev/shm file (tmpfs), a path with a space
    (0x7f0001500100, 1),   # /dev/zero shared-anonymous
    (0x7f0001600100, 0),   # anon_inode:dmabuf
    (0x7f0001700100, 1),   # memfd
    (0x7f0001800100, 0),   # /dmabuf:
    (0x7f0001900100, 0),   # /dev/kfd
    (0x7f0001a00100, 0),   # another /dev file
    (0x7ffd00000100, 1),   # [stack]
    (0x1000, 0),           # below every mapping
    (0x7f0001b00000, 0),   # a gap between mappings
    (0x7ffd00021000, 0),   # one past the last mapping's end
])
def test_maps_rules(shim, addr, want):
    assert shim.maps_count(MAPS) == 13
    assert shim.maps_is_host(MAPS, addr) == want


def test_maps_malformed_lines_skipped(shim):
    text = b"garbage line\n\n" + MAPS + b"zzzz-yyyy rw-p\n"
    assert shim.maps_count(text) == 13
    assert shim.maps_is_host(text, 0x55d0c1800000) == 1


def test_maps_self(shim, tmp_path):
    """This process's own mappings: a numpy array (heap or anonymous), a file mapping and a
    /dev/shm mapping are system memory; an address in a PROT_NONE mapping is not."""
    a = np.zeros(1 << 20, np.uint8)
    assert shim.maps_self_is_host(a.ctypes.data) == 1
    p = tmp_path / "f.bin"
    p.write_bytes(b"\0" * 8192)
    with open(p, "r+b") as f:
        mm = mmap.mmap(f.fileno(), 8192)
        buf = (C.c_char * 8192).from_buffer(mm)
        assert shim.maps_self_is_host(C.addressof(buf)) == 1
        del buf
        mm.close()
    libc = C.CDLL(None)
    libc.mmap.restype = C.c_void_p
    libc.mmap.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_int, C.c_long]
    libc.munmap.argtypes = [C.c_void_p, C.c_size_t]
    addr = libc.mmap(None, 1 << 16, 0, 0x22, -1, 0)  # PROT_NONE, MAP_PRIVATE | MAP_ANONYMOUS
    try:
        assert shim.maps_self_is_host(addr) == 0
    finally:
        libc.munmap(addr, 1 << 16)
