"""ctypes binding of libqfec.so (the HIP kernels + C ABI built from quicknet_amd/csrc).

The library is loaded from the package directory (built in-tree by
``__graft_entry__.build()`` / ``make -C quicknet_amd/csrc``).  There is no fallback: if
the library is missing, importing the codec raises.
"""
import ctypes as C
import os

# QFEC_LIB: another build of the same library, for before/after A/B runs (tools/ab_lib.sh)
LIB_PATH = os.environ.get("QFEC_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libqfec.so")

# every symbol the headers in include/ declare (checked by tests/test_abi.py)
EXPORTS = {
    "qfec_fec.h": ["fec_new", "fec_free", "fec_encode", "fec_decode"],
    "qfec_rs.h": ["reed_solomon_init", "reed_solomon_new", "reed_solomon_release", "reed_solomon_encode",
                  "reed_solomon_reconstruct", "reed_solomon_error"],
    "qfec.h": ["qfec_code_new", "qfec_code_from_rows", "qfec_code_free", "qfec_code_rows", "qfec_code_shape",
               "qfec_encode", "qfec_encode_host", "qfec_reconstruct", "qfec_reconstruct_host", "qfec_prepare_reconstruct", "qfec_decode_rows",
               "qfec_pipe_new", "qfec_pipe_free", "qfec_pipe_encode", "qfec_pipe_reconstruct", "qfec_pipe_wait", "qfec_pipe_slots",
               "qfec_fec_code", "qfec_rs_code", "qfec_fec_matrix", "qfec_pack_datagrams", "qfec_unpack_datagrams",
               "qfec_frame_udp", "qfec_unframe_udp", "qfec_pack_frames", "qfec_unpack_frames", "qfec_gather_rows", "qfec_synth_fill", "qfec_probe_stream", "qfec_probe_reconstruct", "qfec_rs_host_devices", "qfec_rs_host_devices_get",
               "qfec_tune", "qfec_tune_get", "qfec_percall_stats", "qfec_percall_counters", "qfec_set_kernel_variant", "qfec_get_kernel_variant", "qfec_device_count", "qfec_strerror",
               "qfec_last_error", "qfec_version"],
    "qfec_net.h": ["qfec_net_new", "qfec_net_free", "qfec_net_session", "qfec_net_enable", "qfec_net_pack_input", "qfec_net_flush_pack",
                   "qfec_net_unpack_input", "qfec_net_flush_unpack", "qfec_net_stats"],
    "qfec_zfec.h": ["qfec_zfec_new", "qfec_zfec_free", "qfec_zfec_session", "qfec_zfec_set_kn", "qfec_zfec_enable",
                    "qfec_zfec_sorted", "qfec_zfec_dynkn", "qfec_zfec_lost_rate", "qfec_zfec_pack_input",
                    "qfec_zfec_unpack_input", "qfec_zfec_flush", "qfec_zfec_stats"],
}

QFEC_CAUCHY = 0
QFEC_VANDERMONDE = 1
QFEC_VARIANT_PERM = 0
QFEC_VARIANT_LDSLOG = 1

_lib = None


class RSStruct(C.Structure):  # include/qfec_rs.h (== module/rs.h:7-13)
    _fields_ = [("data_shards", C.c_int), ("parity_shards", C.c_int), ("shards", C.c_int),
                ("m", C.POINTER(C.c_ubyte)), ("parity", C.POINTER(C.c_ubyte))]


def lib():
    """The loaded library (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                           "or `make -C quicknet_amd/csrc` (there is no CPU fallback)")
    # One HIP runtime per process: torch ships its own libamdhip64 (SONAME libamdhip64.so.7,
    # but libtorch_hip asks for "libamdhip64.so").  Loaded first, it also satisfies libqfec's
    # libamdhip64.so.7; loaded after /opt/rocm's, it comes in as a second runtime, and the
    # first one then sees no device ("no ROCm-capable device is detected").
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    vp, i, ll, u64 = C.c_void_p, C.c_int, C.c_longlong, C.c_ulonglong
    sig = {
        "qfec_code_new": (vp, [i, i, i]),
        "qfec_code_from_rows": (vp, [i, i, vp, i]),
        "qfec_code_free": (None, [vp]),
        "qfec_code_rows": (i, [vp, vp]),
        "qfec_code_shape": (i, [vp, C.POINTER(i), C.POINTER(i)]),
        "qfec_encode": (i, [vp, vp, vp, ll, i, ll, vp]),
        "qfec_encode_host": (i, [vp, vp, vp, ll, i, ll]),
        "qfec_reconstruct_host": (i, [vp, vp, vp, vp, ll, i, ll, vp]),
        "qfec_reconstruct": (i, [vp, vp, vp, vp, ll, i, ll, vp, vp]),
        "qfec_prepare_reconstruct": (i, [vp]),
        "qfec_pipe_new": (vp, [vp, i, i, ll]),
        "qfec_pipe_free": (None, [vp]),
        "qfec_pipe_encode": (i, [vp, vp, vp, vp, ll, i, ll]),
        "qfec_pipe_reconstruct": (i, [vp, vp, vp, vp, vp, ll, i, ll]),
        "qfec_pipe_wait": (i, [vp, C.POINTER(ll)]),
        "qfec_pipe_slots": (i, [vp]),
        "qfec_decode_rows": (i, [vp, vp, vp, vp, vp]),
        "qfec_fec_code": (vp, [vp]),
        "qfec_rs_code": (vp, [vp]),
        "qfec_fec_matrix": (i, [vp, vp]),
        "qfec_pack_datagrams": (i, [vp, vp, vp, vp, vp, ll, i, vp, ll, vp, ll, vp, vp]),
        "qfec_unpack_datagrams": (i, [vp, vp, ll, vp, ll, i, i, vp, ll, vp, vp, vp, vp, vp]),
        "qfec_frame_udp": (i, [vp, ll, vp, ll, vp, vp, i, i, i, vp, ll, vp, vp]),
        "qfec_pack_frames": (i, [vp, vp, vp, vp, vp, ll, i, vp, ll, vp, vp, i, i, i, vp, ll, vp, vp]),
        "qfec_unpack_frames": (i, [vp, vp, ll, vp, ll, i, i, i, i, vp, ll, vp, vp, vp, vp, vp, vp, vp]),
        "qfec_gather_rows": (i, [vp, vp, vp, ll, i, i, vp, ll, vp, vp]),
        "qfec_net_new": (vp, [i, i, i, i]),
        "qfec_net_free": (None, [vp]),
        "qfec_net_session": (i, [vp, vp]),
        "qfec_net_enable": (i, [vp, i, i]),
        "qfec_net_pack_input": (i, [vp, i, vp, C.c_uint]),
        "qfec_net_flush_pack": (i, [vp, vp, vp]),
        "qfec_net_unpack_input": (i, [vp, i, vp, C.c_uint]),
        "qfec_net_flush_unpack": (i, [vp, vp, i, vp]),
        "qfec_net_stats": (i, [vp, vp]),
        "qfec_unframe_udp": (i, [vp, ll, vp, ll, i, i, vp, ll, vp, vp, vp, vp, vp]),
        "qfec_synth_fill": (i, [vp, ll, u64, vp]),
        "qfec_probe_stream": (i, [vp, vp, ll, i, i, i, ll, vp]),
        "qfec_probe_reconstruct": (i, [vp, vp, vp, ll, i, i, i, ll, i, vp]),
        "qfec_rs_host_devices": (i, [vp, i]),
        "qfec_rs_host_devices_get": (i, [vp, i]),
        "qfec_tune": (i, [C.c_char_p, i]),
        "qfec_tune_get": (i, [C.c_char_p, C.POINTER(i)]),
        "qfec_percall_stats": (i, [vp]),
        "qfec_percall_counters": (i, [vp, i]),
        "qfec_set_kernel_variant": (i, [i]),
        "qfec_get_kernel_variant": (i, []),
        "qfec_device_count": (i, []),
        "qfec_strerror": (C.c_char_p, [i]),
        "qfec_last_error": (C.c_char_p, []),
        "qfec_version": (C.c_char_p, []),
        "fec_new": (vp, [i, i]),
        "fec_free": (None, [vp]),
        "fec_encode": (None, [vp, C.POINTER(vp), vp, i, i]),
        "fec_decode": (i, [vp, C.POINTER(vp), C.POINTER(i), i]),
        "reed_solomon_init": (None, []),
        "reed_solomon_new": (C.POINTER(RSStruct), [i, i]),
        "reed_solomon_release": (None, [C.POINTER(RSStruct)]),
        "reed_solomon_encode": (i, [C.POINTER(RSStruct), C.POINTER(vp), i, i]),
        "reed_solomon_reconstruct": (i, [C.POINTER(RSStruct), C.POINTER(vp), vp, i, i]),
        "reed_solomon_error": (i, []),
    }
    sig.update(ZFEC_SIG)
    compat = os.environ.get("QFEC_LIB_COMPAT") == "1"
    skipped = []
    for name, (res, args) in sig.items():
        if compat and not hasattr(L, name):
            skipped.append(name)  # an older build for a before/after A/B: entry points it predates
            continue
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    if skipped:
        import sys
        print(f"[qfec] QFEC_LIB_COMPAT: {LIB_PATH} lacks {', '.join(skipped)} (left unbound)", file=sys.stderr)
    _lib = L
    return L


_vp, _i = C.c_void_p, C.c_int
ZFEC_SIG = {  # include/qfec_zfec.h
    "qfec_zfec_new": (_vp, []),
    "qfec_zfec_free": (None, [_vp]),
    "qfec_zfec_session": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _i, _i]),
    "qfec_zfec_set_kn": (_i, [_vp, _i, _i, _i, _i]),
    "qfec_zfec_enable": (_i, [_vp, _i, _i]),
    "qfec_zfec_sorted": (_i, [_vp, _i, _i]),
    "qfec_zfec_dynkn": (_i, [_vp, _i, _i]),
    "qfec_zfec_lost_rate": (_i, [_vp, _i, C.c_float]),
    "qfec_zfec_pack_input": (_i, [_vp, _i, _vp, C.c_uint]),
    "qfec_zfec_unpack_input": (_i, [_vp, _i, _vp, C.c_uint]),
    "qfec_zfec_flush": (_i, [_vp, _vp, _vp, _vp]),
    "qfec_zfec_stats": (_i, [_vp, _i, _vp]),
}


def bind_zfec(L):
    """Declare include/qfec_zfec.h's signatures on another build of the layer (the CPU suite's
    host-only build, tests/zfec_host)."""
    for name, (res, args) in ZFEC_SIG.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    return L


class QfecError(RuntimeError):
    pass


def check(rc, what):
    if rc != 0:
        L = lib()
        raise QfecError(f"{what}: {L.qfec_strerror(rc).decode()} ({rc}): {L.qfec_last_error().decode()}")
    return rc
