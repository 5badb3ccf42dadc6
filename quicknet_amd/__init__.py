"""quicknet_amd -- MI355X-native Reed-Solomon FEC path for QuickNet-style packet-loss recovery.

The product is ``libqfec.so`` (quicknet_amd/csrc: HIP kernels for gfx950 + the C ABIs of
the reference's system/fec.h and module/rs.h + a batched device API, include/qfec*.h).
This package is the thin Python face used by the tests and bench.py.
"""
from ._lib import LIB_PATH, QfecError, lib  # noqa: F401
from .codec import (QFEC_CAUCHY, QFEC_VANDERMONDE, Code, FecParms, NetFec, Pipe, ReedSolomon, Zfec,  # noqa: F401
                    device_count, frame_udp, percall_counters, percall_stats, probe_reconstruct, probe_stream, rs_host_devices, set_kernel_variant, synth_fill, tune, tune_get, unframe_udp)

__version__ = "0.1.0"
