"""CPU: the exact FEC layer's host state machines (quicknet_amd/csrc/qfec_zfec.cpp) against the
oracle's NetFecCodec restatement, sequence for sequence, without a GPU.

qfec_zfec.cpp is compiled here with g++ together with tests/zfec_host/stubs.cpp, which stands
in for its two device entry points (qfec_pack_datagrams / qfec_unpack_datagrams) with the
oracle's C restatement of the same wire rules -- test infrastructure, never the product.  The
same scripts run through the real libqfec.so on the MI355X in tests/test_gpu_zfec.py.
Parity of the control flow itself is UNPINNED (see oracle/zfec_ref.py).
"""
import ctypes as C
import os
import subprocess

import pytest

from oracle import zfec_ref
from zfec_script import PAIRS, make_script, replay, run_oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tests", "zfec_host", "_build", "libzfec_host.so")
CSRC = os.path.join(ROOT, "quicknet_amd", "csrc")
SRCS = [os.path.join(CSRC, "qfec_zfec.cpp"), os.path.join(CSRC, "qfec_zfec_flush.cpp"),
        os.path.join(ROOT, "tests", "zfec_host", "stubs.cpp"), os.path.join(CSRC, "qfec_pool.cpp")]
DEPS = SRCS + [os.path.join(CSRC, "qfec_zfec_impl.hpp"), os.path.join(CSRC, "qfec_pool.hpp"),
               os.path.join(ROOT, "include", "qfec_zfec.h"), os.path.join(ROOT, "include", "qfec.h")]
ORACLE_LIB = os.path.join(ROOT, "oracle", "liboracle.so")

pytestmark = pytest.mark.skipif(not (zfec_ref.available() and os.path.exists(ORACLE_LIB)),
                                reason="oracle libraries not built (make -C oracle all ref)")


@pytest.fixture(scope="module")
def host_layer():
    if not os.path.exists(OUT) or os.path.getmtime(OUT) < max(os.path.getmtime(s) for s in DEPS):
        os.makedirs(os.path.dirname(OUT), exist_ok=True)
        subprocess.run(["g++", "-O1", "-std=c++17", "-fPIC", "-shared", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                        "-o", OUT] + SRCS + ["-lpthread", "-L" + os.path.dirname(ORACLE_LIB), "-loracle",
                        "-Wl,-rpath," + os.path.dirname(ORACLE_LIB)], check=True)
    from quicknet_amd._lib import bind_zfec
    return bind_zfec(C.CDLL(OUT))


@pytest.mark.parametrize("mode", ["flush_per_phase", "one_flush"])
@pytest.mark.parametrize("seed", range(8))
def test_host_sequences_vs_oracle(host_layer, seed, mode):
    import quicknet_amd as qa
    scripts = [make_script(1000 * seed + i, phases=6, pair=p) for i, p in enumerate(PAIRS)]
    z = qa.Zfec(_lib=host_layer)
    replay(z, scripts, [run_oracle(s) for s in scripts], mode)
    z.close()


@pytest.mark.parametrize("seed", range(4))
def test_host_threaded_machines_vs_oracle(host_layer, seed, monkeypatch):
    """The receive machines of a flush's sessions on 3 threads (QFEC_ZFEC_RX_THREADS; large
    flushes use threads by themselves): the same sequences as the oracle's."""
    import quicknet_amd as qa
    monkeypatch.setenv("QFEC_ZFEC_RX_THREADS", "3")
    scripts = [make_script(5000 + 1000 * seed + i, phases=6, pair=p) for i, p in enumerate(PAIRS)]
    z = qa.Zfec(_lib=host_layer)
    replay(z, scripts, [run_oracle(s) for s in scripts], "one_flush")
    z.close()


def test_host_many_small_flushes(host_layer):
    """A flush after every queued call: open groups and the receive window carried across
    hundreds of flushes."""
    import quicknet_amd as qa
    sc = make_script(77, phases=4, pair=dict(is_sorted=True))
    res, st = run_oracle(sc)
    z = qa.Zfec(_lib=host_layer)
    A, B = z.session(is_sorted=True), z.session(is_sorted=True)
    sent_all, got_all = [], []
    for p, r in enumerate(res):
        for op in r["tx_ops"]:
            if op[0] == "pack":
                z.pack_input(A, op[1])
            elif op[0] == "set_kn":
                z.set_kn(A, op[1], op[2], op[3])
                z.set_kn(B, op[1], op[2], op[3])
            else:
                getattr(z, op[0])(A, op[1])
            sent, got = z.flush()
            sent_all += [d for s, d in sent if s == A]
        for op in sc["phases"][p]["rx_cfg"]:
            z.sorted(B, op[1])
        for d in r["rx"]:
            z.unpack_input(B, d)
            _, got = z.flush()
            got_all += [(x[1], x[2]) for x in got if x[0] == B]
    assert sent_all == [d for r in res for d in r["datagrams"]]
    assert got_all == [d for r in res for d in r["deliv"]]
    s = z.stats(B)
    assert (s["fec_src_count"], s["fec_restore_count"], s["i_expected_packet"]) == \
        (st["fec_src_count"], st["fec_restore_count"], st["i_expected_packet"])
    z.close()


@pytest.mark.parametrize("seed", range(4))
def test_host_forged_check_packets(host_layer, seed):
    """Half the check datagrams forged (shard bytes changed, datagram checksum recomputed):
    decodes then produce arbitrary size fields, some beyond the decode's first pitch, which the
    layer decodes again at dec_pkt_size + 4 as the reference reads them."""
    import quicknet_amd as qa
    scripts = [make_script(5000 + 1000 * seed + i, phases=6, pair=p) for i, p in enumerate(PAIRS)]
    for sc in scripts:
        for ph in sc["phases"]:
            ph["chan"]["forge"] = 0.5
    z = qa.Zfec(_lib=host_layer)
    replay(z, scripts, [run_oracle(s) for s in scripts], "one_flush")
    z.close()


def test_host_arena_register_failure(host_layer):
    """The arenas' 2 MiB-page blocks are registered with the runtime; when registration fails (no
    device), later growths skip the mapping: one registration attempt over many arena growths, and
    the layer's datagrams and deliveries unchanged (hipHostMalloc / malloc arenas)."""
    import quicknet_amd as qa
    raw = C.CDLL(OUT)
    fail = C.c_int.in_dll(raw, "stub_register_fail")
    calls = C.c_int.in_dll(raw, "stub_register_calls")
    fail.value = 1
    before = calls.value
    try:
        z = qa.Zfec(_lib=host_layer)
        A, B = z.session(k=10, n=13), z.session(k=10, n=13)
        payloads = [bytes([(i * 7 + j) & 0xFF for j in range(64)]) * 16 for i in range(256)]
        for rep in range(24):  # ~6 MiB queued per direction: the arenas grow several times
            for p in payloads:
                z.pack_input(A, p)
        sent, _ = z.flush()
        for s, d in sent:
            assert s == A
            z.unpack_input(B, d)
        _, got = z.flush()
        assert [g[1] for g in got if g[0] == B] == payloads * 24
        z.close()
    finally:
        fail.value = 0
    assert calls.value - before == 1
