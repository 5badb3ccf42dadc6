"""GPU: libqfec's exact FEC layer (include/qfec_zfec.h) against the oracle's restatement of
network/NetFecCodec.cpp (oracle/zfec_ref.py), SEQUENCE for sequence.

Scripts (tests/zfec_script.py) drive sender/receiver pairs through seeded lossy channels:
drops, bursts, duplicates, adjacent swaps, shard corruption, late datagrams; set_zfec_kn at
group boundaries (with and without add_new, including redundancy collisions that leave a
NULL codec-list entry), enable_zfec toggles (FEC-off [0x13] datagrams in the middle of
groups), dynamic k/n from the lost rate, sorted/unsorted receive and switches between them.
For every pair the product must emit the oracle's datagrams in the oracle's order, byte for
byte, and deliver the oracle's (payload, source index) sequence; the receive counters must
agree.  Several pairs share one context, so one flush batches all of them.

The control flow restated by the oracle is PARITY UNPINNED (NetFecCodec.cpp does not build
here: it needs the absent system/option.h); every buffer and codec operation inside it is
the reference's own compiled FecCodecBuf.cpp / fec.c.
"""
import pytest

import quicknet_amd as qa
from zfec_script import PAIRS, make_script, replay, run_oracle

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)


@pytest.mark.parametrize("mode", ["flush_per_phase", "one_flush"])
@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_zfec_sequences_vs_oracle(seed, mode):
    scripts = [make_script(1000 * seed + i, phases=6, pair=p) for i, p in enumerate(PAIRS)]
    z = qa.Zfec()
    replay(z, scripts, [run_oracle(s) for s in scripts], mode)
    z.close()


def test_zfec_loopback_one_session():
    """One session both sends and receives (a NetFecCodecLayer is bidirectional): its own
    datagrams fed back, lossless -> every payload delivered once, in order, unsorted."""
    z = qa.Zfec()
    s = z.session()
    pay = [bytes([i]) * (i * 37 % 1500) for i in range(50)]
    for p in pay:
        z.pack_input(s, p)
    sent, _ = z.flush()
    for _, d in sent:
        z.unpack_input(s, d)
    _, got = z.flush()
    assert [g[1] for g in got] == pay
    assert [g[2] for g in got] == list(range(50))
    z.close()


def test_zfec_forged_check_packets():
    """As tests/test_zfec_host.py::test_host_forged_check_packets, on the device."""
    scripts = [make_script(7000 + i, phases=6, pair=p) for i, p in enumerate(PAIRS)]
    for sc in scripts:
        for ph in sc["phases"]:
            ph["chan"]["forge"] = 0.5
    z = qa.Zfec()
    replay(z, scripts, [run_oracle(s) for s in scripts], "one_flush")
    z.close()


def test_zfec_rate_tool_large_flush_verified():
    """A large flush (16 sessions x 3000 datagrams of ~1 KiB, ~50 MB of arena, the threaded
    session machines): the send flush, the per-datagram input calls and the receive flush; every
    payload arrives (count, bytes, word sum) and the sampled ones match byte for byte
    (tools/zfec_rate.py)."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, os.path.join(root, "tools", "zfec_rate.py"), "--sessions", "16",
                          "--packets", "3000", "--reps", "2", "--json"], capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-2000:]
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert res["verified"] and res["e2e"]["verified"], res
    assert res["e2e"]["byte_check"]["mismatched"] == 0 and res["e2e"]["byte_check"]["sampled"] > 0
