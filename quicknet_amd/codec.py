"""Python face of libqfec: the batched device codec and the reference's per-call ABIs.

* ``Code``          -- a (k, m) code on the MI355X; ``encode`` / ``reconstruct`` run whole
                       batches of groups on device tensors (torch, uint8) on the current
                       HIP stream.  Mirrors module/rs.c's batched API (rs.h:22-49) over the
                       contiguous layout of include/qfec.h.
* ``FecParms``      -- system/fec.h's per-packet codec (fec_new / fec_encode / fec_decode),
                       the interface network/FecCodec.cpp and network/FecCodecBuf.cpp bind.
* ``ReedSolomon``   -- module/rs.h's per-call codec over shard pointer arrays.

All arithmetic runs in the HIP kernels of libqfec.so; these classes only marshal.
"""
import ctypes as C

import numpy as np

from ._lib import QFEC_CAUCHY, QFEC_VANDERMONDE, RSStruct, QfecError, check, lib

__all__ = ["Code", "FecParms", "ReedSolomon", "QfecError", "QFEC_CAUCHY", "QFEC_VANDERMONDE",
           "set_kernel_variant", "tune", "synth_fill", "probe_stream", "probe_reconstruct", "rs_host_devices", "device_count", "frame_udp", "unframe_udp",
           "NetFec", "Pipe", "Zfec"]


def _stream_handle(stream):
    if stream is None:
        import torch
        if not torch.cuda.is_available():  # host-only calls (e.g. qfec_net's FEC-off traffic)
            return None
        return C.c_void_p(torch.cuda.current_stream().cuda_stream)
    if isinstance(stream, int):
        return C.c_void_p(stream)
    return C.c_void_p(stream.cuda_stream)


_U8, _I32, _I64 = "u8", "i32", "i64"


def _dev_ptr(t, kind=_U8, what="tensor"):
    """Device pointer of a contiguous tensor on the CURRENT device (the C side launches on the
    calling thread's current device and stream), with the element type the ABI reads:
    u8 = torch.uint8 bytes, i32 = 4-byte integers (int32 / uint32), i64 = int64."""
    if t is None:
        return None
    if not getattr(t, "is_cuda", False):
        raise QfecError(f"{what}: expected a device tensor")
    if not t.is_contiguous():
        raise QfecError(f"{what}: expected a contiguous tensor")
    import torch
    ok = {_U8: t.dtype == torch.uint8,
          _I32: t.dtype in (torch.int32, getattr(torch, "uint32", torch.int32)),
          _I64: t.dtype == torch.int64}[kind]
    if not ok:
        raise QfecError(f"{what}: dtype {t.dtype} where the ABI reads {kind}")
    if t.device.index != torch.cuda.current_device():
        raise QfecError(f"{what}: on {t.device} but the current device is cuda:{torch.cuda.current_device()} "
                        "(use `with torch.cuda.device(...)`)")
    return C.c_void_p(t.data_ptr())


def device_count():
    return lib().qfec_device_count()


def set_kernel_variant(v):
    check(lib().qfec_set_kernel_variant(v), "qfec_set_kernel_variant")


def tune(key, value):
    """Experiment knob (see include/qfec.h qfec_tune); outputs are identical either way."""
    check(lib().qfec_tune(key.encode(), int(value)), f"qfec_tune({key})")


def tune_get(key):
    """The current value of a qfec_tune knob."""
    v = C.c_int(0)
    check(lib().qfec_tune_get(key.encode(), C.byref(v)), f"qfec_tune_get({key})")
    return v.value


def percall_stats():
    """The current device's resident per-call server (include/qfec.h qfec_percall_stats)."""
    out = (C.c_ulonglong * 5)()
    check(lib().qfec_percall_stats(out), "qfec_percall_stats")
    usable = out[4] if out[4] < 2**63 else out[4] - 2**64
    return {"calls": out[0], "launches": out[1], "relaunches": out[2], "running": bool(out[3]), "usable": usable}


def percall_counters():
    """qfec_percall_counters: percall_stats plus timeouts, fec_encode group-cache hits / misses, the
    current percall_idle_us and the servers abandoned after percall_stop_us."""
    out = (C.c_ulonglong * 10)()
    n = lib().qfec_percall_counters(out, 10)
    check(n if n < 0 else 0, "qfec_percall_counters")
    usable = out[4] if out[4] < 2**63 else out[4] - 2**64
    return {"calls": out[0], "launches": out[1], "relaunches": out[2], "running": bool(out[3]), "usable": usable,
            "timeouts": out[5], "group_hits": out[6], "group_misses": out[7], "idle_us": out[8],
            "abandoned": out[9]}


def synth_fill(t, seed, stream=None):
    """Fill a device uint8 tensor with quicknet_amd.synth.synth_bytes(seed, t.numel())."""
    check(lib().qfec_synth_fill(_dev_ptr(t, what="synth_fill"), t.numel(), seed & 0xFFFFFFFFFFFFFFFF, _stream_handle(stream)),
          "qfec_synth_fill")


def rs_host_devices(devices=None):
    """qfec_rs_host_devices: spread module/rs.h's host-pointer pipelines over two slots per listed
    device (repeats allowed); None or [] -> the calling thread's current device.  Returns the list
    now in force."""
    devs = list(devices or [])
    arr = (C.c_int * max(1, len(devs)))(*devs)
    check(lib().qfec_rs_host_devices(arr if devs else None, len(devs)), "qfec_rs_host_devices")
    out = (C.c_int * 64)()
    n = lib().qfec_rs_host_devices_get(out, 64)
    check(min(n, 0), "qfec_rs_host_devices_get")
    return list(out[:n])


def probe_reconstruct(data, parity, marks, block_size, lds_cap=0, stream=None):
    """Calibration only: the reconstruct's memory skeleton (RS(10,3), RS(16,4)); the erased rows
    of `data` receive garbage.  lds_cap: LDS bytes per block (0 none), a residency cap."""
    G, k, pitch = data.shape
    m = parity.shape[1]
    check(lib().qfec_probe_reconstruct(_dev_ptr(data, what="data"), _dev_ptr(parity, what="parity"),
                                       _dev_ptr(marks, what="marks"), G, k, m, block_size, pitch, lds_cap,
                                       _stream_handle(stream)), "qfec_probe_reconstruct")


def probe_stream(data, parity, block_size, stream=None):
    """Calibration only: the encode's traffic with XOR in place of GF arithmetic."""
    G, k, pitch = data.shape
    m = parity.shape[1]
    check(lib().qfec_probe_stream(_dev_ptr(data, what="data"), _dev_ptr(parity, what="parity"), G, k, m, block_size, pitch,
                                  _stream_handle(stream)), "qfec_probe_stream")


def frame_udp(rows, lengths, masks, gmask=0, cmd=0x11, protocol=0xFF, conv_hid=None, out_pitch=None, stream=None):
    """ProtocolUdp framing of a datagram batch (include/qfec.h qfec_frame_udp): rows uint8
    [R, pitch] device tensor, lengths int32 [R], masks uint8 [R] (per-packet Session _mask),
    conv_hid uint32/int32 [R, 2] or None.  Defaults: QUICKNET_CMD_DATA, QUICKNET_PROTOCOL_FEC
    (network/ProtocolBasic.h:82,95), as Session::TransmissionOutput sets them for FEC datagrams
    (network/SessionDesc.cpp:513-519).  Returns (framed [R, out_pitch], framed_len [R])."""
    import torch
    R, pitch = rows.shape
    P = 12 if conv_hid is not None else 4
    if out_pitch is None:
        out_pitch = (pitch + P + 15) // 16 * 16
    out = torch.empty((R, out_pitch), dtype=torch.uint8, device=rows.device)
    out_len = torch.empty(R, dtype=torch.int32, device=rows.device)
    check(lib().qfec_frame_udp(_dev_ptr(rows, what="rows"), pitch, _dev_ptr(lengths, _I32, "lengths"), R,
                               _dev_ptr(masks, what="masks"),
                               _dev_ptr(conv_hid, _I32, "conv_hid") if conv_hid is not None else None, int(gmask), int(cmd),
                               int(protocol), _dev_ptr(out), out_pitch, _dev_ptr(out_len, _I32), _stream_handle(stream)),
          "qfec_frame_udp")
    return out, out_len


def unframe_udp(frames, lengths, gmask=0, session=False, out_pitch=None, stream=None):
    """Reverse of frame_udp (qfec_unframe_udp).  Returns (data [R, out_pitch], data_len [R],
    status [R], info uint8 [R, 4], conv_hid int32 [R, 2] or None)."""
    import torch
    R, pitch = frames.shape
    if out_pitch is None:
        out_pitch = pitch
    dev = frames.device
    out = torch.empty((R, out_pitch), dtype=torch.uint8, device=dev)
    out_len = torch.empty(R, dtype=torch.int32, device=dev)
    status = torch.empty(R, dtype=torch.int32, device=dev)
    info = torch.empty((R, 4), dtype=torch.uint8, device=dev)
    ch = torch.zeros((R, 2), dtype=torch.int32, device=dev) if session else None
    check(lib().qfec_unframe_udp(_dev_ptr(frames, what="frames"), pitch, _dev_ptr(lengths, _I32, "lengths"), R, int(gmask),
                                 int(bool(session)), _dev_ptr(out), out_pitch, _dev_ptr(out_len, _I32),
                                 _dev_ptr(status, _I32), _dev_ptr(info),
                                 _dev_ptr(ch, _I32) if ch is not None else None, _stream_handle(stream)), "qfec_unframe_udp")
    return out, out_len, status, info, ch


class Code:
    """A GF(2^8) RS code with k data and m parity shards per group."""

    def __init__(self, handle, owner=True):
        if not handle:
            raise QfecError(f"invalid code: {lib().qfec_last_error().decode()}")
        self._h = C.c_void_p(handle)
        self._owner = owner
        k, m = C.c_int(), C.c_int()
        check(lib().qfec_code_shape(self._h, C.byref(k), C.byref(m)), "qfec_code_shape")
        self.k, self.m = k.value, m.value

    @classmethod
    def cauchy(cls, k, m):
        """module/rs.c's matrix (reed_solomon_new, rs.c:437-440)."""
        return cls(lib().qfec_code_new(QFEC_CAUCHY, k, m))

    @classmethod
    def vandermonde(cls, k, m):
        """module/fec.c's matrix (fec_new(k, k + m), fec.c:653-707)."""
        return cls(lib().qfec_code_new(QFEC_VANDERMONDE, k, m))

    @classmethod
    def from_rows(cls, rows, rs_stale_quirk=False):
        rows = np.ascontiguousarray(rows, dtype=np.uint8)
        m, k = rows.shape
        return cls(lib().qfec_code_from_rows(k, m, rows.ctypes.data, int(rs_stale_quirk)))

    def close(self):
        if self._h and self._owner:
            lib().qfec_code_free(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def rows(self):
        out = np.zeros((self.m, self.k), dtype=np.uint8)
        check(lib().qfec_code_rows(self._h, out.ctypes.data), "qfec_code_rows")
        return out

    def encode_host(self, data, parity, block_size=None):
        """qfec_encode_host: data uint8 [G, k, pitch] and parity [G, m, pitch] in HOST memory
        (numpy arrays, or CPU tensors, pinned or not); returns when parity is written."""
        G, k, pitch = data.shape
        if k != self.k or parity.shape[0] != G or parity.shape[1] != self.m or parity.shape[2] != pitch:
            raise QfecError(f"shape mismatch: data {tuple(data.shape)} parity {tuple(parity.shape)} for ({self.k},{self.m})")
        block_size = pitch if block_size is None else block_size
        ptr = (lambda a: a.ctypes.data) if isinstance(data, np.ndarray) else (lambda t: t.data_ptr())
        for a in (data, parity):
            if not (a.flags["C_CONTIGUOUS"] if isinstance(a, np.ndarray) else a.is_contiguous()):
                raise QfecError("encode_host: contiguous host buffers required")
        check(lib().qfec_encode_host(self._h, ptr(data), ptr(parity), G, block_size, pitch), "qfec_encode_host")

    def reconstruct_host(self, data, parity, marks, block_size=None):
        """qfec_reconstruct_host: data uint8 [G, k, pitch] rewritten in place from parity
        [G, m, pitch] and rs.c-layout marks [G*(k+m)], all in HOST memory (numpy arrays, or
        CPU tensors, pinned or not).  Returns the number of under-determined groups."""
        G, k, pitch = data.shape
        nmarks = marks.size if isinstance(marks, np.ndarray) else marks.numel()
        if k != self.k or tuple(parity.shape) != (G, self.m, pitch) or nmarks != G * (self.k + self.m):
            raise QfecError("reconstruct_host: shape mismatch")
        block_size = pitch if block_size is None else block_size
        nf = C.c_longlong(0)
        check(lib().qfec_reconstruct_host(self._h, _host_ptr(data, "data"), _host_ptr(parity, "parity"),
                                          _host_ptr(marks, "marks"), G, block_size, pitch, C.byref(nf)),
              "qfec_reconstruct_host")
        return int(nf.value)

    def encode(self, data, parity, block_size=None, stream=None):
        """parity[g] = P x data[g]; data uint8 [G, k, pitch], parity uint8 [G, m, pitch] on device."""
        G, k, pitch = data.shape
        if k != self.k or parity.shape[0] != G or parity.shape[1] != self.m or parity.shape[2] != pitch:
            raise QfecError(f"shape mismatch: data {tuple(data.shape)} parity {tuple(parity.shape)} for ({self.k},{self.m})")
        block_size = pitch if block_size is None else block_size
        check(lib().qfec_encode(self._h, _dev_ptr(data, what="data"), _dev_ptr(parity, what="parity"), G, block_size, pitch,
                                _stream_handle(stream)), "qfec_encode")

    def prepare_reconstruct(self):
        check(lib().qfec_prepare_reconstruct(self._h), "qfec_prepare_reconstruct")

    def reconstruct(self, data, parity, marks, block_size=None, failed=None, stream=None):
        """Rewrite erased data shards in place.  marks: uint8 [G*k + G*m] (rs.c layout) on device;
        failed: optional device int32/uint32 [1] counter of under-determined groups."""
        G, k, pitch = data.shape
        if k != self.k or parity.shape[0] != G or parity.shape[1] != self.m or marks.numel() != G * (self.k + self.m):
            raise QfecError("shape mismatch")
        block_size = pitch if block_size is None else block_size
        check(lib().qfec_reconstruct(self._h, _dev_ptr(data, what="data"), _dev_ptr(parity, what="parity"),
                                     _dev_ptr(marks, what="marks"), G, block_size, pitch,
                                     _dev_ptr(failed, _I32, "failed"), _stream_handle(stream)), "qfec_reconstruct")

    # -- FEC datagram batches (network/FecCodecBuf.cpp wire format); n = k + m <= 15
    def pack_datagrams(self, payload, offsets, sizes, seq, checksum=True, shard_pitch=None, wire_pitch=None,
                       stream=None):
        """payload: uint8 device tensor (16 readable bytes past the last packet); offsets int64
        [G*k]; sizes int32 [G*k]; seq uint32/int32 [G, 2] (sent, src index of each group's first
        packet).  Returns (shards [G, n, pitch], wire [G, n, wire_pitch], wire_len int32 [G, n]).
        wire_pitch defaults to the 64-B multiple above 13 + shard_pitch (1088 for 1 KiB payloads;
        round 1 used the 16-B multiple, 1056): the fused send then writes whole 64-B lines.  Pass
        wire_pitch explicitly where a consumer needs another row layout."""
        import torch
        G = sizes.numel() // self.k
        n = self.k + self.m
        head = 4 if checksum else 2
        if shard_pitch is None:
            shard_pitch = (int(sizes.max().item()) + head + 15) // 16 * 16 if G else 16
        if wire_pitch is None:  # the 64-B multiple: the fused send then writes whole lines
            wire_pitch = (shard_pitch + 13 + 63) // 64 * 64
        dev = payload.device
        shards = torch.empty((G, n, shard_pitch), dtype=torch.uint8, device=dev)
        wire = torch.empty((G, n, wire_pitch), dtype=torch.uint8, device=dev)
        wire_len = torch.empty((G, n), dtype=torch.int32, device=dev)
        check(lib().qfec_pack_datagrams(self._h, _dev_ptr(payload, what="payload"), _dev_ptr(offsets, _I64, "offsets"),
                                        _dev_ptr(sizes, _I32, "sizes"), _dev_ptr(seq, _I32, "seq"),
                                        G, int(bool(checksum)), _dev_ptr(shards), shard_pitch, _dev_ptr(wire),
                                        wire_pitch, _dev_ptr(wire_len, _I32), _stream_handle(stream)), "qfec_pack_datagrams")
        return shards, wire, wire_len

    def unpack_datagrams(self, wire, wire_len, checksum=True, dec_pkt_size=2068, shard_pitch=None, stream=None):
        """wire [G, n, wire_pitch] uint8, wire_len int32 [G, n] (0 = not received).  Returns
        (shards [G, n, pitch], status int32 [G, k], psize int32 [G, k], rx_size int32 [G, n])."""
        import torch
        G, n, wire_pitch = wire.shape
        if shard_pitch is None:
            shard_pitch = (wire_pitch - 13) // 16 * 16
        dev = wire.device
        shards = torch.empty((G, n, shard_pitch), dtype=torch.uint8, device=dev)
        marks = torch.empty(G * n, dtype=torch.uint8, device=dev)
        rx = torch.empty((G, n), dtype=torch.int32, device=dev)
        status = torch.empty((G, self.k), dtype=torch.int32, device=dev)
        psize = torch.empty((G, self.k), dtype=torch.int32, device=dev)
        check(lib().qfec_unpack_datagrams(self._h, _dev_ptr(wire, what="wire"), wire_pitch,
                                          _dev_ptr(wire_len, _I32, "wire_len"), G, int(bool(checksum)),
                                          dec_pkt_size, _dev_ptr(shards), shard_pitch, _dev_ptr(marks), _dev_ptr(rx, _I32),
                                          _dev_ptr(status, _I32), _dev_ptr(psize, _I32), _stream_handle(stream)),
              "qfec_unpack_datagrams")
        return shards, status, psize, rx

    # -- the same batches straight to / from ProtocolUdp frames (qfec_pack_frames / qfec_unpack_frames)
    def pack_frames(self, payload, offsets, sizes, seq, masks, gmask=0, cmd=0x11, protocol=0xFF, conv_hid=None,
                    checksum=True, shard_pitch=None, frame_pitch=None, stream=None):
        """pack_datagrams + frame_udp in one call: masks uint8 [G*n] (one per datagram), conv_hid
        int32/uint32 [G*n, 2] or None (no Session prefix).  frame_pitch defaults to the 64-B
        multiple above prefix + 13 + shard_pitch (the one-pass kernel's pitch for 1 KiB and
        512-B payloads).  Returns (frames [G, n, frame_pitch], frame_len int32 [G, n])."""
        import torch
        G = sizes.numel() // self.k
        n = self.k + self.m
        head = 4 if checksum else 2
        P = 12 if conv_hid is not None else 4
        if shard_pitch is None:
            shard_pitch = (int(sizes.max().item()) + head + 15) // 16 * 16 if G else 16
        if frame_pitch is None:
            frame_pitch = (shard_pitch + 13 + P + 63) // 64 * 64
        dev = payload.device
        shards = torch.empty((G, n, shard_pitch), dtype=torch.uint8, device=dev)
        frames = torch.empty((G, n, frame_pitch), dtype=torch.uint8, device=dev)
        flen = torch.empty((G, n), dtype=torch.int32, device=dev)
        check(lib().qfec_pack_frames(self._h, _dev_ptr(payload, what="payload"), _dev_ptr(offsets, _I64, "offsets"),
                                     _dev_ptr(sizes, _I32, "sizes"), _dev_ptr(seq, _I32, "seq"), G, int(bool(checksum)),
                                     _dev_ptr(shards), shard_pitch, _dev_ptr(masks, what="masks"),
                                     _dev_ptr(conv_hid, _I32, "conv_hid") if conv_hid is not None else None,
                                     int(gmask), int(cmd), int(protocol), _dev_ptr(frames), frame_pitch,
                                     _dev_ptr(flen, _I32), _stream_handle(stream)), "qfec_pack_frames")
        return frames, flen

    def unpack_frames(self, frames, frame_len, gmask=0, session=False, checksum=True, dec_pkt_size=2068,
                      shard_pitch=None, stream=None):
        """unframe_udp + unpack_datagrams in one call.  frames [G, n, frame_pitch], frame_len int32
        [G, n] (0 = not received).  Returns (shards, status, psize, rx_size, frame_status [G, n],
        conv_hid [G, n, 2] int32 or None)."""
        import torch
        G, n, fpitch = frames.shape
        P = 12 if session else 4
        if shard_pitch is None:
            shard_pitch = (fpitch - 13 - P) // 16 * 16
        dev = frames.device
        shards = torch.empty((G, n, shard_pitch), dtype=torch.uint8, device=dev)
        marks = torch.empty(G * n, dtype=torch.uint8, device=dev)
        rx = torch.empty((G, n), dtype=torch.int32, device=dev)
        status = torch.empty((G, self.k), dtype=torch.int32, device=dev)
        psize = torch.empty((G, self.k), dtype=torch.int32, device=dev)
        fst = torch.empty((G, n), dtype=torch.int32, device=dev)
        ch = torch.zeros((G, n, 2), dtype=torch.int32, device=dev) if session else None
        check(lib().qfec_unpack_frames(self._h, _dev_ptr(frames, what="frames"), fpitch,
                                       _dev_ptr(frame_len, _I32, "frame_len"), G, int(gmask), int(bool(session)),
                                       int(bool(checksum)), dec_pkt_size, _dev_ptr(shards), shard_pitch, _dev_ptr(marks),
                                       _dev_ptr(rx, _I32), _dev_ptr(status, _I32), _dev_ptr(psize, _I32),
                                       _dev_ptr(fst, _I32), _dev_ptr(ch, _I32) if ch is not None else None,
                                       _stream_handle(stream)), "qfec_unpack_frames")
        return shards, status, psize, rx, fst, ch

    def decode_rows(self, marks_n):
        """Host-side decode matrix for one group-order mark vector: (e, rows[e,k], survivors[k], erased[e])."""
        marks_n = np.ascontiguousarray(marks_n, dtype=np.uint8)
        rows = np.zeros((self.m, self.k), dtype=np.uint8)
        surv = np.zeros(self.k, dtype=np.int32)
        lost = np.zeros(max(self.m, 1), dtype=np.int32)
        e = lib().qfec_decode_rows(self._h, marks_n.ctypes.data, rows.ctypes.data, surv.ctypes.data, lost.ctypes.data)
        if e <= 0:
            return e, None, None, None
        return e, rows[:e].copy(), surv, lost[:e].copy()


class FecParms:
    """system/fec.h: fec_new(k, n) / fec_encode / fec_decode / fec_free over packet buffers."""

    def __init__(self, k, n):
        self.k, self.n = k, n
        self._h = lib().fec_new(k, n)
        if not self._h:
            raise QfecError(f"fec_new({k}, {n}) failed")
        self._h = C.c_void_p(self._h)

    def close(self):
        if self._h:
            lib().fec_free(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def matrix(self):
        out = np.zeros((self.n, self.k), dtype=np.uint8)
        check(lib().qfec_fec_matrix(self._h, out.ctypes.data), "qfec_fec_matrix")
        return out

    def code(self):
        """The batched Code sharing this handle's matrix (not owned)."""
        return Code(lib().qfec_fec_code(self._h), owner=False)

    def encode(self, src, dst, index, sz):
        """src: k host uint8 arrays (or one [k, >=sz] array); dst: uint8 array written in place."""
        rows = [np.ascontiguousarray(s) for s in src]
        ptrs = (C.c_void_p * len(rows))(*[r.ctypes.data for r in rows])
        lib().fec_encode(self._h, ptrs, C.c_void_p(dst.ctypes.data), index, sz)

    def decode(self, pkts, index, sz):
        """pkts: [k, >=sz] uint8 array (slots), index: k ints.  Returns (rc, pkts_after, index_after)
        with the reference's in-place pointer/index permutation applied to copies."""
        buf = np.ascontiguousarray(pkts, dtype=np.uint8).copy()
        k, stride = buf.shape
        base = buf.ctypes.data
        ptrs = (C.c_void_p * k)(*[base + s * stride for s in range(k)])
        ia = (C.c_int * k)(*[int(x) for x in index])
        rc = lib().fec_decode(self._h, ptrs, ia, sz)
        after = np.stack([buf[(ptrs[s] - base) // stride] for s in range(k)])
        return rc, after, np.array(list(ia), dtype=np.int32)


class ReedSolomon:
    """module/rs.h: reed_solomon_new / encode / reconstruct / release over shard pointers."""

    def __init__(self, k, m):
        L = lib()
        L.reed_solomon_init()
        self._h = L.reed_solomon_new(k, m)
        if not self._h:
            raise QfecError(f"reed_solomon_new({k}, {m}) failed: errno {L.reed_solomon_error()}")
        self.k, self.m = k, m

    def close(self):
        if self._h:
            lib().reed_solomon_release(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def parity(self):
        """The public parity matrix (editable, as in rs.h:12)."""
        return np.ctypeslib.as_array(self._h.contents.parity, shape=(self.m, self.k))

    @property
    def m_matrix(self):
        """The public n x k matrix rs->m (editable, as in rs.h:11): reconstruct decodes from it."""
        return np.ctypeslib.as_array(self._h.contents.m, shape=(self.k + self.m, self.k))

    def code(self):
        """The batched code behind this handle (qfec_rs_code): the handle's current matrices."""
        return Code(lib().qfec_rs_code(self._h), owner=False)

    @staticmethod
    def _ptrs(data, parity):
        G, k, pitch = data.shape
        m = parity.shape[1]
        db, pb = data.ctypes.data, parity.ctypes.data
        return (C.c_void_p * (G * (k + m)))(*([db + i * pitch for i in range(G * k)] +
                                               [pb + i * pitch for i in range(G * m)]))

    def encode(self, data, parity, block_size):
        """data [G,k,pitch], parity [G,m,pitch] host uint8 arrays (parity written)."""
        G = data.shape[0]
        return lib().reed_solomon_encode(self._h, self._ptrs(data, parity), G * (self.k + self.m), block_size)

    def reconstruct(self, data, parity, marks, block_size):
        G = data.shape[0]
        marks = np.ascontiguousarray(marks, dtype=np.uint8)
        return lib().reed_solomon_reconstruct(self._h, self._ptrs(data, parity), C.c_void_p(marks.ctypes.data),
                                              G * (self.k + self.m), block_size)


_PACK_OUT = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_char), C.c_uint)
_UNPACK_OUT = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_char), C.c_uint, C.c_uint)


class NetFec:
    """Batched NetFecCodec layer (include/qfec_net.h): sessions keep zfec_pack_input's
    numbering; complete groups of all sessions go out in one device launch per flush, and
    received groups come back the same way.  Callbacks get (session, bytes[, src index])."""

    def __init__(self, k, n, max_pkt_size=2048, checksum=True):
        self._h = lib().qfec_net_new(k, n, max_pkt_size, int(bool(checksum)))
        if not self._h:
            raise QfecError(f"qfec_net_new({k}, {n}, {max_pkt_size}) failed")
        self.k, self.n = k, n

    def close(self):
        if self._h:
            lib().qfec_net_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def session(self):
        """A new session; its id is also its callback peer (id + 1)."""
        self._nsess = getattr(self, "_nsess", 0)
        s = lib().qfec_net_session(self._h, C.c_void_p(self._nsess + 1))
        check(min(s, 0), "qfec_net_session")
        self._nsess += 1
        return s

    def enable(self, session, on=True):
        """enable_zfec: with FEC off a session's packets go out as [0x13][payload]."""
        check(lib().qfec_net_enable(self._h, session, int(bool(on))), "qfec_net_enable")

    def pack_input(self, session, data):
        b = bytes(data)
        check(lib().qfec_net_pack_input(self._h, session, b, len(b)), "qfec_net_pack_input")

    def flush_pack(self, stream=None):
        """-> [(session, datagram bytes)] in emission order (each session's in sent order)."""
        out = []

        def cb(peer, p, size):
            out.append((int(peer) - 1, C.string_at(p, size)))
            return 0

        f = _PACK_OUT(cb)
        rc = lib().qfec_net_flush_pack(self._h, f, _stream_handle(stream))
        check(min(rc, 0), "qfec_net_flush_pack")
        return out

    def unpack_input(self, session, datagram):
        b = bytes(datagram)
        rc = lib().qfec_net_unpack_input(self._h, session, b, len(b))
        check(min(rc, 0), "qfec_net_unpack_input")
        return rc

    def flush_unpack(self, all_groups=False, stream=None):
        """-> [(session, payload bytes, src index)] delivered, group by group in source order."""
        out = []

        def cb(peer, p, size, src):
            out.append((int(peer) - 1, C.string_at(p, size), src))
            return 0

        f = _UNPACK_OUT(cb)
        rc = lib().qfec_net_flush_unpack(self._h, f, int(bool(all_groups)), _stream_handle(stream))
        check(min(rc, 0), "qfec_net_flush_unpack")
        return out

    def stats(self):
        a = (C.c_longlong * 8)()
        check(lib().qfec_net_stats(self._h, a), "qfec_net_stats")
        keys = ["groups_packed", "datagrams_out", "groups_unpacked", "delivered", "recovered", "undecodable",
                "foreign", "late"]
        return dict(zip(keys, list(a)))


class Zfec:
    """The exact NetFecCodec layer (include/qfec_zfec.h): per-session calls are queued in call
    order and flush() runs them through the reference's zfec_pack_input / zfec_unpack_input
    state machines, all byte work in batched device launches.  flush() returns
    (datagrams, deliveries): [(session, bytes)] and [(session, payload, src index)], each
    session's in the order the reference's PackOutput / UnpackOutput would have seen them."""

    def __init__(self, _lib=None):
        self._L = _lib or lib()  # (_lib: another build of the layer, for the CPU suite)
        self._h = self._L.qfec_zfec_new()
        if not self._h:
            raise QfecError("qfec_zfec_new failed")
        self._nsess = 0

    def close(self):
        if self._h:
            self._L.qfec_zfec_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def session(self, max_pkt_size=2048, buf_items=48, kmax=10, k=4, n=5, enabled=True, is_sorted=False):
        """FecTransmission::Init (CreateFecTransmission's defaults); the callback peer is id + 1."""
        s = self._L.qfec_zfec_session(self._h, C.c_void_p(self._nsess + 1), max_pkt_size, buf_items, kmax, k, n,
                                    int(bool(enabled)), int(bool(is_sorted)))
        check(min(s, 0), "qfec_zfec_session")
        self._nsess += 1
        return s

    def set_kn(self, session, k, n, add_new=True):
        rc = self._L.qfec_zfec_set_kn(self._h, session, k, n, int(bool(add_new)))
        check(rc, f"qfec_zfec_set_kn({k}, {n})")

    def enable(self, session, on=True):
        check(self._L.qfec_zfec_enable(self._h, session, int(bool(on))), "qfec_zfec_enable")

    def sorted(self, session, on=True):
        check(self._L.qfec_zfec_sorted(self._h, session, int(bool(on))), "qfec_zfec_sorted")

    def dynkn(self, session, on=True):
        check(self._L.qfec_zfec_dynkn(self._h, session, int(bool(on))), "qfec_zfec_dynkn")

    def lost_rate(self, session, rate):
        check(self._L.qfec_zfec_lost_rate(self._h, session, float(rate)), "qfec_zfec_lost_rate")

    def pack_input(self, session, data):
        b = bytes(data)
        check(self._L.qfec_zfec_pack_input(self._h, session, b, len(b)), "qfec_zfec_pack_input")

    def unpack_input(self, session, datagram):
        b = bytes(datagram)
        check(self._L.qfec_zfec_unpack_input(self._h, session, b, len(b)), "qfec_zfec_unpack_input")

    def flush(self, stream=None):
        sent, got = [], []

        def pcb(peer, p, size):
            sent.append((int(peer) - 1, C.string_at(p, size)))
            return 0

        def ucb(peer, p, size, src):
            got.append((int(peer) - 1, C.string_at(p, size), src))
            return 0

        f, g = _PACK_OUT(pcb), _UNPACK_OUT(ucb)
        rc = self._L.qfec_zfec_flush(self._h, f, g, _stream_handle(stream))
        check(min(rc, 0), "qfec_zfec_flush")
        return sent, got

    def stats(self, session):
        a = (C.c_longlong * 8)()
        check(self._L.qfec_zfec_stats(self._h, session, a), "qfec_zfec_stats")
        keys = ["fec_src_count", "fec_restore_count", "i_sent_pkt", "i_recv_pkt", "i_expected_packet", "k", "n",
                "undefined"]
        return dict(zip(keys, list(a)))


def _host_ptr(a, what):
    """Address of a contiguous uint8 host buffer (numpy array or CPU tensor)."""
    if isinstance(a, np.ndarray):
        if not a.flags["C_CONTIGUOUS"] or a.dtype != np.uint8:
            raise QfecError(f"{what}: contiguous uint8 host array required")
        return C.c_void_p(a.ctypes.data)
    import torch
    if a.is_cuda or not a.is_contiguous() or a.dtype != torch.uint8:
        raise QfecError(f"{what}: contiguous uint8 host tensor required")
    return C.c_void_p(a.data_ptr())


class Pipe:
    """include/qfec.h qfec_pipe: batches streamed host -> device -> host over `streams` HIP
    streams per device on `devices` (None: every visible device), each stream slot holding
    `slot_bytes` of device staging.  encode / reconstruct queue a batch and return; wait()
    blocks until every queued batch is done and returns the under-determined group count.
    Buffers must be PINNED host memory (torch .pin_memory() tensors or hipHostMalloc'd) and
    are kept referenced here until wait()."""

    def __init__(self, devices=None, streams=3, slot_bytes=96 << 20):
        devs = list(devices) if devices else []
        arr = (C.c_int * len(devs))(*devs) if devs else None
        h = lib().qfec_pipe_new(arr, len(devs), streams, slot_bytes)
        if not h:
            raise QfecError(f"qfec_pipe_new: {lib().qfec_last_error().decode()}")
        self._h = C.c_void_p(h)
        self.slots = lib().qfec_pipe_slots(self._h)
        self._held = []

    def close(self):
        if self._h:
            lib().qfec_pipe_free(self._h)
            self._h = None
            self._held = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def encode(self, code, data, parity, block_size=None):
        G, k, pitch = data.shape
        if k != code.k or tuple(parity.shape) != (G, code.m, pitch):
            raise QfecError("pipe encode: shape mismatch")
        block_size = pitch if block_size is None else block_size
        check(lib().qfec_pipe_encode(self._h, code._h, _host_ptr(data, "data"), _host_ptr(parity, "parity"), G,
                                     block_size, pitch), "qfec_pipe_encode")
        self._held += [code, data, parity]

    def reconstruct(self, code, data, parity, marks, block_size=None):
        G, k, pitch = data.shape
        nmarks = marks.size if isinstance(marks, np.ndarray) else marks.numel()
        if k != code.k or tuple(parity.shape) != (G, code.m, pitch) or nmarks != G * (code.k + code.m):
            raise QfecError("pipe reconstruct: shape mismatch")
        block_size = pitch if block_size is None else block_size
        check(lib().qfec_pipe_reconstruct(self._h, code._h, _host_ptr(data, "data"), _host_ptr(parity, "parity"),
                                          _host_ptr(marks, "marks"), G, block_size, pitch), "qfec_pipe_reconstruct")
        self._held += [code, data, parity, marks]

    def wait(self):
        nf = C.c_longlong(0)
        rc = lib().qfec_pipe_wait(self._h, C.byref(nf))
        self._held = []
        check(rc, "qfec_pipe_wait")
        return int(nf.value)
