"""ctypes front-end for the parity checkers -- TEST INFRASTRUCTURE ONLY.

Importable only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.

* ``Oracle``   -- oracle/liboracle.so, the CPU restatement of the reference codecs
                  (oracle/qfec_oracle.c; every function cites module/rs.c or module/fec.c).
* ``RefCodec`` -- oracle/_ref/libref_{rs,fec}.so, the reference's own C compiled from
                  /root/reference by ``make -C oracle ref`` (present only when built).
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
U8P = C.POINTER(C.c_ubyte)


def _p(a):
    return C.c_void_p(a.ctypes.data)


class Oracle:
    def __init__(self, path=None):
        path = path or os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle`")
        L = C.CDLL(path)
        vp, i, ll = C.c_void_p, C.c_int, C.c_longlong
        L.orc_init()
        L.orc_cauchy_parity.argtypes = [i, i, vp]
        L.orc_vandermonde_parity.argtypes = [i, i, vp]
        L.orc_invert.argtypes = [vp, i]
        L.orc_rs_encode_contig.argtypes = [i, i, vp, vp, vp, ll, i, ll]
        L.orc_fec_encode_contig.argtypes = [i, i, vp, vp, vp, ll, i, ll]
        L.orc_rs_reconstruct_contig.argtypes = [i, i, vp, vp, vp, vp, ll, i, ll]
        L.orc_rs_reconstruct_full_contig.argtypes = [i, i, vp, vp, vp, vp, ll, i, ll]
        L.orc_fec_reconstruct_contig.argtypes = [i, i, vp, vp, vp, vp, ll, i, ll]
        L.orc_fec_reconstruct_contig.restype = ll
        L.orc_fec_decode.argtypes = [i, i, vp, C.POINTER(vp), C.POINTER(C.c_int), i]
        L.orc_fec_encode.argtypes = [i, i, vp, C.POINTER(vp), vp, i, i]
        L.orc_mul.restype = C.c_ubyte
        L.orc_mul.argtypes = [C.c_ubyte, C.c_ubyte]
        L.orc_inv.restype = C.c_ubyte
        L.orc_inv.argtypes = [C.c_ubyte]
        L.orc_byte_sum.restype = C.c_uint32
        L.orc_byte_sum.argtypes = [vp, ll]
        L.orc_pack_group.argtypes = [i, i, vp, vp, vp, vp, C.c_uint32, C.c_uint32, i, i, vp, ll, vp]
        L.orc_unpack_head.argtypes = [vp, i] + [C.POINTER(C.c_uint32)] * 2 + [C.POINTER(i)] * 4 + [vp, C.POINTER(i)]
        L.orc_dec_src.argtypes = [vp, i, i, C.POINTER(i)]
        L.orc_frame_udp.argtypes = [vp, i, i, i, i, i, i, C.c_uint32, C.c_uint32, vp]
        L.orc_unframe_udp.argtypes = [vp, i, i, i, vp, vp]
        self.L = L

    # -- matrices
    def cauchy(self, k, m):
        out = np.zeros((max(m, 1), max(k, 1)), dtype=np.uint8)
        rc = self.L.orc_cauchy_parity(k, m, _p(out))
        return None if rc else out

    def vandermonde(self, k, n):
        """Parity rows k..n-1 of the fec.c systematic matrix ((n-k) x k)."""
        out = np.zeros((max(n - k, 1), max(k, 1)), dtype=np.uint8)
        rc = self.L.orc_vandermonde_parity(k, n, _p(out))
        return None if rc else out[: n - k]

    def invert(self, mat):
        a = np.ascontiguousarray(mat, dtype=np.uint8).copy()
        rc = self.L.orc_invert(_p(a), a.shape[0])
        return None if rc else a

    def invert_partial(self, mat):
        """invert_mat as rs.c uses it: (rc, matrix as left), the partial state when singular."""
        a = np.ascontiguousarray(mat, dtype=np.uint8).copy()
        return self.L.orc_invert(_p(a), a.shape[0]), a

    def mul(self, a, b):
        return int(self.L.orc_mul(a, b))

    # -- contiguous batches: data[G][k][pitch], parity[G][m][pitch]
    def rs_encode(self, rows, data, parity, length):
        G, k, pitch = data.shape
        m = parity.shape[1]
        self.L.orc_rs_encode_contig(k, m, _p(np.ascontiguousarray(rows)), _p(data), _p(parity), G, length, pitch)

    def fec_encode(self, rows, data, parity, length):
        G, k, pitch = data.shape
        m = parity.shape[1]
        self.L.orc_fec_encode_contig(k, m, _p(np.ascontiguousarray(rows)), _p(data), _p(parity), G, length, pitch)

    def rs_reconstruct(self, rows, data, parity, marks_rs, length):
        G, k, pitch = data.shape
        m = parity.shape[1]
        return self.L.orc_rs_reconstruct_contig(k, m, _p(np.ascontiguousarray(rows)), _p(data), _p(parity),
                                                _p(marks_rs), G, length, pitch)

    def rs_reconstruct_full(self, full, data, parity, marks_rs, length):
        """reed_solomon_reconstruct with the handle's whole n x k matrix rs->m (rs.c:505, 536-556)."""
        G, k, pitch = data.shape
        m = parity.shape[1]
        return self.L.orc_rs_reconstruct_full_contig(k, m, _p(np.ascontiguousarray(full, dtype=np.uint8)), _p(data),
                                                     _p(parity), _p(marks_rs), G, length, pitch)

    def fec_reconstruct(self, rows, data, parity, marks_rs, length):
        G, k, pitch = data.shape
        m = parity.shape[1]
        return self.L.orc_fec_reconstruct_contig(k, m, _p(np.ascontiguousarray(rows)), _p(data), _p(parity),
                                                 _p(marks_rs), G, length, pitch)

    def fec_decode(self, k, n, full, pkts, idx):
        """fec_decode on a copy: returns (rc, pkts_after[k][B], idx_after)."""
        buf = np.ascontiguousarray(pkts, dtype=np.uint8).copy()
        B = buf.shape[1]
        base = buf.ctypes.data
        ptrs = (C.c_void_p * k)(*[base + s * B for s in range(k)])
        ia = (C.c_int * k)(*[int(x) for x in idx])
        rc = self.L.orc_fec_decode(k, n, _p(np.ascontiguousarray(full)), ptrs, ia, B)
        after = np.stack([buf[(ptrs[s] - base) // B] for s in range(k)])
        return rc, after, np.array(list(ia), dtype=np.int32)

    def byte_sum(self, a):
        return int(self.L.orc_byte_sum(_p(a), a.size))

    # -- FEC wire marshalling (network/FecCodecBuf.cpp)
    def pack_group(self, k, n, rows_full, payload, offs, sizes, sent0, src0, checksum, shard_cap=2052, pitch=2068):
        """One full group through zfec_pack_input's send path: (datagrams [n][pitch], lengths[n], groupMax)."""
        out = np.zeros((n, pitch), dtype=np.uint8)
        ln = np.zeros(n, dtype=np.int32)
        offs = np.ascontiguousarray(offs, dtype=np.int64)
        sizes = np.ascontiguousarray(sizes, dtype=np.int32)
        pl = payload if payload.size else np.zeros(1, np.uint8)
        gmax = self.L.orc_pack_group(k, n, _p(np.ascontiguousarray(rows_full)), _p(pl), _p(offs), _p(sizes),
                                     sent0, src0, checksum, shard_cap, _p(out), pitch, _p(ln))
        return out, ln, gmax

    def frame_udp(self, data, mask, gmask=0, cmd=0x11, protocol=0xFF, conv_hid=None):
        """ProtocolUdp framing of one datagram (parity unpinned: ProtocolBasic.cpp does not build)."""
        d = np.ascontiguousarray(data, dtype=np.uint8)
        out = np.zeros(len(d) + 12, np.uint8)
        sess = conv_hid is not None
        conv, hid = (int(conv_hid[0]) & 0xFFFFFFFF, int(conv_hid[1]) & 0xFFFFFFFF) if sess else (0, 0)
        n = self.L.orc_frame_udp(_p(d), len(d), int(mask), int(gmask), int(cmd), int(protocol), int(sess), conv, hid,
                                 _p(out))
        return out[:n]

    def unframe_udp(self, frame, gmask=0, session=False):
        """-> (status, un-XORed frame bytes, info[4])."""
        f = np.ascontiguousarray(frame, dtype=np.uint8)
        work = np.zeros(max(len(f), 1), np.uint8)
        info = np.zeros(4, np.uint8)
        st = self.L.orc_unframe_udp(_p(f), len(f), int(gmask), int(bool(session)), _p(work), _p(info))
        return st, work[:len(f)], info

    def unpack_head(self, dgram):
        """unpack_fec_head: (rc, sent, src, n, k, ik, is_checksum, shard bytes)."""
        d = np.ascontiguousarray(dgram, dtype=np.uint8)
        sent, src = C.c_uint32(), C.c_uint32()
        n, k, ik, cs, sl = (C.c_int() for _ in range(5))
        shard = np.zeros(max(d.size, 1), dtype=np.uint8)
        rc = self.L.orc_unpack_head(_p(d), d.size, C.byref(sent), C.byref(src), C.byref(n), C.byref(k), C.byref(ik),
                                    C.byref(cs), _p(shard), C.byref(sl))
        body = shard[: sl.value].copy() if rc == 1 else None
        return rc, sent.value, src.value, n.value, k.value, ik.value, cs.value, body

    def dec_src(self, shard, dec_pkt_size, checksum):
        sz = C.c_int()
        s = np.ascontiguousarray(shard, dtype=np.uint8)
        off = self.L.orc_dec_src(_p(s), dec_pkt_size, checksum, C.byref(sz))
        return off, sz.value


class RS(C.Structure):  # module/rs.h:7-13
    _fields_ = [("data_shards", C.c_int), ("parity_shards", C.c_int), ("shards", C.c_int),
                ("m", U8P), ("parity", U8P)]


class RefCodec:
    """The reference's own codecs (oracle/_ref), for the CPU baseline and cross-checks."""

    def __init__(self):
        d = os.path.join(HERE, "_ref")
        self.rs = C.CDLL(os.path.join(d, "libref_rs.so"))
        self.fec = C.CDLL(os.path.join(d, "libref_fec.so"))
        self.rs.reed_solomon_new.restype = C.POINTER(RS)
        self.rs.reed_solomon_new.argtypes = [C.c_int, C.c_int]
        self.rs.reed_solomon_release.argtypes = [C.POINTER(RS)]
        self.rs.reed_solomon_encode.argtypes = [C.POINTER(RS), C.POINTER(C.c_void_p), C.c_int, C.c_int]
        self.rs.reed_solomon_reconstruct.argtypes = [C.POINTER(RS), C.POINTER(C.c_void_p), C.c_void_p, C.c_int, C.c_int]
        self.fec.fec_new.restype = C.c_void_p
        self.fec.fec_new.argtypes = [C.c_int, C.c_int]
        self.fec.fec_free.argtypes = [C.c_void_p]
        self.fec.fec_encode.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.c_void_p, C.c_int, C.c_int]
        self.fec.fec_decode.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_int), C.c_int]
        self.rs.reed_solomon_init()

    @staticmethod
    def available():
        d = os.path.join(HERE, "_ref")
        return all(os.path.exists(os.path.join(d, f)) for f in ("libref_rs.so", "libref_fec.so"))

    def shard_ptrs(self, data, parity):
        """module/rs.c pointer layout: all data shards, then all parity shards."""
        G, k, pitch = data.shape
        m = parity.shape[1]
        db, pb = data.ctypes.data, parity.ctypes.data
        return (C.c_void_p * (G * (k + m)))(*([db + i * pitch for i in range(G * k)] +
                                               [pb + i * pitch for i in range(G * m)]))

    def rs_encode(self, h, ptrs, nshards, length):
        return self.rs.reed_solomon_encode(h, ptrs, nshards, length)

    def rs_reconstruct(self, h, ptrs, marks, nshards, length):
        return self.rs.reed_solomon_reconstruct(h, ptrs, _p(marks), nshards, length)


class FecCodecBufS(C.Structure):  # network/FecCodecBuf.h:19-36
    _fields_ = [("enc_pkt_size", C.c_int), ("enc_kmax", C.c_int), ("is_checksum", C.c_bool),
                ("is_send_checksum", C.c_bool), ("fec_en_buf", C.c_void_p), ("sent_buf", C.c_void_p),
                ("en_check_pkt", C.c_void_p), ("dec_pkt_size", C.c_int), ("dec_kmax", C.c_int),
                ("fecDecoderBuf", C.c_void_p), ("fecDecoderIndices", C.c_void_p), ("dec_buf", C.c_void_p),
                ("dec_check_pkt", C.c_void_p)]


class FecCodecHead(C.Structure):  # network/FecCodecBuf.h:10-17
    _fields_ = [("sent_pkt_index", C.c_uint32), ("src_pkt_index", C.c_uint32), ("codec_n", C.c_ubyte),
                ("codec_k", C.c_ubyte), ("ik", C.c_ubyte)]


def load_callers(path):
    """The reference's network/FecCodec.cpp + FecCodecBuf.cpp built by `make -C oracle ref`."""
    L = C.CDLL(path)
    P, vp, i, ip = C.POINTER(FecCodecBufS), C.c_void_p, C.c_int, C.POINTER(C.c_int)
    L.init_fec_buf.argtypes = [P, i, i]
    L.release_fec_buf.argtypes = [P]
    L.set_fec_enc_buf.argtypes = [P, i, vp, i, ip]
    L.set_fec_enc_buf.restype = vp
    L.get_fec_encoded_pkt.argtypes = [P, vp, i, i, ip]
    L.get_fec_encoded_pkt.restype = vp
    L.pack_fec_head.argtypes = [P, C.POINTER(FecCodecHead), vp, i, ip]
    L.pack_fec_head.restype = vp
    L.unpack_fec_head.argtypes = [P, C.POINTER(FecCodecHead), vp, i, ip]
    L.unpack_fec_head.restype = vp
    L.set_fec_dec_buf.argtypes = [P, i, vp, i, i]
    L.set_fec_dec_buf.restype = vp
    L.reset_fec_dec_buf.argtypes = [P]
    L.fec_decode_pkts.argtypes = [P, vp, i]
    L.get_fec_decoded_pkt.argtypes = [P, i]
    L.get_fec_decoded_pkt.restype = vp
    L.dec_src_pkt_info.argtypes = [vp, P, C.POINTER(C.c_uint16)]
    L.dec_src_pkt_info.restype = vp
    return L
