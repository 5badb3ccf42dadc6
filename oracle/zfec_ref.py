"""TEST INFRASTRUCTURE ONLY -- never imported by the product (quicknet_amd/, libqfec.so).

A restatement of network/NetFecCodec.cpp's per-packet FEC layer (one NetFecCodecLayer per
session), the checker for libqfec's batched exact layer (include/qfec_zfec.h):

  ZfecLayer.pack_input      zfec_pack_input       NetFecCodec.cpp:68-175
  ZfecLayer.unpack_input    zfec_unpack_input     NetFecCodec.cpp:189-371
  ZfecLayer._add_packet     add_packet_fec_buf    NetFecCodec.cpp:485-535
  ZfecLayer._update_window  update_fec_dec_buf    NetFecCodec.cpp:540-554
  ZfecLayer._flush_avail    flush_avail_pkts      NetFecCodec.cpp:407-443
  ZfecLayer.set_kn          set_zfec_kn           NetFecCodec.cpp:591-611
  ZfecLayer._recalc_kn      recalc_zfec_kn        NetFecCodec.cpp:51-65
  ZfecLayer.__init__        init_zfec_layer       NetFecCodec.cpp:613-669, with FecTransmission::Init's
                            candidate (k, n) list  FecTransmission.cpp:240-257
  _CodecList                FecCodecList (std::map<float, FecCodec*>): find_codec, get_codec_by,
                            add_new_codec         FecCodec.cpp:18-95
  _Slot                     FecPacket             FecPacket.h:10-140

Only the CONTROL FLOW above is restated.  Every buffer and codec operation it makes is the
reference's own compiled code: network/FecCodecBuf.cpp (unpack_fec_head, set_fec_dec_buf,
reset_fec_dec_buf, fec_decode_pkts, get_fec_decoded_pkt, dec_src_pkt_info, set_fec_enc_buf,
pack_fec_head, get_fec_encoded_pkt, pack_fec_off_tag, init_fec_buf) and system/fec.c (fec_new),
as built by `make -C oracle ref` into oracle/_ref/libref_feccodec_ref.so.  NetFecCodec.cpp itself
does not build here (its Trace comes from ProtocolBasic.cpp, which needs the absent
system/option.h), so the control flow is PARITY UNPINNED: it is checked by reading, line by line,
against the cited source, and by round trips through the reference's own buffer code.

Unsigned 32-bit sequence arithmetic (IUINT32) wraps as in C; `int ck = IUINT32 - IUINT32 + i`
conversions are reproduced with _i32.
"""
import ctypes as C
import os

from oracle.oracle import FecCodecBufS, FecCodecHead, load_callers

REF_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_ref", "libref_feccodec_ref.so")
U32 = 0xFFFFFFFF


def _u32(x):
    return x & U32


def _i32(x):
    x &= U32
    return x - (1 << 32) if x & 0x80000000 else x


def _cmod(a, b):
    """C's int % (truncating division)."""
    r = abs(a) % abs(b)
    return -r if a < 0 else r


def available():
    return os.path.exists(REF_LIB)


_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        L = load_callers(REF_LIB)
        L.fec_new.restype = C.c_void_p
        L.fec_new.argtypes = [C.c_int, C.c_int]
        L.fec_free.argtypes = [C.c_void_p]
        L.pack_fec_off_tag.argtypes = [C.POINTER(FecCodecBufS), C.c_void_p, C.c_int, C.POINTER(C.c_int)]
        L.pack_fec_off_tag.restype = C.c_void_p
        _LIB = L
    return _LIB


class _Slot:
    """FecPacket (FecPacket.h): one dec_pkts_buf entry of the receive window.  `fec_buf` models
    the whole FecBuf allocation (MaxBufSize bytes), since dec_src_pkt_info may read past BufSize."""

    def __init__(self, max_size):
        self.iPacket = -1
        self.fec_buf = bytearray(max_size)  # Reset() in init_zfec_layer calloc's it (:661-664)
        self.BufSize = 0
        self.bValid = False
        self.MaxBufSize = max_size
        self.bSourcePkt = True
        self.i_source_pkt = -1
        self.bUsed = False

    def _resize(self, size):           # realloc: the kept prefix, zeros past it (calloc'd pool)
        if len(self.fec_buf) < size:
            self.fec_buf.extend(bytes(size - len(self.fec_buf)))
        else:
            del self.fec_buf[size:]

    def set_packet(self, data):        # SetPacket (FecPacket.h:78-98)
        if len(data) > self.MaxBufSize:
            self.MaxBufSize = len(data)
        self._resize(self.MaxBufSize)
        self.fec_buf[:] = bytes(self.MaxBufSize)
        self.fec_buf[:len(data)] = data
        self.BufSize = len(data)
        self.bValid = True
        self.bUsed = False

    def reset(self, max_size):         # Reset (:99-122)
        self.iPacket = -1
        self.BufSize = 0
        self._resize(max_size)
        self.fec_buf[:] = bytes(max_size)
        self.MaxBufSize = max_size
        self.bValid = False
        self.bUsed = False

    def assign(self, o):               # operator= (:42-68): copies o's BufSize bytes only
        self.iPacket = o.iPacket
        self.MaxBufSize = o.MaxBufSize
        self._resize(self.MaxBufSize)
        self.fec_buf[:o.BufSize] = o.fec_buf[:o.BufSize]
        self.BufSize = o.BufSize
        self.bValid = o.bValid
        self.bSourcePkt = o.bSourcePkt
        self.i_source_pkt = o.i_source_pkt
        self.bUsed = o.bUsed

    @property
    def buf(self):
        return bytes(self.fec_buf)

    def valid(self):                   # IsValid (:124-127)
        return self.bValid


class _CodecList:
    """FecCodecList = std::map<float redundancy 1 - k/n, FecCodec*> (FecCodec.h, FecCodec.cpp).
    An entry may hold NULL (None): add_new_codec deletes the entry of equal redundancy and its
    std::map::insert of the new item then does not replace the key (:86-93)."""

    def __init__(self):
        self.items = {}   # float32 key -> (k, n, fec handle) or None

    def find(self, k, n):              # find_codec (FecCodec.cpp:18-34): map order, first match
        for key in sorted(self.items):
            it = self.items[key]
            if it is not None and it[0] == k and it[1] == n:
                return it
        return None

    def add(self, k, n):               # add_new_codec (:77-95)
        key = C.c_float(1.0 - C.c_float(float(k) / float(n)).value).value
        item = (k, n, lib().fec_new(k, n))
        if key in self.items:
            self.items[key] = None     # delete it->second; it->second = NULL; insert() keeps the key
        else:
            self.items[key] = item
        return item

    def by_lost(self, lost):           # get_codec_by (:36-72); NULL entries are not skipped
        if not self.items:
            return None
        lost = C.c_float(lost).value
        last_rate, last = 0.0, None
        for i, key in enumerate(sorted(self.items)):
            it = self.items[key]
            if i == 0:
                if last_rate <= lost <= key and it is not None:
                    return it
            elif last_rate < lost <= key and it is not None:
                return it
            last_rate, last = key, it
        return last


class ZfecLayer:
    """One session's NetFecCodecLayer, set up as FecTransmission::Init does."""

    def __init__(self, max_pkt_size=2048, buf_items=48, kmax=10, k=4, n=5, enabled=True, is_sorted=False):
        L = lib()
        self.buf = FecCodecBufS()
        L.init_fec_buf(C.byref(self.buf), max_pkt_size, kmax)   # init_zfec_layer :616
        self.buf.is_send_checksum = True                       # :617
        self.buf.is_checksum = False                           # :619
        self.codecs = _CodecList()
        self.fec_codec = None
        self.max_pkt_size = max_pkt_size
        self.i_sent_pkt = self.i_recv_pkt = self.i_sent_src_pkt = 0
        self.i_cur_segment_beg = self.i_expected_packet = 0
        self.limit = buf_items
        self.first, self.second = 0, buf_items                 # dec_buf_ipkt_range :629
        self.slots = [_Slot(max_pkt_size + 16) for _ in range(buf_items)]
        self.lost_rate = 0.20                                  # :632
        self.is_sorted = True
        self.dynkn = False
        self.fec_restore_count = self.fec_src_count = 0
        self.nGroupMaxPktSize = 0
        self.is_enabled = False                                # :665
        for kk, nn in zip((2, 3, 5, 4, 3, 4, 5, 7), (4, 5, 8, 6, 4, 5, 6, 8)):  # FecTransmission.cpp:247-253
            self.set_kn(kk, nn, True)
        self.set_kn(k, n, True)
        self.is_enabled = enabled
        self.is_sorted = is_sorted
        self.out = []     # PackOutput datagrams, in order
        self.deliv = []   # UnpackOutput (payload, i_src_pkt), in order

    def close(self):
        L = lib()
        for it in self.codecs.items.values():
            if it is not None:
                L.fec_free(it[2])
        L.release_fec_buf(C.byref(self.buf))

    # ---- configuration
    def set_kn(self, k, n, add_new=True):                      # :591-611
        if k < 0 or n < 0 or k > n:
            return -1
        cur = self.codecs.find(k, n)
        if cur:
            self.fec_codec = cur
        elif add_new:
            self.fec_codec = self.codecs.add(k, n)
        return -2 if self.fec_codec is None else 0

    def _recalc_kn(self):                                      # :51-65
        if self.fec_codec is None:
            return
        cur = self.codecs.by_lost(self.lost_rate)
        self.fec_codec = cur if cur is not None else self.fec_codec

    # ---- send
    def pack_input(self, data):                                # zfec_pack_input :68-175
        L = lib()
        data = bytes(data)
        size = len(data)
        if not self.is_enabled or self.fec_codec is None:      # :75-94
            ps = C.c_int(0)
            p = L.pack_fec_off_tag(C.byref(self.buf), data, size, C.byref(ps))
            self.out.append(C.string_at(p, ps.value) if p and ps.value > 0 else data)
            return
        cur_k, cur_n = self.fec_codec[0], self.fec_codec[1]
        ik = _u32(self.i_sent_pkt - self.i_cur_segment_beg) % cur_n
        if ik < cur_k:                                         # :100-132
            head = FecCodecHead(self.i_sent_pkt, self.i_sent_src_pkt, cur_n, cur_k, ik)
            en = C.c_int(-1)
            penc = L.set_fec_enc_buf(C.byref(self.buf), ik, data, size, C.byref(en))
            self.nGroupMaxPktSize = en.value if ik == 0 else max(self.nGroupMaxPktSize, en.value)
            ps = C.c_int(-1)
            pp = L.pack_fec_head(C.byref(self.buf), C.byref(head), penc, en.value, C.byref(ps))
            if pp and ps.value > 0:
                self.out.append(C.string_at(pp, ps.value))
            self.i_sent_pkt = _u32(self.i_sent_pkt + 1)
            self.i_sent_src_pkt = _u32(self.i_sent_src_pkt + 1)
        if ik == cur_k - 1:                                    # :133-172
            enc = self.fec_codec[2]
            for ik in range(cur_k, cur_n):
                head = FecCodecHead(self.i_sent_pkt, _u32(self.i_sent_src_pkt - 1), cur_n, cur_k, ik)
                if self.nGroupMaxPktSize <= 0:
                    self.nGroupMaxPktSize = self.max_pkt_size
                en = C.c_int(-1)
                pchk = L.get_fec_encoded_pkt(C.byref(self.buf), enc, ik, self.nGroupMaxPktSize, C.byref(en))
                ps = C.c_int(-1)
                pp = L.pack_fec_head(C.byref(self.buf), C.byref(head), pchk, en.value, C.byref(ps))
                if ps.value > 0 and pp:
                    self.out.append(C.string_at(pp, ps.value))
                self.i_sent_pkt = _u32(self.i_sent_pkt + 1)
            if self.dynkn:
                self._recalc_kn()
            self.i_cur_segment_beg = self.i_sent_pkt

    # ---- receive
    def _deliver(self, p, size, src):
        self.deliv.append((C.string_at(p, size), _u32(src)))

    def _used(self, i):                                        # is_fec_dec_buf_used :556-564
        if self.first <= i < self.second:
            return self.slots[i - self.first].bUsed
        return False

    def _set_used(self, i, v):                                 # set_fec_dec_buf_used :566-572
        if self.first <= i < self.second:
            self.slots[i - self.first].bUsed = v

    def _update_window(self, seg_beg, n):                      # update_fec_dec_buf :540-554
        end = _u32(seg_beg + n)
        if end > self.second:
            ns = _i32(end - self.second)
            span = _i32(self.second - self.first)
            for i in range(ns, span):
                self.slots[i - ns].assign(self.slots[i])
                self.slots[i].reset(self.slots[i].MaxBufSize)
            self.first = _u32(self.first + ns)
            self.second = _u32(self.second + ns)

    def _add_packet(self, ipkt, isrc, data, k, n, seg_beg):    # add_packet_fec_buf :485-535
        L = lib()
        if self.first <= ipkt < self.second:
            s = self.slots[ipkt - self.first]
            s.set_packet(data)
            s.iPacket = ipkt
            s.bSourcePkt = _u32(ipkt - seg_beg) < k
            s.i_source_pkt = isrc
        else:
            return False, 0
        valid, all_src, max_size = 0, True, 0
        L.reset_fec_dec_buf(C.byref(self.buf))
        i = 0
        while valid < k and i < n:
            ck = _i32(seg_beg - self.first + i)
            if 0 <= ck < len(self.slots):
                s = self.slots[ck]
                if s.valid() and s.iPacket == _u32(seg_beg + i):
                    L.set_fec_dec_buf(C.byref(self.buf), valid, bytes(s.fec_buf), s.BufSize, i)
                    max_size = s.BufSize if valid == 0 else max(max_size, s.BufSize)
                    valid += 1
                    if ck >= k:          # (sic: the window index, :523)
                        all_src = False
            i += 1
        return valid == k and not all_src, max_size

    def _flush_avail(self, lastis, lastie):                    # flush_avail_pkts :407-443
        L = lib()
        ret = False
        if (lastie > lastis and self.first <= lastis < self.second and self.first < lastie <= self.second):
            for i in range(lastis, lastie):
                s = self.slots[i - self.first]
                if s.valid() and s.bSourcePkt:
                    sz = C.c_uint16(0)
                    fb = C.create_string_buffer(bytes(s.fec_buf), len(s.fec_buf))
                    p = L.dec_src_pkt_info(fb, C.byref(self.buf), C.byref(sz))
                    if not p:
                        continue
                    if not self._used(i):
                        self.fec_src_count += 1
                        self._deliver(p, sz.value, s.i_source_pkt)
                        self._set_used(i, True)
                    s.reset(s.MaxBufSize)
                    ret = True
        return ret

    def unpack_input(self, dgram):                             # zfec_unpack_input :189-371
        L = lib()
        dgram = bytes(dgram)
        size = len(dgram)
        head = FecCodecHead()
        usz = C.c_int(-1)
        pu = L.unpack_fec_head(C.byref(self.buf), C.byref(head), dgram, size, C.byref(usz))
        if usz.value == size - 1 and pu:                       # :201-209 non-FEC datagram
            self._deliver(pu, usz.value, 0)
            return
        if not pu or usz.value < 0:                            # :210-213
            return
        unpacked = C.string_at(pu, usz.value)
        i_recv = head.sent_pkt_index
        src = head.src_pkt_index
        cur_n, cur_k, cur_ni = head.codec_n, head.codec_k, head.ik
        seg_beg = _u32(i_recv - cur_ni)
        self.i_recv_pkt = max(i_recv, self.i_recv_pkt)
        seg_src_beg = _u32(src - cur_ni) if cur_ni < cur_k else _u32(src - cur_k + 1)
        self._update_window(seg_beg, cur_n)
        used = False
        if cur_ni < cur_k:                                     # :238-283 source packet
            sz = C.c_uint16(0)
            p = L.dec_src_pkt_info(pu, C.byref(self.buf), C.byref(sz))
            if not p:
                return
            if not self.is_sorted:
                if not self._used(i_recv):
                    self.fec_src_count += 1
                    self._deliver(p, sz.value, seg_src_beg + cur_ni)
                used = True
            if i_recv == self.i_expected_packet and self.is_sorted:
                self.fec_src_count += 1
                self._deliver(p, sz.value, seg_src_beg + cur_ni)
                used = True
                self.i_expected_packet = _u32(self.i_expected_packet + 1)
                if _cmod(_i32(self.i_expected_packet - seg_beg), cur_n) == cur_k:
                    self.i_expected_packet = _u32(seg_beg + cur_n)
        dec, max_size = self._add_packet(i_recv, src, unpacked, cur_k, cur_n, seg_beg)
        self._set_used(i_recv, used)
        if not dec and _u32(i_recv - self.i_expected_packet) >= 2 * cur_n and self.is_sorted:  # :289-293
            self._flush_avail(self.i_expected_packet, seg_beg)
            self.i_expected_packet = seg_beg
        if not dec:
            return
        if self.is_sorted:                                     # :296-299
            self._flush_avail(self.i_expected_packet, seg_beg)
        codec = self.codecs.find(cur_k, cur_n)                 # :301-305
        if codec is None:
            return
        L.fec_decode_pkts(C.byref(self.buf), codec[2], max_size)
        for i in range(cur_k):                                 # :308-366
            pd = L.get_fec_decoded_pkt(C.byref(self.buf), i)
            if not pd:
                continue
            sz = C.c_uint16(0)
            p = L.dec_src_pkt_info(pd, C.byref(self.buf), C.byref(sz))
            if not p:
                continue
            if not self.is_sorted:
                if not self._used(_u32(seg_beg + i)):
                    self._deliver(p, sz.value, seg_src_beg + i)
                    self._set_used(_u32(seg_beg + i), True)
                    self.fec_src_count += 1
                    self.fec_restore_count += 1
            if _u32(seg_beg + i) >= self.i_expected_packet and self.is_sorted:
                if not self._used(_u32(seg_beg + i)):
                    self._deliver(p, sz.value, seg_src_beg + i)
                    self._set_used(_u32(seg_beg + i), True)
                    self.fec_src_count += 1
                    self.fec_restore_count += 1
                self.i_expected_packet = _u32(seg_beg + i + 1)
                if _cmod(_i32(self.i_expected_packet - seg_beg), cur_n) == cur_k:
                    self.i_expected_packet = _u32(seg_beg + cur_n)
            self._set_used(i_recv, used)
