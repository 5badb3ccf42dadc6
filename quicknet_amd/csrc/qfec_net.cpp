// qfec_net.cpp -- batched NetFecCodec layer (include/qfec_net.h).
//
// Host bookkeeping only: per-session numbering as zfec_pack_input keeps it
// (network/NetFecCodec.cpp:68-175), grouping of received datagrams by (session, first sent
// index) as zfec_unpack_input derives it (:189-251), pinned staging, and one
// qfec_pack_datagrams / qfec_unpack_datagrams launch per flush for all sessions.  Every
// byte of shards, checksums, headers and GF arithmetic is produced by the device kernels.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <deque>
#include <map>
#include <mutex>
#include <set>
#include <tuple>
#include <utility>
#include <vector>

#include "../../include/qfec.h"
#include "../../include/qfec_net.h"

namespace {

size_t round16(size_t x) { return (x + 15) & ~(size_t)15; }

// grow-only device / pinned host buffers
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    bool ensure(size_t bytes) {
        if (bytes <= cap) return true;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = round16(bytes + bytes / 4 + 4096);
        if (hipMalloc(&p, want) != hipSuccess) return false;
        cap = want;
        return true;
    }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
};

struct HostBuf {
    void* p = nullptr;
    size_t cap = 0;
    bool ensure(size_t bytes) {
        if (bytes <= cap) return true;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = round16(bytes + bytes / 4 + 4096);
        if (hipHostMalloc(&p, want, hipHostMallocDefault) != hipSuccess) return false;
        cap = want;
        return true;
    }
    ~HostBuf() {
        if (p) (void)hipHostFree(p);
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
};

struct Session {
    void* peer = nullptr;
    bool enabled = true;                          // enable_zfec (FecTransmission.cpp:72-77)
    uint32_t i_sent_pkt = 0, i_sent_src_pkt = 0;  // init_zfec_layer: both 0 (:623-625)
    std::vector<uint8_t> part;                    // the open group's payloads
    std::vector<int> part_sizes;
};

struct TxGroup {
    int session;
    uint32_t sent0, src0;
};

struct RxGroup {
    int session = 0;
    int k = 0, n = 0;             // the group's code, from its headers (find_codec per header)
    uint32_t sent0 = 0, src0 = 0;
    int have = 0;
    bool ck = true;               // 0xED datagrams
    std::vector<uint8_t> rows;    // [n][wire_pitch]
    std::vector<int> len;         // [n], 0 = not received
};

uint32_t rd32(const uint8_t* p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }

}  // namespace

struct qfec_net {
    int k = 0, n = 0, max_pkt = 0, checksum = 1;
    qfec_code* code = nullptr;
    size_t shard_pitch = 0, wire_pitch = 0;
    std::mutex mu;
    std::vector<Session> sessions;
    // send queue: complete groups, payloads back to back
    std::vector<uint8_t> tx_payload;
    std::vector<long long> tx_offs;
    std::vector<int> tx_sizes;
    std::vector<TxGroup> tx_groups;
    // FEC-off traffic: [0x13][payload] datagrams to send (pack_fec_off_tag, FecCodecBuf.cpp:
    // 237-269), and received non-FEC datagrams minus their tag (unpack_fec_head, :366-372)
    std::vector<std::pair<int, std::vector<uint8_t>>> tx_plain, rx_plain;
    // receive queue
    std::map<std::pair<int, uint32_t>, RxGroup> rx;
    std::map<int, qfec_code*> rx_codes;  // (k << 4 | n) -> code, for groups of another (k, n)
    std::set<std::pair<int, uint32_t>> rx_done;
    std::deque<std::pair<int, uint32_t>> rx_done_fifo;
    long long stats[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // staging
    HostBuf h_in, h_aux, h_out, h_out2;
    DevBuf d_in, d_aux, d_shards, d_wire, d_len, d_small;
};

namespace {

int pick_stream(void* stream, hipStream_t* out) {
    *out = (hipStream_t)stream;
    return QFEC_OK;
}

void remember_done(qfec_net* net, const std::pair<int, uint32_t>& key) {
    net->rx_done.insert(key);
    net->rx_done_fifo.push_back(key);
    while (net->rx_done_fifo.size() > (1u << 16)) {
        net->rx_done.erase(net->rx_done_fifo.front());
        net->rx_done_fifo.pop_front();
    }
}

// the code for (k, n): the handle's own, or one made on first sight of another (k, n) --
// the reference looks the codec up per header (find_codec, NetFecCodec.cpp:301)
qfec_code* rx_code(qfec_net* net, int k, int n) {
    if (k == net->k && n == net->n) return net->code;
    qfec_code*& c = net->rx_codes[k << 4 | n];
    if (!c) c = qfec_code_new(QFEC_VANDERMONDE, k, n - k);  // fec_new(k, n): FecCodec.cpp:84
    return c;
}

// unpack the groups in `keys` (all with the same checksum mode and (k, n)) in one launch
int unpack_batch(qfec_net* net, const std::vector<std::pair<int, uint32_t>>& keys, int ck, int k, int n,
                 qfec_unpack_output_fn out, hipStream_t s) {
    qfec_code* code = rx_code(net, k, n);
    if (!code) return QFEC_ENOMEM;
    const size_t G = keys.size();
    if (!G) return 0;
    const size_t wp = net->wire_pitch, sp = net->shard_pitch;
    const size_t wbytes = G * n * wp, lbytes = G * n * sizeof(int);
    if (!net->h_in.ensure(wbytes + lbytes) || !net->d_wire.ensure(wbytes) || !net->d_len.ensure(lbytes) ||
        !net->d_shards.ensure(G * n * sp) || !net->d_small.ensure(G * n * (1 + 4) + 2 * G * k * 4 + 64) ||
        !net->h_out.ensure(G * k * sp) || !net->h_out2.ensure(G * n + 2 * G * k * 4 + 64))
        return QFEC_ENOMEM;
    uint8_t* hw = net->h_in.as<uint8_t>();
    int* hl = reinterpret_cast<int*>(hw + wbytes);
    for (size_t g = 0; g < G; ++g) {
        const RxGroup& R = net->rx[keys[g]];
        memcpy(hw + g * n * wp, R.rows.data(), (size_t)n * wp);
        memcpy(hl + g * n, R.len.data(), (size_t)n * sizeof(int));
    }
    uint8_t* d_marks = net->d_small.as<uint8_t>();
    int* d_rx = reinterpret_cast<int*>(d_marks + round16(G * n));
    int* d_status = d_rx + G * n;
    int* d_psize = d_status + G * k;
    if (hipMemcpyAsync(net->d_wire.p, hw, wbytes, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(net->d_len.p, hl, lbytes, hipMemcpyHostToDevice, s) != hipSuccess)
        return QFEC_EHIP;
    int rc = qfec_unpack_datagrams(code, net->d_wire.as<unsigned char>(), (long long)wp, net->d_len.as<int>(),
                                   (long long)G, ck, net->max_pkt + 20 /* getPackedPktSize, FecCodecBuf.cpp:16-25 */,
                                   net->d_shards.as<unsigned char>(), (long long)sp, d_marks, d_rx, d_status, d_psize,
                                   s);
    if (rc) return rc;
    uint8_t* h_rows = net->h_out.as<uint8_t>();
    uint8_t* h_marks = net->h_out2.as<uint8_t>();
    int* h_status = reinterpret_cast<int*>(h_marks + round16(G * n));
    int* h_psize = h_status + G * k;
    // data rows only: the first k rows of each group
    if (hipMemcpy2DAsync(h_rows, (size_t)k * sp, net->d_shards.p, (size_t)n * sp, (size_t)k * sp, G,
                         hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(h_marks, d_marks, G * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(h_status, d_status, G * k * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(h_psize, d_psize, G * k * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return QFEC_EHIP;
    int delivered = 0;
    for (size_t g = 0; g < G; ++g) {
        const RxGroup& R = net->rx[keys[g]];
        void* peer = net->sessions[R.session].peer;
        bool lost_group = false;
        for (int i = 0; i < k; ++i) {
            const int st = h_status[g * k + i];
            if (st == -2) lost_group = true;
            if (st < 0) continue;
            // marks are in rs.c layout: data marks of all groups first
            if (h_marks[g * k + i]) net->stats[4]++;
            if (out)
                out(peer, reinterpret_cast<const char*>(h_rows + (g * k + i) * sp + st), (unsigned)h_psize[g * k + i],
                    R.src0 + (uint32_t)i);
            ++delivered;
        }
        if (lost_group) net->stats[5]++;
    }
    net->stats[2] += (long long)G;
    net->stats[3] += delivered;
    return delivered;
}

}  // namespace

extern "C" {

qfec_net* qfec_net_new(int k, int n, int max_pkt_size, int checksum) {
    if (k < 1 || n <= k || n > 15 || max_pkt_size < 1 || max_pkt_size > 65535 || (checksum != 0 && checksum != 1))
        return nullptr;
    qfec_code* code = qfec_code_new(QFEC_VANDERMONDE, k, n - k);  // fec_new(k, n): FecCodec.cpp:84
    if (!code) return nullptr;
    qfec_net* net = new qfec_net();
    net->k = k;
    net->n = n;
    net->max_pkt = max_pkt_size;
    net->checksum = checksum;
    net->code = code;
    net->shard_pitch = round16((size_t)max_pkt_size + 4);
    net->wire_pitch = round16(net->shard_pitch + 13);
    return net;
}

void qfec_net_free(qfec_net* net) {
    if (!net) return;
    qfec_code_free(net->code);
    for (auto& kv : net->rx_codes) qfec_code_free(kv.second);
    delete net;
}

int qfec_net_session(qfec_net* net, void* peer) {
    if (!net) return QFEC_EINVAL;
    std::lock_guard<std::mutex> lk(net->mu);
    net->sessions.emplace_back();
    net->sessions.back().peer = peer;
    return (int)net->sessions.size() - 1;
}

int qfec_net_enable(qfec_net* net, int session, int on) {
    if (!net) return QFEC_EINVAL;
    std::lock_guard<std::mutex> lk(net->mu);
    if (session < 0 || session >= (int)net->sessions.size()) return QFEC_EINVAL;
    net->sessions[session].enabled = on != 0;
    return QFEC_OK;
}

int qfec_net_pack_input(qfec_net* net, int session, const void* data, unsigned int size) {
    if (!net || (!data && size)) return QFEC_EINVAL;
    std::lock_guard<std::mutex> lk(net->mu);
    if (session < 0 || session >= (int)net->sessions.size() || size > (unsigned)net->max_pkt) return QFEC_EINVAL;
    Session& S = net->sessions[session];
    const uint8_t* p = static_cast<const uint8_t*>(data);
    if (!S.enabled) {  // zfec_pack_input with FEC off (NetFecCodec.cpp:75-94): numbering unchanged
        std::vector<uint8_t> d(1 + (size_t)size, 0x13);  // tagFecOFFTag
        if (size) memcpy(d.data() + 1, p, size);
        net->tx_plain.emplace_back(session, std::move(d));
        return QFEC_OK;
    }
    S.part.insert(S.part.end(), p, p + size);
    S.part_sizes.push_back((int)size);
    if ((int)S.part_sizes.size() < net->k) return QFEC_OK;
    // the group is complete: sent indices i_sent_pkt .. + n - 1, sources i_sent_src_pkt ..
    // + k - 1 (zfec_pack_input numbering, NetFecCodec.cpp:98-171)
    net->tx_groups.push_back(TxGroup{session, S.i_sent_pkt, S.i_sent_src_pkt});
    long long off = (long long)net->tx_payload.size();
    for (int sz : S.part_sizes) {
        net->tx_offs.push_back(off);
        net->tx_sizes.push_back(sz);
        off += sz;
    }
    net->tx_payload.insert(net->tx_payload.end(), S.part.begin(), S.part.end());
    S.part.clear();
    S.part_sizes.clear();
    S.i_sent_pkt += (uint32_t)net->n;
    S.i_sent_src_pkt += (uint32_t)net->k;
    return QFEC_OK;
}

int qfec_net_flush_pack(qfec_net* net, qfec_pack_output_fn out, void* stream) {
    if (!net) return QFEC_EINVAL;
    std::lock_guard<std::mutex> lk(net->mu);
    // FEC-off datagrams first, in queue order (no device work)
    int plain = 0;
    for (auto& pd : net->tx_plain) {
        if (out) out(net->sessions[pd.first].peer, reinterpret_cast<const char*>(pd.second.data()),
                     (unsigned)pd.second.size());
        ++plain;
    }
    net->tx_plain.clear();
    net->stats[1] += plain;
    const size_t G = net->tx_groups.size();
    if (!G) return plain;
    if (qfec_device_count() <= 0) return QFEC_ENODEV;
    const int k = net->k, n = net->n;
    hipStream_t s;
    pick_stream(stream, &s);
    const size_t pbytes = round16(net->tx_payload.size() + 16);
    const size_t obytes = G * k * sizeof(long long), zbytes = G * k * sizeof(int), qbytes = G * 2 * sizeof(uint32_t);
    const size_t wp = net->wire_pitch, sp = net->shard_pitch;
    if (!net->h_in.ensure(pbytes) || !net->h_aux.ensure(obytes + zbytes + qbytes) || !net->d_in.ensure(pbytes) ||
        !net->d_aux.ensure(obytes + zbytes + qbytes) || !net->d_shards.ensure(G * n * sp) ||
        !net->d_wire.ensure(G * n * wp) || !net->d_len.ensure(G * n * sizeof(int)) ||
        !net->h_out.ensure(G * n * wp) || !net->h_out2.ensure(G * n * sizeof(int)))
        return QFEC_ENOMEM;
    memcpy(net->h_in.p, net->tx_payload.data(), net->tx_payload.size());
    memset(net->h_in.as<uint8_t>() + net->tx_payload.size(), 0, pbytes - net->tx_payload.size());
    uint8_t* ha = net->h_aux.as<uint8_t>();
    memcpy(ha, net->tx_offs.data(), obytes);
    memcpy(ha + obytes, net->tx_sizes.data(), zbytes);
    uint32_t* hq = reinterpret_cast<uint32_t*>(ha + obytes + zbytes);
    for (size_t g = 0; g < G; ++g) {
        hq[2 * g] = net->tx_groups[g].sent0;
        hq[2 * g + 1] = net->tx_groups[g].src0;
    }
    uint8_t* da = net->d_aux.as<uint8_t>();
    if (hipMemcpyAsync(net->d_in.p, net->h_in.p, pbytes, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(da, ha, obytes + zbytes + qbytes, hipMemcpyHostToDevice, s) != hipSuccess)
        return QFEC_EHIP;
    int rc = qfec_pack_datagrams(net->code, net->d_in.as<unsigned char>(), reinterpret_cast<const long long*>(da),
                                 reinterpret_cast<const int*>(da + obytes),
                                 reinterpret_cast<const unsigned int*>(da + obytes + zbytes), (long long)G,
                                 net->checksum, net->d_shards.as<unsigned char>(), (long long)sp,
                                 net->d_wire.as<unsigned char>(), (long long)wp, net->d_len.as<int>(), s);
    if (rc) return rc;
    uint8_t* hw = net->h_out.as<uint8_t>();
    int* hl = net->h_out2.as<int>();
    if (hipMemcpyAsync(hw, net->d_wire.p, G * n * wp, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(hl, net->d_len.p, G * n * sizeof(int), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return QFEC_EHIP;
    int emitted = 0;
    for (size_t g = 0; g < G; ++g) {
        void* peer = net->sessions[net->tx_groups[g].session].peer;
        for (int j = 0; j < n; ++j) {
            const int len = hl[g * n + j];
            if (len <= 0) continue;
            if (out) out(peer, reinterpret_cast<const char*>(hw + (g * n + j) * wp), (unsigned)len);
            ++emitted;
        }
    }
    net->stats[0] += (long long)G;
    net->stats[1] += emitted;
    net->tx_groups.clear();
    net->tx_payload.clear();
    net->tx_offs.clear();
    net->tx_sizes.clear();
    return plain + emitted;
}

int qfec_net_unpack_input(qfec_net* net, int session, const char* datagram, unsigned int size) {
    if (!net || (!datagram && size)) return QFEC_EINVAL;
    std::lock_guard<std::mutex> lk(net->mu);
    if (session < 0 || session >= (int)net->sessions.size()) return QFEC_EINVAL;
    const uint8_t* d = reinterpret_cast<const uint8_t*>(datagram);
    // header fields only (unpack_fec_head, FecCodecBuf.cpp:334-411); every validity and
    // checksum test is the device's
    if (size == 0) {
        net->stats[6]++;
        return 0;
    }
    if (size < 11 || (d[0] != 0xEC && d[0] != 0xED)) {
        // not an FEC datagram (FEC off at the sender, tag 0x13, or too short): handed over
        // as it is minus the tag byte, source index 0 (zfec_unpack_input, :200-209)
        net->rx_plain.emplace_back(session, std::vector<uint8_t>(d + 1, d + size));
        return 1;
    }
    if (size > net->wire_pitch) {  // longer than this handle's datagrams can be
        net->stats[6]++;
        return 0;
    }
    const uint32_t sent = rd32(d + 1), src = rd32(d + 5);
    const uint32_t ikn = (uint32_t)d[9] | (uint32_t)d[10] << 8;
    const int hn = (int)(ikn & 0xF), hk = (int)((ikn >> 4) & 0xF), ik = (int)((ikn >> 8) & 0xF);
    if (hk < 1 || hk >= hn || ik >= hn) {  // no codec can be made for it
        net->stats[6]++;
        return 0;
    }
    // group identity: its first sent index (iPktCurSegBeg = i_recv_pkt - cur_ni, :222) and its
    // first source index (iPktCurSegSrcBeg, :226-234)
    const uint32_t sent0 = sent - (uint32_t)ik;
    const uint32_t src0 = ik < hk ? src - (uint32_t)ik : src - (uint32_t)hk + 1u;
    const std::pair<int, uint32_t> key(session, sent0);
    if (net->rx_done.count(key)) {
        net->stats[7]++;
        return 0;
    }
    RxGroup& R = net->rx[key];
    if (R.len.empty()) {
        R.session = session;
        R.k = hk;
        R.n = hn;
        R.sent0 = sent0;
        R.src0 = src0;
        R.ck = d[0] == 0xED;
        R.rows.assign((size_t)hn * net->wire_pitch, 0);
        R.len.assign((size_t)hn, 0);
    } else if (R.k != hk || R.n != hn) {  // the group's other datagrams say another code
        net->stats[6]++;
        return 0;
    }
    if (R.len[ik]) return 0;  // duplicate
    memcpy(R.rows.data() + (size_t)ik * net->wire_pitch, d, size);
    R.len[ik] = (int)size;
    R.have++;
    return 1;
}

int qfec_net_flush_unpack(qfec_net* net, qfec_unpack_output_fn out, int all, void* stream) {
    if (!net) return QFEC_EINVAL;
    std::lock_guard<std::mutex> lk(net->mu);
    hipStream_t s;
    pick_stream(stream, &s);
    // non-FEC datagrams first, in arrival order (no device work)
    int delivered = 0;
    for (auto& pd : net->rx_plain) {
        if (out) out(net->sessions[pd.first].peer, reinterpret_cast<const char*>(pd.second.data()),
                     (unsigned)pd.second.size(), 0u);
        ++delivered;
    }
    net->rx_plain.clear();
    net->stats[3] += delivered;
    // groups: one launch per (checksum mode, k, n)
    std::map<std::tuple<int, int, int>, std::vector<std::pair<int, uint32_t>>> batches;
    for (auto& kv : net->rx)
        if (all || kv.second.have >= kv.second.k)
            batches[std::make_tuple(kv.second.ck ? 1 : 0, kv.second.k, kv.second.n)].push_back(kv.first);
    if (!batches.empty() && qfec_device_count() <= 0) return QFEC_ENODEV;
    for (auto& b : batches) {
        const int rc = unpack_batch(net, b.second, std::get<0>(b.first), std::get<1>(b.first), std::get<2>(b.first),
                                    out, s);
        if (rc < 0) return rc;
        delivered += rc;
        for (auto& key : b.second) {
            net->rx.erase(key);
            remember_done(net, key);
        }
    }
    return delivered;
}

int qfec_net_stats(const qfec_net* net, long long* out8) {
    if (!net || !out8) return QFEC_EINVAL;
    for (int i = 0; i < 8; ++i) out8[i] = net->stats[i];
    return QFEC_OK;
}

}  // extern "C"
