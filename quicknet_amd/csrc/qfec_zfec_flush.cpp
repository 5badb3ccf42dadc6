// qfec_zfec_flush.cpp -- qfec_zfec_flush (include/qfec_zfec.h): every session's queued calls run
// through host restatements of NetFecCodec.cpp's zfec_pack_input / zfec_unpack_input state
// machines, all byte work in batched device launches (design: qfec_zfec.cpp).
#include "qfec_zfec_impl.hpp"

using namespace qfec_zfec_impl;

namespace {
// QFEC_ZFEC_TIMING=1: phase times of each flush on stderr (profiling aid)
const bool g_zfec_timing = getenv("QFEC_ZFEC_TIMING") != nullptr;
thread_local std::chrono::steady_clock::time_point t_zfec_phase;

int flush_body(qfec_zfec* z, qfec_pack_output_fn pack_out, qfec_unpack_output_fn unpack_out, void* stream) {
    const bool timing = g_zfec_timing;
    auto& t_prev = t_zfec_phase;
    t_prev = std::chrono::steady_clock::now();
    auto phase = [&](const char* name) {
        if (!timing) return;
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "[qfec] zfec flush %-12s %8.3f ms\n", name, std::chrono::duration<double, std::milli>(t - t_prev).count());
        t_prev = t;
    };
    hipStream_t st = (hipStream_t)stream;
    auto tsync = [&](const char* name) {  // timing only: attribute the stream's work to its phase
        if (!timing) return;
        (void)hipStreamSynchronize(st);
        phase(name);
    };
    const size_t NS = z->sessions.size();
    HostArena& RXA = z->rx[z->rxc];
    HostArena& TXA = z->tx[z->txc];
    std::vector<std::vector<Emit>> tx_out(NS), rx_out(NS);
    std::vector<std::vector<uint8_t>> own(NS);
    size_t n_ops = 0;
    for (auto& S : z->sessions) n_ops += S.ops.size();
    const unsigned threads = flush_threads(n_ops, NS);
    int rc = 0;
    // the arenas' bytes start for the device now, so the copies run while the machines do
    // (a context with no device -- FEC-off sessions only -- skips this; whatever needs the
    // device later fails there)
    bool tx_staged = false, rx_staged = false;
    {
        bool any_pack = false, any_unpack = false;
        for (auto& S : z->sessions)
            for (auto& op : S.ops) {
                any_pack |= op.t == OP_PACK;
                any_unpack |= op.t == OP_UNPACK;
            }
        if (any_pack && TXA.used && z->d_tx.ensure(TXA.used + 16) == QFEC_OK)
            tx_staged = hipMemcpyAsync(z->d_tx.d, TXA.h, TXA.used + 16, hipMemcpyHostToDevice, st) == hipSuccess;
        // (copying the arena to the device while the input calls still fill it, 16 MiB at a time,
        // moved the time into the input calls instead: slower overall, profiles/r05l)
        if (any_unpack && RXA.used && z->d_rx.ensure(RXA.used + 16) == QFEC_OK)
            rx_staged = hipMemcpyAsync(z->d_rx.d, RXA.h, RXA.used + 16, hipMemcpyHostToDevice, st) == hipSuccess;
        (void)hipGetLastError();
    }
    // ---- send: the machines (threaded over sessions), then their groups merged per (k, n)
    std::vector<std::vector<LocalGroup>> lgroups(NS);
    parallel_for(z, NS, threads, [&](size_t si) {  // (local vectors: see the receive machines)
        std::vector<Emit> out;
        std::vector<LocalGroup> groups;
        std::vector<uint8_t> own_b;
        tx_machine(z->sessions[si], out, groups, own_b, TXA.h);
        out.swap(tx_out[si]);
        groups.swap(lgroups[si]);
        own_b.swap(own[si]);
    });
    std::vector<PackBatch> packs;
    std::map<std::pair<int, int>, int> pack_of;  // (k, n) -> index in packs
    z->io.used = 0;
    for (size_t si = 0; si < NS; ++si) {
        std::vector<std::pair<int, long long>> place(lgroups[si].size());
        for (size_t i = 0; i < lgroups[si].size(); ++i) {
            const LocalGroup& lg = lgroups[si][i];
            auto it = pack_of.find(std::make_pair(lg.k, lg.n));
            int bi;
            if (it == pack_of.end()) {
                PackBatch b;
                b.k = lg.k;
                b.n = lg.n;
                packs.push_back(std::move(b));
                bi = (int)packs.size() - 1;
                pack_of.emplace(std::make_pair(lg.k, lg.n), bi);
            } else {
                bi = it->second;
            }
            place[i] = std::make_pair(bi, (long long)packs[(size_t)bi].groups.size());
            packs[(size_t)bi].groups.push_back(lg.g);
        }
        for (auto& e : tx_out[si])
            if (e.kind == 0) {
                e.batch = place[(size_t)e.group].first;
                e.group = place[(size_t)e.group].second;
            }
    }
    phase("tx machine");
    if (!packs.empty()) {
        // the send arena to the device in one copy; per batch: offsets / sizes / seq in, the
        // datagrams and their lengths out, all through the pinned io arena
        Stage io, work;
        for (auto& b : packs) {
            const size_t G = b.groups.size();
            size_t maxp = 1;
            for (auto& g : b.groups)
                for (int i = 0; i < b.k; ++i) maxp = std::max(maxp, (size_t)g.pay[i].len);
            b.sp = round16(maxp + 4);
            b.wp = (b.sp + 13 + 63) & ~(size_t)63;  // the 64-B multiple: the fused send writes whole lines
            b.o_offs = io.take(G * b.k * 8);
            b.o_sizes = io.take(G * b.k * 4);
            b.o_seq = io.take(G * 8);
            b.o_wlen = io.take(G * b.n * 4);
            b.o_wire = io.take(G * b.n * b.wp);
            b.d_shards = work.take(G * b.n * b.sp);
        }
        z->io.used = 0;
        if (!z->io.reserve(io.o + 16) || (rc = z->d_io.ensure(io.o + 16)) || (rc = z->d_work.ensure(work.o + 16)))
            return rc ? rc : QFEC_ENOMEM;
        if (!tx_staged) {
            if ((rc = z->d_tx.ensure(TXA.used + 16))) return rc;
            if (hipMemcpyAsync(z->d_tx.d, TXA.h, TXA.used + 16, hipMemcpyHostToDevice, st) != hipSuccess)
                return QFEC_EHIP;
        }
        tsync("pack h2d");
        uint8_t* h = z->io.h;
        uint8_t* d = z->d_io.d;
        // QFEC_ZFEC_TX_ZC=1 (A/B): the kernels write the datagrams straight into the pinned io
        // arena over PCIe instead of HBM + one copy back
        static const bool tx_zc = getenv("QFEC_ZFEC_TX_ZC") && atoi(getenv("QFEC_ZFEC_TX_ZC")) == 1;
        const bool zc = tx_zc && z->io.pinned && !z->io.mapped;  // (a registered block's device address differs)
        for (auto& b : packs) {
            const size_t G = b.groups.size();
            long long* offs = reinterpret_cast<long long*>(h + b.o_offs);
            int* sizes = reinterpret_cast<int*>(h + b.o_sizes);
            uint32_t* seq = reinterpret_cast<uint32_t*>(h + b.o_seq);
            for (size_t g = 0; g < G; ++g) {
                seq[2 * g] = b.groups[g].sent0;
                seq[2 * g + 1] = b.groups[g].src0;
                for (int i = 0; i < b.k; ++i) {
                    const View& p = b.groups[g].pay[i];
                    offs[g * b.k + i] = (long long)p.off;
                    sizes[g * b.k + i] = (int)p.len;
                }
            }
            if (hipMemcpyAsync(d + b.o_offs, h + b.o_offs, b.o_wlen - b.o_offs, hipMemcpyHostToDevice, st) != hipSuccess)
                return QFEC_EHIP;
            uint8_t* out = zc ? h : d;
            if ((rc = qfec_pack_datagrams(code_for(z, b.k, b.n), z->d_tx.d, reinterpret_cast<const long long*>(d + b.o_offs),
                                          reinterpret_cast<const int*>(d + b.o_sizes),
                                          reinterpret_cast<const unsigned int*>(d + b.o_seq), (long long)G,
                                          1 /* is_send_checksum */, z->d_work.d + b.d_shards, (long long)b.sp,
                                          out + b.o_wire, (long long)b.wp, reinterpret_cast<int*>(out + b.o_wlen), st)))
                return rc;
        }
        tsync("pack kernels");
        if (!zc)
            for (auto& b : packs) {
                const size_t G = b.groups.size();
                if (hipMemcpyAsync(h + b.o_wlen, d + b.o_wlen, b.o_wire + G * b.n * b.wp - b.o_wlen, hipMemcpyDeviceToHost,
                                   st) != hipSuccess)
                    return QFEC_EHIP;
            }
        z->io.used = io.o;  // the datagrams stay until the callbacks (the receive stages go after)
        if (hipStreamSynchronize(st) != hipSuccess) return QFEC_EHIP;
    }
    phase("pack launch");
    // ---- receive: verdicts of this flush's FEC datagrams (pseudo-groups by (k, n, tag, dec_pkt_size))
    std::vector<std::vector<Verdict>> verd(NS);
    std::vector<UnpackBatch> vb;
    using Key = std::tuple<int, int, int, int>;
    struct Local {
        Key key;
        int groups = 0;
        size_t need = 0;
        std::vector<UnpackRow> rows;
        std::vector<uint16_t> taken;  // per group: bit ik
    };
    std::vector<std::vector<Local>> loc;  // (the batches visit their rows in place: kept to the verdicts)
    {
        // per session (on the session threads): its rows placed into pseudo-groups of its own
        // batches; then the sessions' batches are concatenated per key in session order (any
        // placement is valid: a row's verdict is its own)
        loc.assign(NS, {});
        parallel_for(z, NS, threads, [&](size_t si) {
            Session& S = z->sessions[si];
            std::vector<Local> L;  // (local vectors: see the receive machines)
            std::vector<Verdict> V;
            V.reserve(S.ops.size());
            int dps = S.rx.dec_pkt_size;  // its growth over the queue (unpack_fec_head realloc)
            int last = -1;
            for (auto& op : S.ops) {
                if (op.t != OP_UNPACK) continue;
                Verdict v;
                const size_t size = op.size;
                if ((int)size > dps) dps = (int)size;
                v.fec = size >= 11 && (op.a == 0xEC || op.a == 0xED);
                if (v.fec) {
                    const uint32_t ikn = op_ikn(op);
                    const int n = (int)(ikn & 0xF), k = (int)((ikn >> 4) & 0xF), ik = (int)((ikn >> 8) & 0xF);
                    v.usable = k >= 1 && k < n && n <= 15 && ik < n;
                    if (v.usable) {
                        const int cs = op.a == 0xED ? 1 : 0;
                        const Key key = std::make_tuple(k, n, cs, dps);
                        if (last < 0 || L[(size_t)last].key != key) {
                            last = -1;
                            for (size_t x = 0; x < L.size(); ++x)
                                if (L[x].key == key) last = (int)x;
                            if (last < 0) {
                                L.emplace_back();
                                L.back().key = key;
                                L.back().rows.reserve(S.ops.size());
                                last = (int)L.size() - 1;
                            }
                        }
                        Local& b = L[(size_t)last];
                        int g = -1;
                        for (size_t gi = b.taken.size() > 8 ? b.taken.size() - 8 : 0; gi < b.taken.size(); ++gi)
                            if (!((b.taken[gi] >> ik) & 1u)) {
                                g = (int)gi;
                                break;
                            }
                        if (g < 0) {
                            b.taken.push_back(0);
                            g = b.groups++;
                        }
                        b.taken[(size_t)g] |= (uint16_t)(1u << ik);
                        b.rows.push_back(UnpackRow{g, ik, op.off, (uint32_t)size});
                        // the row bytes dec_src_pkt_info may read: head + the shard's size field
                        const size_t hdr = cs ? 13 : 11;
                        if (ik < k && size >= hdr + 2) b.need = std::max(b.need, (size_t)(cs ? 4 : 2) + op_szf(op));
                        v.batch = last;  // local until the merge
                        v.group = g;
                        v.ik = ik;
                    }
                }
                V.push_back(v);
            }
            V.swap(verd[si]);
            L.swap(loc[si]);
        });
        std::map<Key, int> vb_of;
        std::vector<std::vector<std::pair<int, int>>> where_s(NS);  // local batch -> (batch, group offset)
        for (size_t si = 0; si < NS; ++si) {
            auto& where = where_s[si];
            where.assign(loc[si].size(), std::make_pair(0, 0));
            for (size_t x = 0; x < loc[si].size(); ++x) {
                Local& lb = loc[si][x];
                auto it = vb_of.find(lb.key);
                int bi;
                if (it == vb_of.end()) {
                    UnpackBatch b;
                    b.k = std::get<0>(lb.key);
                    b.n = std::get<1>(lb.key);
                    b.checksum = std::get<2>(lb.key);
                    b.dec_pkt_size = std::get<3>(lb.key);
                    vb.push_back(std::move(b));
                    bi = (int)vb.size() - 1;
                    vb_of.emplace(lb.key, bi);
                } else {
                    bi = it->second;
                }
                UnpackBatch& b = vb[(size_t)bi];
                const int goff = b.groups;
                where[x] = std::make_pair(bi, goff);
                b.groups += lb.groups;
                b.need = std::max(b.need, lb.need);
                b.segs.emplace_back(&lb.rows, goff);
            }
        }
        parallel_for(z, NS, threads, [&](size_t si) {
            const auto& where = where_s[si];
            for (auto& v : verd[si])
                if (v.batch >= 0) {
                    v.group += where[(size_t)v.batch].second;
                    v.batch = where[(size_t)v.batch].first;
                }
        });
    }
    phase("rx grouping");
    // the receive arena's bytes on the device once: verdict and decode launches gather from it
    if (!vb.empty() && !rx_staged) {
        if ((rc = z->d_rx.ensure(RXA.used + 16))) return rc;
        if (hipMemcpyAsync(z->d_rx.d, RXA.h, RXA.used + 16, hipMemcpyHostToDevice, st) != hipSuccess) return QFEC_EHIP;
    }
    tsync("rx h2d");
    if (!vb.empty()) {
        Stage io{round16(z->io.used)}, work;
        for (auto& b : vb) unpack_layout(b, io, work);
        if (!z->io.reserve(io.o + 16) || (rc = z->d_io.ensure(io.o + 16)) || (rc = z->d_work.ensure(work.o + 16)))
            return rc ? rc : QFEC_ENOMEM;
        for (auto& b : vb)
            if ((rc = run_unpack(z, b, z->d_rx.d, st))) return rc;
        if (hipStreamSynchronize(st) != hipSuccess) return QFEC_EHIP;
    }
    parallel_for(z, NS, threads, [&](size_t si) {
        size_t v = 0;
        for (auto& op : z->sessions[si].ops) {
            if (op.t != OP_UNPACK) continue;
            Verdict& vd = verd[si][v++];
            if (vd.group < 0) continue;
            const UnpackBatch& b = vb[(size_t)vd.batch];
            const size_t row = (size_t)vd.group * b.n + vd.ik;
            const uint32_t hdr = op.a == 0xED ? 13 : 11;
            vd.ok = b.rx[row] >= 0;
            if (vd.ok) vd.shard = View{SRC_RX, op.off + hdr, op.size - hdr};
            if (vd.ik < b.k && vd.ok) {
                const int stt = b.status[(size_t)vd.group * b.k + vd.ik];
                vd.src_ok = stt >= 0;
                vd.src_size = b.psize[(size_t)vd.group * b.k + vd.ik];
                // a received row's payload is the datagram's own bytes
                if (vd.src_ok) vd.payload = View{SRC_RX, op.off + hdr + (uint32_t)stt, (uint32_t)vd.src_size};
            }
        }
    });
    phase("verdicts");
    // ---- the receive machines.  A pass that meets a decode without a device result assumes
    // every row of it decoded and passed (the common case) and leaves placeholders for its
    // deliveries; after the launches the placeholders are filled when that held for every such
    // decode, and otherwise the machines are replayed from the flush's starting state.
    std::vector<DecodeCache> caches(NS);  // per session (keys name their session)
    std::vector<RxState> start(NS);
    for (size_t si = 0; si < NS; ++si) start[si] = z->sessions[si].rx;
    std::vector<uint8_t> dec_bytes;  // decoded payloads that are not views of an input shard
    dec_bytes.reserve((size_t)4 << 20);
    std::vector<const DecodeReq*> missing;  // this pass's requests (in the sessions' miss_s)
    std::vector<std::vector<DecodeReq>> miss_s(NS);
    for (int pass_no = 0;; ++pass_no) {
        missing.clear();
        parallel_for(z, NS, threads, [&](size_t si) {  // sessions are independent
            Session& S = z->sessions[si];
            if (pass_no) S.rx = start[si];
            // thread-local vectors, swapped in at the end: the per-session vector headers lie
            // side by side, and a push_back on each would bounce their cache lines between threads
            std::vector<Emit> out;
            out.swap(rx_out[si]);
            out.clear();
            std::vector<DecodeReq> miss;
            DecodeCache& cache = caches[si];
            RxPass pass{&cache, &miss};
            RxMachine m(S, (int)si, verd[si], pass, out);
            m.run();
            // this session's new keys enter its cache (node addresses survive rehashing)
            cache.reserve(cache.size() + miss.size());
            for (auto& q : miss) {
                auto ins = cache.emplace(q.key, DecodeOut{});
                q.out = &ins.first->second;
                q.fresh = ins.second;
            }
            out.swap(rx_out[si]);
            miss.swap(miss_s[si]);
        });
        // the requests numbered in session order, as one thread would have numbered them
        for (size_t si = 0; si < NS; ++si) {
            const int base = (int)missing.size();
            if (base)
                for (auto& e : rx_out[si])
                    if (e.kind == 3) e.batch += base;
            for (auto& q : miss_s[si]) missing.push_back(&q);
        }
        phase("rx machine");
        if (missing.empty()) break;
        // one launch per (k, n, mode, dec_pkt_size): each decode is a group holding exactly its k
        // shards, an 0xEC header synthesized in front of each (no shard checksum to re-check).
        // Round 0 decodes at the shards' own length; a row whose size field reaches past that
        // pitch (only a corrupt one can) is decoded again at dec_pkt_size + 4 in round 1, as the
        // reference reads it.
        std::vector<const DecodeReq*> todo;
        for (const DecodeReq* q : missing)
            if (q->fresh) todo.push_back(q);
        phase("decode dedup");
        for (int round = 0; round < 2 && !todo.empty(); ++round) {
            std::vector<UnpackBatch> db;
            std::map<std::tuple<int, int, int, int>, int> db_of;
            std::vector<std::vector<const DecodeReq*>> reqs;
            for (const DecodeReq* q : todo) {
                const auto key = std::make_tuple(q->key.k, q->key.n, q->key.mode, q->key.dec_pkt_size);
                auto it = db_of.find(key);
                int bi;
                if (it == db_of.end()) {
                    UnpackBatch b;
                    b.k = q->key.k;
                    b.n = q->key.n;
                    b.checksum = q->key.mode;
                    b.dec_pkt_size = q->key.dec_pkt_size;
                    b.want_shards = true;
                    b.wrap = 1;
                    b.need = round ? (size_t)b.dec_pkt_size + 4 : 0;
                    db.push_back(std::move(b));
                    reqs.emplace_back();
                    bi = (int)db.size() - 1;
                    db_of.emplace(key, bi);
                } else {
                    bi = it->second;
                }
                UnpackBatch& b = db[(size_t)bi];
                const int g = b.groups++;
                uint32_t have = 0;
                for (int r = 0; r < q->nsh; ++r) {
                    b.rows.push_back(UnpackRow{g, (int)q->key.ik[r], q->shard[r].off, q->shard[r].len});
                    have |= 1u << q->key.ik[r];
                }
                for (int i = 0; i < b.k; ++i)  // the rebuilt rows come back; inputs are views
                    if (!((have >> i) & 1u)) b.fetch.push_back((uint32_t)(g * b.n + i));
                reqs[(size_t)bi].push_back(q);
            }
            Stage io{round16(z->io.used)}, work;
            for (auto& b : db) unpack_layout(b, io, work);
            if (!z->io.reserve(io.o + 16) || (rc = z->d_io.ensure(io.o + 16)) || (rc = z->d_work.ensure(work.o + 16)))
                return rc ? rc : QFEC_ENOMEM;
            phase("decode plan");
            for (auto& b : db)
                if ((rc = run_unpack(z, b, z->d_rx.d, st))) return rc;
            if (hipStreamSynchronize(st) != hipSuccess) return QFEC_EHIP;
            phase("decode launch");
            std::vector<const DecodeReq*> again;
            for (size_t bi = 0; bi < db.size(); ++bi) {
                const UnpackBatch& b = db[bi];
                const auto& rq = reqs[bi];
                const int head = b.checksum ? 4 : 2;
                std::vector<int> fidx((size_t)b.groups * b.n, -1);  // row -> its fetched copy
                for (size_t f = 0; f < b.fetch.size(); ++f) fidx[b.fetch[f]] = (int)f;
                // A decode's input rows come back unchanged (zero past their shard), so a
                // delivered payload that lies inside its input shard is a view of that shard;
                // only the rebuilt rows (and payloads reaching past an input's shard) are copied
                // into the flush's decoded bytes.
                for (size_t g = 0; g < rq.size(); ++g) {
                    bool cut = false;
                    DecodeOut& o = *rq[g]->out;
                    const View* src_of[16] = {};
                    for (int r = 0; r < rq[g]->nsh; ++r)
                        if (rq[g]->key.ik[r] < b.k) src_of[rq[g]->key.ik[r]] = &rq[g]->shard[r];
                    for (int i = 0; i < b.k; ++i) {
                        const int stt = b.status[g * b.k + i], ps = b.psize[g * b.k + i];
                        cut |= stt == -1 && ps < b.dec_pkt_size && (size_t)(head + ps) > b.sp;
                        o.ok[i] = stt >= 0;
                        o.payload[i] = View{};
                        if (stt < 0) continue;
                        const View* in = src_of[i];
                        if (in && (size_t)stt + (size_t)ps <= in->len) {
                            o.payload[i] = View{SRC_RX, in->off + (uint32_t)stt, (uint32_t)ps};
                        } else {
                            o.payload[i] = View{SRC_DEC, (uint32_t)dec_bytes.size(), (uint32_t)ps};
                            const int fi = fidx[g * b.n + (size_t)i];
                            if (fi >= 0) {  // the rebuilt row where it came back (the io arena keeps it)
                                o.payload[i] = View{SRC_IO, (uint32_t)(b.o_hsh + (size_t)fi * b.sp + (size_t)stt), (uint32_t)ps};
                            } else {  // an input whose size field reaches past its shard (corrupt): rare
                                const size_t at = dec_bytes.size();
                                dec_bytes.resize(at + (size_t)ps);
                                if (ps && (hipMemcpyAsync(dec_bytes.data() + at,
                                                          z->d_work.d + b.w_sh + (g * b.n + (size_t)i) * b.sp + (size_t)stt,
                                                          (size_t)ps, hipMemcpyDeviceToHost, st) != hipSuccess ||
                                           hipStreamSynchronize(st) != hipSuccess))
                                    return QFEC_EHIP;
                            }
                        }
                    }
                    if (cut && round == 0) again.push_back(rq[g]);
                }
            }
            z->io.used = io.o;  // this round's rebuilt rows stay until the callbacks
            todo.swap(again);
        }
        phase("decode results");
        bool all_ok = true;
        for (const DecodeReq* q : missing) {
            const DecodeOut& o = *q->out;
            for (int i = 0; i < q->key.k; ++i) all_ok &= o.ok[i];
        }
        if (!all_ok) continue;  // replay with the results
        for (size_t si = 0; si < NS; ++si)  // the assumption held: fill the placeholders
            for (auto& e : rx_out[si])
                if (e.kind == 3) {
                    e.kind = 2;
                    e.v = missing[(size_t)e.batch]->out->payload[e.row];
                }
        break;
    }  // (terminates: a pass that asks for decodes adds their keys to the cache)
    // ---- callbacks, session by session, op by op (a send op's emits and a receive op's
    // deliveries never share an op, so the two lists merge by op index)
    Bufs B;
    B.rx = RXA.h;
    B.tx = TXA.h;
    B.dec = dec_bytes.data();
    B.io = z->io.h;
    B.own = &own;
    int calls = 0;
    // the bytes a callback is handed: an emit's datagram or payload (nullptr: nothing handed)
    auto bytes_of = [&](const Emit& e, size_t si, unsigned* len) -> const uint8_t* {
        if (e.kind == 0) {
            const PackBatch& b = packs[(size_t)e.batch];
            const size_t row = (size_t)e.group * b.n + e.row;
            const int wl = reinterpret_cast<const int*>(z->io.h + b.o_wlen)[row];
            *len = wl > 0 ? (unsigned)wl : 0u;
            return wl > 0 ? z->io.h + b.o_wire + row * b.wp : nullptr;
        }
        *len = e.v.len;
        return B.p(e.v, si);
    };
    // the arenas are far larger than the caches: the bytes a few callbacks ahead are requested
    // now, so a consumer reading every byte (a socket send, a checksum) finds them on the way
    // (3, 6 and 10 ahead measured alike, profiles/r05j; streaming stores for the input copies
    // instead made them slower, 20 -> 36 ms, profiles/r05g)
    constexpr size_t kAhead = 4;
    auto prefetch = [&](const std::vector<Emit>& l, size_t i, size_t si) {
        if (i >= l.size() || l[i].kind == 3) return;
        unsigned len = 0;
        const uint8_t* q = bytes_of(l[i], si, &len);
        if (!q) return;
        for (unsigned o = 0; o < len; o += 64) __builtin_prefetch(q + o, 0, 0);
    };
    for (size_t si = 0; si < NS; ++si) {
        Session& S = z->sessions[si];
        const auto& to = tx_out[si];
        const auto& ro = rx_out[si];
        size_t a = 0, c = 0;
        for (size_t i = 0; i < kAhead; ++i) {
            prefetch(to, i, si);
            prefetch(ro, i, si);
        }
        while (a < to.size() || c < ro.size()) {
            const bool take_tx = c >= ro.size() || (a < to.size() && to[a].op <= ro[c].op);
            if (take_tx) prefetch(to, a + kAhead, si);
            else prefetch(ro, c + kAhead, si);
            const Emit& e = take_tx ? to[a++] : ro[c++];
            if (e.kind == 0) {
                const PackBatch& b = packs[(size_t)e.batch];
                const size_t row = (size_t)e.group * b.n + e.row;
                const int wl = reinterpret_cast<const int*>(z->io.h + b.o_wlen)[row];
                if (wl > 0 && pack_out)
                    pack_out(S.peer, reinterpret_cast<const char*>(z->io.h + b.o_wire + row * b.wp), (unsigned)wl);
            } else if (e.kind == 1) {
                if (pack_out) pack_out(S.peer, reinterpret_cast<const char*>(B.p(e.v, si)), e.v.len);
            } else if (unpack_out) {
                unpack_out(S.peer, reinterpret_cast<const char*>(B.p(e.v, si)), e.v.len, e.src);
            }
            ++calls;
        }
        S.ops.clear();
    }
    phase("callbacks");
    // the per-session scratch is freed on the session threads (its blocks came from their
    // allocator arenas; one thread freeing ~10^5 decode-cache nodes took ~3 ms, r05i)
    parallel_for(z, NS, threads, [&](size_t si) {
        DecodeCache().swap(caches[si]);
        std::vector<DecodeReq>().swap(miss_s[si]);
        std::vector<Emit>().swap(rx_out[si]);
        std::vector<Emit>().swap(tx_out[si]);
        std::vector<Verdict>().swap(verd[si]);
        if (si < loc.size()) std::vector<Local>().swap(loc[si]);
    });
    // ---- what the state still refers to moves to the spare arenas: the window slots'
    // datagrams and the open send groups' payloads; everything else is dropped
    {
        HostArena& NR = z->rx[z->rxc ^ 1];
        NR.used = 0;
        for (auto& S : z->sessions)
            for (auto& s : S.rx.slots) {
                if (!s.bValid) continue;
                uint32_t no = 0;
                if (!NR.append(RXA.h + s.dg_off, s.dg_len, &no)) return QFEC_ENOMEM;
                const uint32_t delta = no - s.dg_off;  // (mod 2^32: offsets move together)
                s.dg_off = no;
                s.shard.off += delta;
                s.payload.off += delta;
            }
        RXA.used = 0;
        z->rxc ^= 1;
        HostArena& NT = z->tx[z->txc ^ 1];
        NT.used = 0;
        for (auto& S : z->sessions)
            for (auto& p : S.tx.g_pay) {
                uint32_t no = 0;
                if (!NT.append(TXA.h + p.off, p.len, &no)) return QFEC_ENOMEM;
                p.off = no;
            }
        TXA.used = 0;
        z->txc ^= 1;
    }
    phase("compact");
    return calls;
}
}  // namespace

extern "C" {

int qfec_zfec_flush(qfec_zfec* z, qfec_pack_output_fn pack_out, qfec_unpack_output_fn unpack_out, void* stream) {
    if (!z) return QFEC_EINVAL;
    std::lock_guard<std::mutex> lk(z->mu);
    const int rc = flush_body(z, pack_out, unpack_out, stream);
    if (g_zfec_timing)  // what the flush's locals cost to free
        fprintf(stderr, "[qfec] zfec flush %-12s %8.3f ms\n", "teardown",
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_zfec_phase).count());
    return rc;
}

}  // extern "C"
