// qfec_pipe.cpp -- qfec_pipe_* (include/qfec.h): batches that start and end in pinned host memory,
// streamed over several HIP streams and devices (BASELINE configs[4]).
#include "qfec_rt.hpp"

using namespace qfec;

// ====================================================================== host streaming pipe
// BASELINE config 5: batches that start and end in (pinned) host memory, streamed over
// several HIP streams per device and several devices.  Each slot = (device, stream, event,
// device staging, failed counter).  A piece of a batch takes the next slot round-robin
// (devices interleaved), waits for that slot's previous piece, and queues H2D -> kernel ->
// D2H on the slot's stream, so one piece's copies overlap the other slots' kernels and
// copies.  The caller's buffers must be pinned (DMA'd directly, no host memcpy) and stay
// untouched until qfec_pipe_wait.
struct qfec_pipe {
    struct Slot {
        int device = 0;
        DevCtx* ctx = nullptr;
        hipStream_t stream = nullptr;
        hipEvent_t done = nullptr;
        uint8_t* d_buf = nullptr;
        unsigned* d_failed = nullptr;  // accumulated under-determined groups (reconstruct)
        unsigned* h_failed = nullptr;  // pinned read-back
        bool busy = false;
    };
    std::mutex mu;
    std::vector<Slot> slots;
    size_t next = 0;
    size_t cap = 0;  // staging bytes per slot
};

namespace {

// wait for every queued piece (errors are reported after all slots are drained, so no DMA
// is left in flight into caller memory when an error returns)
int pipe_drain(qfec_pipe* p) {
    int rc = QFEC_OK;
    for (auto& s : p->slots) {
        if (!s.busy) continue;
        hipError_t e = hipEventSynchronize(s.done);
        if (e != hipSuccess) {
            (void)hipSetDevice(s.device);
            (void)hipStreamSynchronize(s.stream);
            if (!rc) rc = hip_fail(e, "qfec_pipe: piece failed");
        }
        s.busy = false;
    }
    return rc;
}

struct DeviceRestore {
    int prev = -1;
    DeviceRestore() { if (hipGetDevice(&prev) != hipSuccess) prev = -1; }
    ~DeviceRestore() { if (prev >= 0) (void)hipSetDevice(prev); }
};

// the next slot, with its previous piece finished
int pipe_take(qfec_pipe* p, qfec_pipe::Slot** out) {
    qfec_pipe::Slot& s = p->slots[p->next++ % p->slots.size()];
    HIP_TRY(hipSetDevice(s.device));
    if (s.busy) {
        HIP_TRY(hipEventSynchronize(s.done));
        s.busy = false;
    }
    *out = &s;
    return QFEC_OK;
}

// groups per piece: fits a slot, and a batch spreads over all slots
long long pipe_piece(const qfec_pipe* p, long long groups, size_t per_group) {
    long long fit = (long long)(p->cap / per_group);
    long long even = (groups + (long long)p->slots.size() - 1) / (long long)p->slots.size();
    return std::max<long long>(1, std::min(fit, std::max<long long>(even, 64)));
}

}  // namespace

extern "C" {

qfec_pipe* qfec_pipe_new(const int* devices, int ndev, int nstreams, long long slot_bytes) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
        (void)hipGetLastError();
        set_error("qfec_pipe_new: no HIP device available");
        return nullptr;
    }
    if (nstreams < 1 || nstreams > 16 || slot_bytes < (1 << 16) || ndev < 0 || ndev > 64 || (ndev > 0 && !devices)) {
        set_error("qfec_pipe_new: invalid argument");
        return nullptr;
    }
    std::vector<int> devs;
    if (ndev == 0)
        for (int d = 0; d < count; ++d) devs.push_back(d);
    else
        devs.assign(devices, devices + ndev);
    for (int d : devs)
        if (d < 0 || d >= count || d >= kMaxDevices) {
            set_error("qfec_pipe_new: device %d out of range (%d visible)", d, count);
            return nullptr;
        }
    DeviceRestore restore;
    qfec_pipe* p = new (std::nothrow) qfec_pipe();
    if (!p) return nullptr;
    p->cap = round_up((size_t)slot_bytes, 4096);
    p->slots.resize((size_t)nstreams * devs.size());
    int rc = QFEC_OK;
    for (size_t i = 0; i < p->slots.size() && !rc; ++i) {
        qfec_pipe::Slot& s = p->slots[i];
        s.device = devs[i % devs.size()];  // devices interleaved: consecutive pieces land on different GPUs
        if (hipSetDevice(s.device) != hipSuccess) { rc = QFEC_EHIP; break; }
        if ((rc = current_ctx(&s.ctx))) break;
        if (hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&s.done, hipEventDisableTiming) != hipSuccess ||
            hipMalloc(&s.d_buf, p->cap) != hipSuccess || hipMalloc(&s.d_failed, 16) != hipSuccess ||
            hipMemset(s.d_failed, 0, 16) != hipSuccess ||
            hipHostMalloc(&s.h_failed, 16, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            set_error("qfec_pipe_new: allocation on device %d failed", s.device);
            rc = QFEC_ENOMEM;
        }
    }
    if (rc) {
        qfec_pipe_free(p);
        return nullptr;
    }
    return p;
}

void qfec_pipe_free(qfec_pipe* p) {
    if (!p) return;
    DeviceRestore restore;
    {
        std::lock_guard<std::mutex> lk(p->mu);
        (void)pipe_drain(p);
        for (auto& s : p->slots) {
            if (hipSetDevice(s.device) != hipSuccess) continue;
            if (s.d_buf) (void)hipFree(s.d_buf);
            if (s.d_failed) (void)hipFree(s.d_failed);
            if (s.h_failed) (void)hipHostFree(s.h_failed);
            if (s.done) (void)hipEventDestroy(s.done);
            if (s.stream) (void)hipStreamDestroy(s.stream);
        }
    }
    delete p;
}

int qfec_pipe_encode(qfec_pipe* p, qfec_code* code, const unsigned char* h_data, unsigned char* h_parity,
                     long long groups, int block_size, long long pitch) {
    if (!p || !code || groups < 0 || block_size < 1 || pitch < block_size || (groups > 0 && (!h_data || !h_parity))) {
        set_error("qfec_pipe_encode: invalid argument");
        return QFEC_EINVAL;
    }
    if (groups == 0 || code->m == 0) return QFEC_OK;
    const int k = code->k, m = code->m;
    const size_t in_g = (size_t)k * (size_t)pitch, out_g = (size_t)m * (size_t)pitch;
    if (in_g + out_g > p->cap) {
        set_error("qfec_pipe_encode: one group (%zu B) exceeds the slot staging (%zu B)", in_g + out_g, p->cap);
        return QFEC_EINVAL;
    }
    if (!is_pinned_host(h_data) || !is_pinned_host(h_parity)) {
        set_error("qfec_pipe_encode: host buffers must be pinned (hipHostMalloc / hipHostRegister)");
        return QFEC_EINVAL;
    }
    std::lock_guard<std::mutex> lk(p->mu);
    DeviceRestore restore;
    const long long gp = pipe_piece(p, groups, in_g + out_g);
    int rc = QFEC_OK;
    for (long long g0 = 0; g0 < groups && !rc; g0 += gp) {
        const long long gn = std::min(gp, groups - g0);
        qfec_pipe::Slot* s = nullptr;
        if ((rc = pipe_take(p, &s))) break;
        uint32_t* tab = nullptr;
        {
            std::lock_guard<std::mutex> ck(code->mu);
            rc = ensure_enc(code, s->device, &tab);
        }
        if (rc) break;
        uint8_t *z_in = nullptr, *z_out = nullptr;
        if (tuning().host_zero_copy && host_dev(h_data, &z_in) && host_dev(h_parity, &z_out)) {
            // zero copy: the piece's kernel reads and writes the pinned host buffers directly
            s->busy = true;
            if ((rc = run_encode(*s->ctx, code, tab, m, z_in + (size_t)g0 * in_g, z_out + (size_t)g0 * out_g, gn,
                                 block_size, pitch, s->stream, -1, -1, true)))
                break;
            if (hipEventRecord(s->done, s->stream) != hipSuccess) { rc = hip_fail(hipGetLastError(), "event"); break; }
            continue;
        }
        uint8_t* d_in = s->d_buf;
        uint8_t* d_out = s->d_buf + (size_t)gn * in_g;
        if (hipMemcpyAsync(d_in, h_data + (size_t)g0 * in_g, (size_t)gn * in_g, hipMemcpyHostToDevice, s->stream) !=
            hipSuccess) { rc = hip_fail(hipGetLastError(), "qfec_pipe_encode: H2D"); break; }
        s->busy = true;
        if ((rc = run_encode(*s->ctx, code, tab, m, d_in, d_out, gn, block_size, pitch, s->stream))) break;
        if (hipMemcpyAsync(h_parity + (size_t)g0 * out_g, d_out, (size_t)gn * out_g, hipMemcpyDeviceToHost,
                           s->stream) != hipSuccess) { rc = hip_fail(hipGetLastError(), "qfec_pipe_encode: D2H"); break; }
        if (hipEventRecord(s->done, s->stream) != hipSuccess) { rc = hip_fail(hipGetLastError(), "event"); break; }
    }
    if (rc) {
        const std::string err = t_last_error;
        (void)pipe_drain(p);
        t_last_error = err;
    }
    return rc;
}

int qfec_pipe_reconstruct(qfec_pipe* p, qfec_code* code, unsigned char* h_data, const unsigned char* h_parity,
                          const unsigned char* h_marks, long long groups, int block_size, long long pitch) {
    if (!p || !code || groups < 0 || block_size < 1 || pitch < block_size ||
        (groups > 0 && (!h_data || !h_marks || (code->m > 0 && !h_parity)))) {
        set_error("qfec_pipe_reconstruct: invalid argument");
        return QFEC_EINVAL;
    }
    if (groups == 0) return QFEC_OK;
    const int k = code->k, m = code->m;
    if (k + m > QFEC_LUT_MAX_N) {
        set_error("qfec_pipe_reconstruct: k + m = %d > %d", k + m, QFEC_LUT_MAX_N);
        return QFEC_EUNSUP;
    }
    const size_t dg = (size_t)k * (size_t)pitch, pg = (size_t)m * (size_t)pitch;
    const size_t per_group = dg + pg + (size_t)(k + m);
    if (per_group + 64 > p->cap) {
        set_error("qfec_pipe_reconstruct: one group exceeds the slot staging (%zu B)", p->cap);
        return QFEC_EINVAL;
    }
    if (!is_pinned_host(h_data) || (m && !is_pinned_host(h_parity)) || !is_pinned_host(h_marks)) {
        set_error("qfec_pipe_reconstruct: host buffers must be pinned (hipHostMalloc / hipHostRegister)");
        return QFEC_EINVAL;
    }
    std::lock_guard<std::mutex> lk(p->mu);
    DeviceRestore restore;
    const long long gp = pipe_piece(p, groups, per_group + 1);
    int rc = QFEC_OK;
    for (long long g0 = 0; g0 < groups && !rc; g0 += gp) {
        const long long gn = std::min(gp, groups - g0);
        qfec_pipe::Slot* s = nullptr;
        if ((rc = pipe_take(p, &s))) break;
        DevTables* d = nullptr;
        {
            std::lock_guard<std::mutex> ck(code->mu);
            rc = ensure_lut(code, s->device, &d);
        }
        if (rc) break;
        // slot layout: data [gn][k][pitch] | parity [gn][m][pitch] | marks in rs.c layout
        // for the piece: gn*k data marks, then gn*m parity marks (module/rs.c:609-612)
        uint8_t *z_data = nullptr, *z_par = nullptr;
        if (tuning().host_zero_copy && host_dev(h_data, &z_data) && (m == 0 || host_dev(h_parity, &z_par))) {
            // zero copy: survivors read and erased rows written in host memory; the piece's
            // marks (rs.c layout for gn groups) staged into the slot
            uint8_t* dm = s->d_buf;
            s->busy = true;
            if (hipMemcpyAsync(dm, h_marks + (size_t)g0 * k, (size_t)gn * k, hipMemcpyHostToDevice, s->stream) ||
                (m && hipMemcpyAsync(dm + (size_t)gn * k, h_marks + (size_t)groups * k + (size_t)g0 * m, (size_t)gn * m,
                                     hipMemcpyHostToDevice, s->stream))) {
                rc = hip_fail(hipGetLastError(), "qfec_pipe_reconstruct: marks H2D");
                break;
            }
            if ((rc = run_reconstruct(*s->ctx, code, d->d_lut, nullptr, d->d_rec, z_data + (size_t)g0 * dg,
                                      m ? z_par + (size_t)g0 * pg : nullptr, dm, gn, block_size, pitch, s->d_failed,
                                      s->stream)))
                break;
            if (hipEventRecord(s->done, s->stream) != hipSuccess) { rc = hip_fail(hipGetLastError(), "event"); break; }
            continue;
        }
        uint8_t* dd = s->d_buf;
        uint8_t* dp = dd + (size_t)gn * dg;
        uint8_t* dm = dp + (size_t)gn * pg;
        s->busy = true;
        if (hipMemcpyAsync(dd, h_data + (size_t)g0 * dg, (size_t)gn * dg, hipMemcpyHostToDevice, s->stream) ||
            (m && hipMemcpyAsync(dp, h_parity + (size_t)g0 * pg, (size_t)gn * pg, hipMemcpyHostToDevice, s->stream)) ||
            hipMemcpyAsync(dm, h_marks + (size_t)g0 * k, (size_t)gn * k, hipMemcpyHostToDevice, s->stream) ||
            (m && hipMemcpyAsync(dm + (size_t)gn * k, h_marks + (size_t)groups * k + (size_t)g0 * m, (size_t)gn * m,
                                 hipMemcpyHostToDevice, s->stream))) {
            rc = hip_fail(hipGetLastError(), "qfec_pipe_reconstruct: H2D");
            break;
        }
        if ((rc = run_reconstruct(*s->ctx, code, d->d_lut, nullptr, d->d_rec, dd, dp, dm, gn, block_size, pitch,
                                  s->d_failed, s->stream)))
            break;
        if (hipMemcpyAsync(h_data + (size_t)g0 * dg, dd, (size_t)gn * dg, hipMemcpyDeviceToHost, s->stream) !=
            hipSuccess) { rc = hip_fail(hipGetLastError(), "qfec_pipe_reconstruct: D2H"); break; }
        if (hipEventRecord(s->done, s->stream) != hipSuccess) { rc = hip_fail(hipGetLastError(), "event"); break; }
    }
    if (rc) {
        const std::string err = t_last_error;
        (void)pipe_drain(p);
        t_last_error = err;
    }
    return rc;
}

int qfec_pipe_wait(qfec_pipe* p, long long* failed) {
    if (!p) return QFEC_EINVAL;
    std::lock_guard<std::mutex> lk(p->mu);
    DeviceRestore restore;
    int rc = pipe_drain(p);
    long long nf = 0;
    for (auto& s : p->slots) {  // read back and reset the slots' failed counters
        if (hipSetDevice(s.device) != hipSuccess ||
            hipMemcpyAsync(s.h_failed, s.d_failed, 4, hipMemcpyDeviceToHost, s.stream) != hipSuccess ||
            hipMemsetAsync(s.d_failed, 0, 4, s.stream) != hipSuccess || hipStreamSynchronize(s.stream) != hipSuccess) {
            if (!rc) rc = hip_fail(hipGetLastError(), "qfec_pipe_wait");
            continue;
        }
        nf += *s.h_failed;
    }
    if (failed) *failed = nf;
    return rc;
}

int qfec_pipe_slots(const qfec_pipe* p) { return p ? (int)p->slots.size() : QFEC_EINVAL; }

}  // extern "C"

