// ono_ring_impl.h — the ring manager's state, shared by the translation units
// that implement its schedules (ono_ring.cpp: RCCL / hops / direct / TCP /
// host-fed; ono_xgmi.cpp: the xGMI peer-access schedule).  Not part of the ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <cstdint>
#include <memory>
#include <mutex>
#include <utility>
#include <vector>

#include "ono_internal.h"

#define ONO_NCCL(expr)                                                                        \
    do {                                                                                      \
        ncclResult_t ono_r_ = (expr);                                                         \
        if (ono_r_ != ncclSuccess)                                                            \
            return ::ono::set_error(ONO_E_RCCL, "%s failed: %s (%s:%d)", #expr, ncclGetErrorString(ono_r_), \
                             __FILE__, __LINE__);                                             \
    } while (0)

namespace ono {

class HostPool;
struct XgmiState;    // ono_xgmi.cpp
struct SampleAhead;  // ono_tcp.cpp: the default sampler one push ahead
void sample_ahead_free(SampleAhead *a);

struct EventPair {
    hipEvent_t a = nullptr, b = nullptr;
    int kind = 0;  // ono_phase: 0 = library kernel, 1 = RCCL collective / TCP exchange, 2..4 = xGMI, 5 = codec
};

// HIP-event timer for the library's own launches (on the launch stream).
struct Timer {
    bool on = false;
    std::vector<EventPair> pending, pool;
    double kernel_ms = 0, coll_ms = 0;
    int64_t kernels = 0, colls = 0;
    double phase_ms[ONO_PHASES] = {};
    int64_t phase_n[ONO_PHASES] = {};

    hipError_t begin(hipStream_t s, EventPair &p, int kind) {
        if (!pool.empty()) {
            p = pool.back();
            pool.pop_back();
        } else {
            hipError_t e = hipEventCreate(&p.a);
            if (e != hipSuccess) return e;
            e = hipEventCreate(&p.b);
            if (e != hipSuccess) return e;
        }
        p.kind = kind;
        return hipEventRecord(p.a, s);
    }
    hipError_t end(hipStream_t s, EventPair &p) {
        hipError_t e = hipEventRecord(p.b, s);
        pending.push_back(p);
        return e;
    }
    hipError_t drain() {
        for (auto &p : pending) {
            hipError_t e = hipEventSynchronize(p.b);
            if (e != hipSuccess) return e;
            float ms = 0;
            e = hipEventElapsedTime(&ms, p.a, p.b);
            if (e != hipSuccess) return e;
            if (p.kind == ONO_PHASE_KERNEL) { kernel_ms += ms; kernels++; }
            else if (p.kind < ONO_PHASE_SPARSE_CODEC) { coll_ms += ms; colls++; }
            if (p.kind >= 0 && p.kind < ONO_PHASES) { phase_ms[p.kind] += ms; phase_n[p.kind]++; }
            pool.push_back(p);
        }
        pending.clear();
        return hipSuccess;
    }
    void reset() {
        kernel_ms = coll_ms = 0;
        kernels = colls = 0;
        for (int i = 0; i < ONO_PHASES; i++) { phase_ms[i] = 0; phase_n[i] = 0; }
    }
    void destroy() {
        for (auto &p : pending) pool.push_back(p);
        pending.clear();
        for (auto &p : pool) { (void)hipEventDestroy(p.a); (void)hipEventDestroy(p.b); }
        pool.clear();
    }
};

// RAII device guard: run on the ring's device, restore the caller's afterwards.
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};


}  // namespace ono

struct ono_ring {
    int pos = 0, n = 1, device = 0, wire = ONO_WIRE_F32;
    size_t size = 0;
    float *grad = nullptr, *residual = nullptr;
    std::vector<size_t> off;
    size_t maxc = 0;
    void *wbuf[2] = {nullptr, nullptr};  // hop-ring wire buffers, (maxc + 4) x 4 B each
    int algo = ONO_ALGO_AUTO;
    // direct schedule: all-to-all receive slots, all-gather staging (f16),
    // the owner's f16 message
    float *rbuf = nullptr;
    uint16_t *gstage = nullptr, *msg = nullptr;
    // the rank's exchange plan (ono_plan.cpp) for plan_algo / plan_segments
    std::vector<ono_plan_step> plan;
    int plan_algo = -1, plan_segments = -1;
    ncclComm_t comm = nullptr;
    // TCP transport (ono_ring_create_tcp, ono_tcp.cpp): the caller's connected
    // sockets to the previous and next worker, pinned frame buffers (grown on
    // demand; payloads 4-B aligned like the reference's Vec<u32>, source.rs:43-50)
    int fd_prev = -1, fd_next = -1;
    uint8_t *tx = nullptr, *rx = nullptr, *sp_rx = nullptr;
    size_t tx_cap = 0, rx_cap = 0, sp_rx_cap = 0;
    size_t tcp_block = 0;           // pipelining piece of a frame (tcp_block_bytes())
    // SparseCapable serializer (ono_ring_set_sparse): keep ratio r of each
    // pushed chunk (0 = the Base dense serializer); the sampler draws the
    // threshold sample above 16384 values (default: ono_sparse_sample_default
    // over sample_state); sp_dev holds this worker's encoded frame in HBM,
    // sp_tmp (sp_tmp_cap values) an incoming chunk that is not a whole-chunk DenseGrad
    float sparse_r = 0.0f;
    uint64_t sample_state = 0;
    ono_sample_fn sampler = nullptr;
    void *sampler_ctx = nullptr;
    uint32_t *sample_idx = nullptr;   // pinned host: the sampler's output, uploaded in stream order
    uint32_t *sp_idx_dev = nullptr;   // the gathered keys on the device (the threshold's scratch)
    ono::SampleAhead *ahead = nullptr;  // the default sampler's coming draws (a helper thread, a queue)
    float *sp_t_dev = nullptr;        // the push's threshold on the device (sparse_threshold_dev)
    uint8_t *sp_rx_dev = nullptr;     // a received SparseGrad, uploaded for the stream-ordered lift
    size_t sp_rx_dev_cap = 0;
    uint64_t *sp_status = nullptr;    // host-mapped: the stream-ordered lift's status word
    uint64_t *tcp_word = nullptr, *tcp_word_dev = nullptr;  // host-mapped: the hops' stream_wait word
    uint32_t tcp_epoch = 0;
    uint64_t *dn_arrive = nullptr;  // device: the dense hop kernels' wave count (KernelDone), never reset
    uint64_t dn_base = 0;
    uint8_t *sp_dev = nullptr;
    size_t sp_dev_cap = 0;
    uint8_t *sp_tx = nullptr;  // pinned coherent: a small push's SparseGrad frame, encoded in place
    size_t sp_tx_cap = 0;
    float *sp_tmp = nullptr;
    size_t sp_tmp_cap = 0;
    // small-frame TCP rings: the wire buffers are pinned host frames the codec
    // kernels read and write in place (no D2H / H2D per hop); zc[b] + 16 is the
    // payload base, so a frame's 12-byte header sits just before its payload
    uint8_t *zc[2] = {nullptr, nullptr};
    std::vector<hipEvent_t> tx_ev;  // one per piece of a frame's D2H
    // segmented f32 all-reduce (ono_ring_set_pipeline): the finaliser of
    // segment k runs on astream while segment k+1 is still on the wire; the
    // plans' side stream (astream) is also where the direct schedule zeroes
    // the residual beside its all-gather (ev_seg: one event per fork)
    int segments = 0;  // 0 = unresolved: env ONO_AR_SEGMENTS, default 4
    hipStream_t astream = nullptr;
    std::vector<hipEvent_t> ev_seg;
    hipEvent_t ev_ajoin = nullptr;
    std::atomic<bool> aborted{false};
    std::mutex mu;  // serialises host-form calls and the timer
    // host-fed pipeline (ono_ring_pull_grads_host): H2D on hstream, reduce on
    // cstream, D2H on dstream; pinned bounce slots for unregistered buffers
    hipStream_t hstream = nullptr, cstream = nullptr, dstream = nullptr;
    float *pin_in = nullptr, *pin_out = nullptr;  // kSlots x chunk elements each
    std::unique_ptr<ono::HostPool> pool;               // CPU copies of the bounce path
    std::vector<hipEvent_t> ev_h, ev_c, ev_d;
    std::vector<std::pair<void *, size_t>> registered;  // ono_ring_register_host
    ono::Timer timer;
    // xGMI peer-access schedule (ONO_ALGO_XGMI, ono_xgmi.cpp); owned, freed by ono_xgmi_free
    ono::XgmiState *xgmi = nullptr;
    double xgmi_timeout_s = 0;  // ono_ring_set_xgmi_timeout (0 = env ONO_XGMI_TIMEOUT_S, else the default)
};

namespace ono {

template <class F>
int timed(ono_ring *r, hipStream_t s, int kind, F &&f) {
    EventPair p;
    if (r->timer.on) ONO_HIP(r->timer.begin(s, p, kind));
    int rc = f();
    if (rc != ONO_OK) return rc;
    if (r->timer.on) ONO_HIP(r->timer.end(s, p));
    return ONO_OK;
}

#define ONO_K(ring, s, expr) \
    do { int rc_ = timed(ring, s, 0, [&]() -> int { ONO_HIP(expr); return ONO_OK; }); if (rc_) return rc_; } while (0)

// the TCP edge's pull_grads (ono_tcp.cpp)
int tcp_pull_grads(ono_ring *r, float *res, float *grad, hipStream_t s);

// xGMI peer-access schedule (ono_xgmi.cpp)
int xgmi_pull_grads(ono_ring *r, float *res, float *grad, hipStream_t s);
// reg: res_host and grad_host are registered with the ring (ono_ring_register_host)
int xgmi_pull_grads_host(ono_ring *r, float *res_host, float *grad_host, size_t sub_elems, bool reg);
// the ring's host copy pool (ono_ring.cpp; made on first use): dst = src, bytes split over its threads
void host_copy(ono_ring *r, void *dst, const void *src, size_t bytes);
int xgmi_ps_step(ono_ring *r, const float *grad, float *params, size_t N, size_t C, float *gshard, float *wshard,
                 const OptLaunch &opt, float *v, float *s_, hipStream_t s);
void xgmi_abort(ono_ring *r);
void xgmi_set_timeout(ono_ring *r);  // re-reads r->xgmi_timeout_s into an allocated region
void xgmi_free(ono_ring *r);  // collective: a final barrier before unmapping

}  // namespace ono
