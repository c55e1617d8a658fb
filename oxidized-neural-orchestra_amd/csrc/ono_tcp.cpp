// ono_tcp.cpp — the TCP edge: WorkerRingManager over the
// worker's own sockets, speaking the reference's frames byte for byte, with
// the hop arithmetic in HBM.
//
// Frames (comms/src/protocol/msg.rs:120-191, codec/sink.rs:37-58,
// codec/source.rs:34-57):
//   [u64 BE len = 4 + payload][u32 BE kind][payload]
// The kind byte is the header's u32 cast to u8 (msg.rs:168):
//   1 / 2  DenseGrad  (is_last false / true): f16 LE values
//   3 / 4  SparseGrad (is_last false / true): the grad_drop stream
//          [u64 LE total][{u32 LE offset, u32 LE run, f16 LE x run}*]
//          (comms/src/sparse/protocol.rs:57-86)
//   0 control (JSON), 5 params, 6 data chunk: WorkerHandle::recv_event's
//          verdict (ono_msg.cpp): a worker event the ring rejects ->
//          ONO_E_PROTO "Received an invalid worker event" (worker_ring.rs:136-138),
//          "loss diverged", "Unexpected message from worker" or the serde
//          error -> ONO_E_IO (handles/worker.rs:82-130)
//   >= 7   Msg::deserialize's invalid_kind_byte io::Error (msg.rs:187) -> ONO_E_IO
// A worker receives either gradient kind whatever its own serializer is
// (WorkerHandle::recv_event lifts SparseGrad into the handle's zero-filled
// buffer, comms/src/handles/worker.rs:102-108), so MI355X workers share a
// ring with reference workers of either serializer.  A gradient of another
// length than the hop's chunk is added over the shorter length in the scatter
// (the zip of worker_ring.rs:141-143) and refused in the gather, where the
// reference's copy_from_slice (:200) panics.
//
// Serializers of this worker (its push_grad, handles/worker.rs:157-174):
//   Base (default)       DenseGrad of f16(chunk) (compressor.rs:106-118)
//   SparseCapable{r}     (ono_ring_set_sparse) t = calculate_threshold(chunk, r)
//                        (protocol.rs:33-49) and the grad_drop stream; the
//                        SparseGrad goes out only when that stream is no longer
//                        than the f16 payload (2 bytes per value), else the
//                        DenseGrad of f16(chunk) (compressor.rs:79-89).  The ring
//                        takes the branch the push selects (worker_ring.rs:125-134,
//                        177-193): scatter zeroes the sent values (sparse) or the
//                        chunk (dense); gather keeps only the sent values in grad
//                        and leaves the owned residual as it is (sparse), or zeroes
//                        the owned residual at j == 0 (dense).
//
// One hop = the fused kernel (or the sparse encoder) writes the payload, it
// comes down to a pinned frame in pieces (D2H + one event per piece) and a
// sender thread ships each piece as soon as it lands, while this thread reads
// the previous worker's frame, validates the header and sends each complete
// piece of a dense payload up to HBM while the rest is still on the socket.
// Small dense frames (<= 256 KiB, ONO_TCP_ZEROCOPY) skip HBM: the codec
// kernels read and write them in pinned host memory.
#include <hip/hip_runtime.h>

#include <poll.h>
#include <sys/socket.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cerrno>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "ono_internal.h"
#include "ono_ring_impl.h"

using namespace ono;

namespace {

constexpr int kTcpPollMs = 100;                   // abort / peer-failure latency
constexpr size_t kTcpInline = size_t(256) << 10;  // frames up to this go through one poll loop
constexpr size_t kSampleMax = 16384;              // SAMPLE_SIZE (protocol.rs:13-19)
// the next push's sample keys gathered by the hop's add / copy (launch_hop_post) for chunks up to this many
// values: the sampler's helper thread buckets each draw by 256-value block (offsets: L / 256 + 1 words)
constexpr size_t kFuseKeysMax = size_t(1) << 20;
constexpr size_t kFuseBlock = 256;
constexpr size_t kFuseOffs = kFuseKeysMax / kFuseBlock + 1;
// a SparseGrad push whose worst-case stream fits this is encoded straight into a pinned frame (the drop's
// own wait covers it: no D2H and no second wait); larger ones come down in pieces beside the send
constexpr size_t kSparseZeroCopy = size_t(4) << 20;
// measurement A/B (round 6), read once: ONO_TCP_LIFT_PINNED=0 copies a received SparseGrad into HBM before the
// lift (round 5's form) instead of lifting from the pinned frame; ONO_THR_HBM=1 has the sampler's helper
// thread upload each draw to HBM for the gather (measured no gain: profiles/r06_s5_tcp_variants.jsonl)
bool env_on(const char *name) {
    const char *e = getenv(name);
    return !(e && !strcmp(e, "0"));
}
bool lift_pinned() {
    static const bool v = env_on("ONO_TCP_LIFT_PINNED");
    return v;
}
bool thr_hbm() {  // (default off: no gain measured, and the upload lengthened every draw of the queue)
    static const bool v = [] {
        const char *e = getenv("ONO_THR_HBM");
        return e && !strcmp(e, "1");
    }();
    return v;
}
// ONO_TCP_TRACE=1 (measurement): host time per step of every SparseCapable hop, summed over the process's
// rings and printed to stderr at exit — sample (taken from the queue or drawn) / threshold (its launches) /
// drop (launch + wait) / mask / exchange / incoming (lift + wait) / add — for where a config-1 round's time
// goes between the kernels
struct HopTrace {
    static constexpr int kSteps = 7;
    std::atomic<uint64_t> ns[kSteps] = {}, hops{0}, draw_ns{0}, draws{0}, wait_ns{0}, waits{0}, misses{0},
        take_ns{0}, takes{0}, lifts{0}, lift_call_ns{0}, lift_wait_ns{0};
    ~HopTrace() {
        const uint64_t h = hops.load();
        if (!h) return;
        if (draws.load())
            fprintf(stderr, "ONO_TCP_TRACE the sampler queue's draws: %llu, %.2f us each; takes that waited: %llu, "
                    "%.2f us each; misses (drawn inline): %llu\n",
                    (unsigned long long)draws.load(), draw_ns.load() / 1e3 / (double)draws.load(),
                    (unsigned long long)waits.load(), waits.load() ? wait_ns.load() / 1e3 / (double)waits.load() : 0.0,
                    (unsigned long long)misses.load());
        if (takes.load())
            fprintf(stderr, "ONO_TCP_TRACE take() calls: %llu, %.2f us each\n", (unsigned long long)takes.load(),
                    take_ns.load() / 1e3 / (double)takes.load());
        if (lifts.load())
            fprintf(stderr, "ONO_TCP_TRACE lifts: %llu, us each: the call %.2f, until complete %.2f\n",
                    (unsigned long long)lifts.load(), lift_call_ns.load() / 1e3 / (double)lifts.load(),
                    lift_wait_ns.load() / 1e3 / (double)lifts.load());
        static const char *names[kSteps] = {"threshold", "drop", "mask", "exchange", "incoming", "add", "sample"};
        fprintf(stderr, "ONO_TCP_TRACE %llu hops, us per hop:", (unsigned long long)h);
        for (int k = 0; k < kSteps; k++) fprintf(stderr, " %s %.2f", names[k], ns[k].load() / 1e3 / (double)h);
        fprintf(stderr, "\n");
    }
};
HopTrace g_hop_trace;
bool trace_on() {
    static const bool v = getenv("ONO_TCP_TRACE") != nullptr;
    return v;
}
std::atomic<uint64_t> g_hops_seen{0};
struct HopClock {  // one hop's step times into g_hop_trace (a no-op unless ONO_TCP_TRACE; the process's first
                   // 64 hops are left out: they hold the one-time allocations of the warmup round)
    bool on = trace_on() && g_hops_seen++ >= 64;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void step(int k) {
        if (!on) return;
        const auto u = std::chrono::steady_clock::now();
        g_hop_trace.ns[k] += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(u - t).count();
        t = u;
    }
    void done() {
        if (on) g_hop_trace.hops++;
    }
};
// ONO_TCP_SPIN_US (measurement, default 0): an inline exchange tries its socket calls without blocking for up
// to this long before it sleeps in poll(2).  200 us measured slower, not faster: config 1 sparse 0.218 / 0.233
// vs 0.200 / 0.186 ms per round, dense 0.095 / 0.120 vs 0.092 / 0.088 (profiles/r06_s18_variants.txt) — the
// spinning threads take CPU time from the process's quota that the peer's thread and the host waits need
int tcp_spin_us() {
    static const int v = [] {
        const char *e = getenv("ONO_TCP_SPIN_US");
        return e ? std::max(0, atoi(e)) : 0;
    }();
    return v;
}
// Where a sparse push's mask runs (ONO_TCP_MASK): "fused" (default) in one launch with the hop's add or copy
// after the exchange (launch_hop_post: neither the send nor the lift waits for a launch of its own), "early"
// before the exchange, "late" right after it (round 5's form)
enum MaskAt { MASK_FUSED = 0, MASK_EARLY = 1, MASK_LATE = 2 };
int mask_at() {
    static const int v = [] {
        const char *e = getenv("ONO_TCP_MASK");
        if (e && !strcmp(e, "early")) return (int)MASK_EARLY;
        if (e && !strcmp(e, "late")) return (int)MASK_LATE;
        return (int)MASK_FUSED;
    }();
    return v;
}

enum : uint32_t {
    KIND_CONTROL = 0,
    KIND_DENSE = 1,
    KIND_DENSE_LAST = 2,
    KIND_SPARSE = 3,
    KIND_SPARSE_LAST = 4,
    KIND_MAX_VALID = 6,
    KIND_DENSE_OTHER = 16,  // (internal) a DenseGrad of another length than the hop's chunk
};

size_t tcp_block_bytes() {  // env ONO_TCP_BLOCK_KIB (default 4 MiB), read once per ring
    const char *v = getenv("ONO_TCP_BLOCK_KIB");
    long k = v ? atol(v) : 0;
    return k > 0 ? (size_t)k << 10 : size_t(4) << 20;
}

struct TcpErr {
    int code = ONO_OK;
    char msg[192] = {0};
};

// pinned host buffer grown on demand (never while a transfer into it is pending), with a quarter of headroom:
// SparseGrad frames differ in length from hop to hop, and pinning tens of MB costs milliseconds, so a buffer
// sized to each new longest frame exactly was re-pinned round after round
int grow_pinned(uint8_t **p, size_t *cap, size_t need, unsigned flags = hipHostMallocDefault) {
    if (*cap >= need) return ONO_OK;
    if (*p) (void)hipHostFree(*p);
    *p = nullptr;
    *cap = 0;
    const size_t want = need + need / 4;
    ONO_HIP(hipHostMalloc((void **)p, want, flags));
    *cap = want;
    return ONO_OK;
}

int ensure_tx_events(ono_ring *r, size_t pieces) {
    while (r->tx_ev.size() < pieces) {
        hipEvent_t ev;
        ONO_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        r->tx_ev.push_back(ev);
    }
    return ONO_OK;
}

void put_header(uint8_t *h, size_t payload, uint32_t kind) {
    const uint64_t flen = 4 + (uint64_t)payload;
    for (int i = 0; i < 8; i++) h[i] = (uint8_t)(flen >> (56 - 8 * i));
    for (int i = 0; i < 4; i++) h[8 + i] = (uint8_t)(kind >> (24 - 8 * i));
}

// What this worker sends in one hop: a contiguous frame in pinned memory whose
// payload is complete (zero-copy) or arrives by D2H pieces gated on r->tx_ev.
struct Outgoing {
    const uint8_t *frame = nullptr;
    size_t payload = 0;
    size_t pieces = 0;  // 0: complete
};

// Where the previous worker's frame goes.  A DenseGrad of exactly
// dense_bytes (this hop's chunk) lands at dense_host and, when dense_dev is
// set, goes up to HBM piece by piece; every other frame (a DenseGrad of
// another length, a SparseGrad, a non-gradient message) lands whole in
// r->sp_rx (host) for the hop to judge.
struct Incoming {
    size_t dense_bytes = 0;
    uint8_t *dense_host = nullptr;
    uint8_t *dense_dev = nullptr;
    uint32_t kind = 0;  // result: KIND_DENSE, KIND_DENSE_OTHER, KIND_SPARSE, or the kind byte 0 / 5 / 6
    size_t bytes = 0;   // result: payload bytes
    bool sparse_dev = false;  // result: a large SparseGrad also went up to r->sp_rx_dev piece by piece
};
// a SparseGrad longer than this goes up to HBM in pieces while it is still on the socket (as a dense payload
// does), so that its lift starts at its last byte; shorter ones are lifted from the pinned frame
constexpr size_t kSparseUpload = size_t(1) << 20;

// Wait until `fd` is ready for `ev`; false (with e set) on abort, stop or poll error.
bool tcp_wait(ono_ring *r, int fd, short ev, const std::atomic<bool> &stop, TcpErr &e) {
    for (;;) {
        if (r->aborted.load()) { e.code = ONO_E_ABORTED; snprintf(e.msg, sizeof e.msg, "ring aborted"); return false; }
        if (stop.load()) { e.code = ONO_E_OTHER; return false; }  // the other side already failed
        struct pollfd p = {fd, ev, 0};
        int pr = poll(&p, 1, kTcpPollMs);
        if (pr < 0 && errno != EINTR) {
            e.code = ONO_E_IO; snprintf(e.msg, sizeof e.msg, "poll: %s", strerror(errno)); return false;
        }
        if (pr > 0) return true;
    }
}

// One send(2) of the frame's ready bytes; false (e set) on a socket error.
bool tcp_send_some(ono_ring *r, const uint8_t *tx, size_t &sent, size_t ready, TcpErr &e) {
    ssize_t k = send(r->fd_next, tx + sent, ready - sent, MSG_DONTWAIT | MSG_NOSIGNAL);
    if (k < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) {
        e.code = ONO_E_IO; snprintf(e.msg, sizeof e.msg, "send to next worker: %s", strerror(errno));
        return false;
    }
    if (k > 0) sent += (size_t)k;
    return true;
}

// Receive side of one hop: the 12-byte header first, then the payload into
// the destination its kind selects.
struct TcpRecv {
    Incoming &in;
    uint8_t hdr[12];
    size_t got = 0, need = 12, issued = 0;  // got/need count header + payload bytes
    bool have_hdr = false;
    uint8_t *dst = nullptr, *dev = nullptr;
    explicit TcpRecv(Incoming &i) : in(i) {}
    bool done() const { return have_hdr && got >= need; }

    bool header(ono_ring *r, TcpErr &e) {
        uint64_t l = 0;
        for (int i = 0; i < 8; i++) l = (l << 8) | hdr[i];
        const uint32_t kind = hdr[11];  // Header::from_be_bytes(..) as u8 (msg.rs:168)
        if (kind > KIND_MAX_VALID) {     // msg.rs:105-110, 187
            e.code = ONO_E_IO; snprintf(e.msg, sizeof e.msg, "Received an invalid kind byte %u", kind); return false;
        }
        if (l < 4) {  // msg.rs:98-103, 161-163
            e.code = ONO_E_IO;
            snprintf(e.msg, sizeof e.msg, "The given buffer is too small %llu, must at least be 4 bytes",
                     (unsigned long long)l);
            return false;
        }
        const uint64_t pay = l - 4;
        dst = nullptr;
        dev = nullptr;
        if (kind == KIND_DENSE || kind == KIND_DENSE_LAST) {
            if (pay % 2) {  // bytemuck::cast_slice to f16 (msg.rs:175) cannot split a value
                e.code = ONO_E_IO;
                snprintf(e.msg, sizeof e.msg, "DenseGrad payload of %llu bytes is not a whole number of f16 values",
                         (unsigned long long)pay);
                return false;
            }
            if (pay == in.dense_bytes) {
                dst = in.dense_host;
                dev = in.dense_dev;
                in.kind = KIND_DENSE;
            } else {
                in.kind = KIND_DENSE_OTHER;
            }
        } else {
            in.kind = (kind == KIND_SPARSE || kind == KIND_SPARSE_LAST) ? KIND_SPARSE : kind;
        }
        if (!dst) {  // the whole payload to host memory
            // (+64: the lift reads the frame in place in whole 8-byte words, the copy kernel in 4-byte ones)
            if (int rc = grow_pinned(&r->sp_rx, &r->sp_rx_cap, std::max<size_t>(pay, 8) + 64)) {
                e.code = rc; snprintf(e.msg, sizeof e.msg, "%s", ono_last_error()); return false;
            }
            dst = r->sp_rx;
            if (in.kind == KIND_SPARSE && pay > kSparseUpload) {  // and up to HBM piece by piece (the lift's input)
                const size_t want = (size_t)pay + 64;
                if (r->sp_rx_dev_cap < want) {  // (with headroom, as grow_pinned)
                    (void)hipFree(r->sp_rx_dev);
                    r->sp_rx_dev = nullptr;
                    r->sp_rx_dev_cap = 0;
                    if (hipMalloc((void **)&r->sp_rx_dev, want + want / 4) != hipSuccess) {
                        e.code = ONO_E_HIP; snprintf(e.msg, sizeof e.msg, "device buffer for a SparseGrad frame");
                        return false;
                    }
                    r->sp_rx_dev_cap = want + want / 4;
                }
                dev = r->sp_rx_dev;
                in.sparse_dev = true;
            }
        }
        in.bytes = (size_t)pay;
        need = 12 + (size_t)pay;
        have_hdr = true;
        return true;
    }

    // one recv(2); false (e set) on a socket or protocol error
    bool step(ono_ring *r, hipStream_t s, TcpErr &e) {
        uint8_t *p = have_hdr ? dst + (got - 12) : hdr + got;
        const size_t want = have_hdr ? need - got : 12 - got;
        ssize_t k = recv(r->fd_prev, p, want, MSG_DONTWAIT);
        if (k == 0) { e.code = ONO_E_IO; snprintf(e.msg, sizeof e.msg, "previous worker closed the connection"); return false; }
        if (k < 0) {
            if (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR) return true;
            e.code = ONO_E_IO; snprintf(e.msg, sizeof e.msg, "recv from previous worker: %s", strerror(errno));
            return false;
        }
        got += (size_t)k;
        if (!have_hdr && got == 12 && !header(r, e)) return false;
        if (have_hdr && dev) {  // complete pieces go up to HBM while the rest is on the socket
            const size_t blk = r->tcp_block, avail = got - 12, payload = need - 12;
            while (issued < avail && (avail - issued >= blk || avail == payload)) {
                const size_t c = std::min(blk, payload - issued);
                hipError_t he = hipMemcpyAsync(dev + issued, dst + issued, c, hipMemcpyHostToDevice, s);
                if (he != hipSuccess) {
                    e.code = ONO_E_HIP; snprintf(e.msg, sizeof e.msg, "H2D of a frame: %s", hipGetErrorString(he));
                    return false;
                }
                issued += c;
            }
        }
        return true;
    }
};

// Ships `out`, waiting for each D2H piece before sending the bytes it covers.
void tcp_send_frame(ono_ring *r, const Outgoing &out, const std::atomic<bool> &stop, TcpErr &e) {
    const size_t blk = r->tcp_block, total = 12 + out.payload;
    size_t sent = 0;
    for (size_t b = 0; sent < total; b++) {
        const size_t ready = out.pieces ? std::min(total, 12 + (b + 1) * blk) : total;
        if (out.pieces && b < out.pieces) {
            hipError_t he = hipEventSynchronize(r->tx_ev[b]);
            if (he != hipSuccess) {
                e.code = ONO_E_HIP; snprintf(e.msg, sizeof e.msg, "D2H of a frame: %s", hipGetErrorString(he));
                return;
            }
        }
        while (sent < ready)
            if (!tcp_wait(r, r->fd_next, POLLOUT, stop, e) || !tcp_send_some(r, out.frame, sent, ready, e)) return;
    }
}

// Small frames: one thread drives both directions from one poll loop (a
// thread hand-off costs more than the transfer).
int tcp_exchange_inline(ono_ring *r, const Outgoing &out, Incoming &in, hipStream_t s) {
    if (out.pieces) ONO_HIP(hipEventSynchronize(r->tx_ev[out.pieces - 1]));  // the whole payload is down
    const size_t total = 12 + out.payload;
    size_t sent = 0;
    TcpRecv rv(in);
    TcpErr e;
    const int spin = tcp_spin_us();
    if (spin > 0) {  // non-blocking calls first: most small frames are done before a poll would wake
        const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(spin);
        for (unsigned it = 0; sent < total || !rv.done(); it++) {
            if (sent < total && !tcp_send_some(r, out.frame, sent, total, e)) return set_error(e.code, "%s", e.msg);
            if (!rv.done() && !rv.step(r, s, e)) return set_error(e.code, "%s", e.msg);
            if ((it & 15) == 15) {
                if (r->aborted.load()) return set_error(ONO_E_ABORTED, "ring aborted");
                if (std::chrono::steady_clock::now() >= until) break;
            }
        }
    }
    while (sent < total || !rv.done()) {
        if (r->aborted.load()) return set_error(ONO_E_ABORTED, "ring aborted");
        struct pollfd p[2];
        int np = 0, is = -1, ir = -1;
        if (sent < total) { p[np] = {r->fd_next, POLLOUT, 0}; is = np++; }
        if (!rv.done()) { p[np] = {r->fd_prev, POLLIN, 0}; ir = np++; }
        int pr = poll(p, (nfds_t)np, kTcpPollMs);
        if (pr < 0 && errno != EINTR) return set_error(ONO_E_IO, "poll: %s", strerror(errno));
        if (pr <= 0) continue;
        if (is >= 0 && (p[is].revents & (POLLOUT | POLLERR | POLLHUP)) && !tcp_send_some(r, out.frame, sent, total, e))
            return set_error(e.code, "%s", e.msg);
        if (ir >= 0 && (p[ir].revents & (POLLIN | POLLERR | POLLHUP)) && !rv.step(r, s, e))
            return set_error(e.code, "%s", e.msg);
    }
    return ONO_OK;
}

// One hop: send `out` to next while receiving prev's frame (try_join!,
// worker_ring.rs:122-123).  The receive buffers are free: the caller
// synchronized the stream work that read them.
int tcp_exchange(ono_ring *r, const Outgoing &out, Incoming &in, hipStream_t s) {
    if (r->aborted.load()) return set_error(ONO_E_ABORTED, "ring aborted");
    if (out.payload <= kTcpInline && in.dense_bytes <= kTcpInline) return tcp_exchange_inline(r, out, in, s);
    std::atomic<bool> stop_send{false}, stop_recv{false};
    TcpErr es, er;
    std::thread sender([&] {
        tcp_send_frame(r, out, stop_send, es);
        if (es.code) stop_recv.store(true);
    });
    TcpRecv rv(in);
    while (!rv.done())
        if (!tcp_wait(r, r->fd_prev, POLLIN, stop_recv, er) || !rv.step(r, s, er)) {
            stop_send.store(true);
            break;
        }
    sender.join();
    // report the root cause, not the "other side failed" stop
    const TcpErr &e = (er.code && er.code != ONO_E_OTHER) ? er : (es.code && es.code != ONO_E_OTHER) ? es : er;
    if (e.code) return set_error(e.code, "%s", e.msg);
    return ONO_OK;
}

}  // namespace

namespace ono {

// The default sampler, run ahead by a helper thread.  Its draws depend only on the state and the chunk length
// (ono_sparse_sample_default), and a ring's pushes take their chunks in a fixed cyclic order (its round's
// pushes, then the next round's), so the helper draws the coming pushes' samples into a queue of kDepth slots
// — each in pinned memory and uploaded to HBM on the helper's own non-blocking stream — while the ring makes
// and sends its frames.  Round 5 drew one push ahead: a draw (16384 of 54,693 values, 64-bit modulo per
// index) plus its upload outlasts a config-1 hop, and the push waited ~30 us for it (ONO_TCP_TRACE,
// profiles/r06_s8_trace.txt).  A push whose state or length is not the queue's next (ono_ring_set_sparse reset
// the state, the first push) draws inline and re-plans the queue; a caller's sampler is never called ahead.
struct SampleAhead {
    static constexpr int kDepth = 4;
    struct Slot {
        uint64_t st_in = 0, st_out = 0;
        size_t len = 0, m = 0;
        uint32_t *buf = nullptr;   // pinned, kSampleMax indices
        uint32_t *dbuf = nullptr;  // the same draw in HBM
        uint32_t *offs = nullptr;  // pinned, kFuseOffs: the draw bucketed by 256-value block (len <= kFuseKeysMax)
        bool bucketed = false;
        bool ready = false, up = false;
        int rc = ONO_OK;
    };
    std::mutex mu;
    std::condition_variable cv;
    bool stop = false;
    Slot slot[kDepth];
    int head = 0, tail = 0, count = 0;  // slots [head, head + count) drawn or being drawn, in push order
    int held = -1;                      // the slot the ring's current push reads (freed at its next take)
    int drawing = 0;                    // draws in flight (their threads write their slots' buffers unlocked)
    uint64_t gen = 0;                   // a re-plan discards a draw in flight
    // the plan: the next draw's state, and the cyclic push lengths from plan_pos on
    bool planned = false;
    uint64_t plan_st = 0;
    std::vector<size_t> plan_len;
    size_t plan_pos = 0;
    int device = 0;
    hipStream_t ust = nullptr;  // (non-blocking: no implicit order with the ring's stream)
    bool upload = false;        // ONO_THR_HBM=1: each draw also goes up to HBM for the gather
    std::vector<std::thread> th;  // drawing threads (ONO_SAMPLER_THREADS, default 2)

    // The draw's indices reordered by 256-value block of the chunk (a counting sort: the threshold takes the
    // k-th of the sampled values, whatever their order) and offs[b] = the first in block b, offs[nb] = m
    static bool bucket_by_block(uint32_t *idx, size_t m, size_t L, uint32_t *offs, std::vector<uint32_t> &tmp) {
        const size_t nb = (L + kFuseBlock - 1) / kFuseBlock;
        if (nb + 1 > kFuseOffs) return false;
        std::fill(offs, offs + nb + 1, 0u);
        for (size_t j = 0; j < m; j++) offs[idx[j] / kFuseBlock + 1]++;
        for (size_t b = 0; b < nb; b++) offs[b + 1] += offs[b];
        tmp.assign(idx, idx + m);
        std::vector<uint32_t> pos(offs, offs + nb);
        for (size_t j = 0; j < m; j++) idx[pos[tmp[j] / kFuseBlock]++] = tmp[j];
        return true;
    }
    void loop() {
        std::unique_lock<std::mutex> lk(mu);
        (void)hipSetDevice(device);
        std::vector<uint32_t> tmp;
        for (;;) {
            cv.wait(lk, [&] { return stop || (planned && count + (held >= 0) < kDepth); });
            if (stop) return;
            // the next push that draws (a chunk of at most kSampleMax values is its own sample: no draw)
            size_t L = 0;
            for (size_t k = 0; k < plan_len.size(); k++) {
                L = plan_len[plan_pos % plan_len.size()];
                if (L > kSampleMax) break;
                plan_pos++;
            }
            if (L <= kSampleMax) {  // (no push of this ring ever draws)
                planned = false;
                continue;
            }
            const int q = tail;
            Slot &sl = slot[q];
            sl.st_in = plan_st;
            sl.len = L;
            sl.m = kSampleMax;
            sl.ready = false;
            tail = (tail + 1) % kDepth;
            count++;
            const uint64_t g = gen;
            uint64_t st = plan_st;
            // a draw of m indices advances splitmix64 by exactly m steps of its constant (one per index,
            // ono_sparse_sample_default), so the next draw's state is known before this one is made: the
            // drawing threads make the queue's draws side by side
            const uint64_t st_next = plan_st + (uint64_t)kSampleMax * 0x9E3779B97F4A7C15ULL;
            plan_st = st_next;
            plan_pos++;
            drawing++;
            uint32_t *b = sl.buf, *db = sl.dbuf;
            lk.unlock();
            const auto t0 = std::chrono::steady_clock::now();
            const int e = ono_sparse_sample_default(&st, L, b, kSampleMax);
            const bool bk = e == ONO_OK && sl.offs && L <= kFuseKeysMax && bucket_by_block(b, kSampleMax, L, sl.offs, tmp);
            bool u = false;
            if (upload && e == ONO_OK && db && ust &&
                hipMemcpyAsync(db, b, kSampleMax * sizeof(uint32_t), hipMemcpyHostToDevice, ust) == hipSuccess)
                u = hipStreamSynchronize(ust) == hipSuccess;
            if (trace_on()) {
                g_hop_trace.draw_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                                           std::chrono::steady_clock::now() - t0).count();
                g_hop_trace.draws++;
            }
            lk.lock();
            drawing--;
            if (g != gen) {  // re-planned meanwhile: the slot was dropped (plan() waits for this draw to end)
                cv.notify_all();
                continue;
            }
            sl.st_out = st;
            sl.rc = e == ONO_OK && st != st_next ? ONO_E_OTHER : e;  // (never: the state's step is fixed)
            sl.up = u;
            sl.bucketed = bk;
            sl.ready = true;
            if (sl.rc != ONO_OK) planned = false;
            cv.notify_all();
        }
    }
    // the queue restarts at state st with the ring's cyclic push lengths from position pos
    void plan(uint64_t st, const std::vector<size_t> &lens, size_t pos) {
        std::unique_lock<std::mutex> lk(mu);
        // a draw still in flight writes its slot's buffers: with two drawing threads the re-planned queue could
        // hand that slot to the other one (or to a take) before it ends, so the re-plan waits for it
        gen++;  // (a draw ending meanwhile drops its result)
        planned = false;  // (and no new draw starts)
        cv.wait(lk, [&] { return drawing == 0; });
        head = tail = (held >= 0 ? (held + 1) % kDepth : 0);
        count = 0;
        plan_st = st;
        plan_len = lens;
        plan_pos = pos;
        planned = !lens.empty();
        cv.notify_all();
    }
    // the next push's draw for (st, L, mm) if the queue made it: *idx / *didx point at the slot (valid until
    // the next take), *st advanced, *in_hbm when the HBM copy is there.  The slot the previous push read is
    // freed first (its drop, which read the sample, has returned).
    bool take(uint64_t *st, size_t L, size_t mm, uint32_t **idx, uint32_t **didx, bool *in_hbm,
              uint32_t **offs = nullptr) {
        std::unique_lock<std::mutex> lk(mu);
        *in_hbm = false;
        if (offs) *offs = nullptr;
        if (held >= 0) {
            held = -1;
            cv.notify_all();
        }
        if (!count || slot[head].st_in != *st || slot[head].len != L || slot[head].m != mm) {
            if (trace_on()) g_hop_trace.misses++;
            return false;
        }
        Slot &sl = slot[head];
        if (!sl.ready && trace_on()) {
            const auto t0 = std::chrono::steady_clock::now();
            cv.wait(lk, [&] { return sl.ready; });
            g_hop_trace.wait_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                                       std::chrono::steady_clock::now() - t0).count();
            g_hop_trace.waits++;
        }
        cv.wait(lk, [&] { return sl.ready; });
        if (sl.rc != ONO_OK) return false;
        held = head;
        head = (head + 1) % kDepth;
        count--;
        *idx = sl.buf;
        *didx = sl.dbuf;
        *in_hbm = sl.up;
        if (offs && sl.bucketed) *offs = sl.offs;
        *st = sl.st_out;
        cv.notify_all();
        return true;
    }
};

void sample_ahead_free(SampleAhead *a) {
    if (!a) return;
    {
        std::lock_guard<std::mutex> lk(a->mu);
        a->stop = true;
        a->cv.notify_all();
    }
    for (auto &t : a->th)
        if (t.joinable()) t.join();
    for (auto &sl : a->slot) {
        if (sl.buf) (void)hipHostFree(sl.buf);
        if (sl.offs) (void)hipHostFree(sl.offs);
        if (sl.dbuf) (void)hipFree(sl.dbuf);
    }
    if (a->ust) (void)hipStreamDestroy(a->ust);
    delete a;
}

}  // namespace ono

namespace {

// the sample's buffers: pinned host (the sampler writes it), its device copy, the threshold slot
int alloc_sample(ono_ring *r) {
    if (r->sample_idx) return ONO_OK;
    DeviceGuard g(r->device);
    ONO_HIP(hipHostMalloc((void **)&r->sample_idx, kSampleMax * sizeof(uint32_t), hipHostMallocDefault));
    ONO_HIP(hipMalloc((void **)&r->sp_idx_dev, kSampleMax * sizeof(uint32_t)));
    ONO_HIP(hipMalloc((void **)&r->sp_t_dev, sizeof(float)));
    ONO_HIP(hipHostMalloc((void **)&r->sp_status, sizeof(uint64_t), hipHostMallocMapped | hipHostMallocCoherent));
    *r->sp_status = 0;
    return ONO_OK;
}

// splitmix64 (the default sampler's generator)
uint64_t sm_next(uint64_t &x) {
    x += 0x9E3779B97F4A7C15ULL;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

class TcpRing {
public:
    TcpRing(ono_ring *r, hipStream_t s) : r_(r), s_(s), n_(r->n), pos_(r->pos), zc_(r->zc[0] != nullptr) {}

    int pull_grads(float *res, float *grad) {
        return r_->sparse_r > 0.0f ? pull_sparse(res, grad) : pull_dense(res, grad);
    }

private:
    size_t off(int c) const { return r_->off[c]; }
    size_t len(int c) const { return r_->off[c + 1] - r_->off[c]; }
    int mod(int x) const { return ((x % n_) + n_) % n_; }
    // the f16 wire slot b holding chunk c (phase-matched to the chunk start)
    uint16_t *slot(int b, int c) const {
        return (zc_ ? reinterpret_cast<uint16_t *>(r_->zc[b] + 16) : static_cast<uint16_t *>(r_->wbuf[b])) +
               ph(off(c));
    }

    // everything enqueued on the ring's stream so far has run (a spin on a host-mapped word)
    // (the sparse hop's waits; a dense zero-copy hop synchronizes the stream instead: config-1 rings,
    // ms per round spin / synchronize, one box: dense 2 workers 0.106 / 0.101, 4 workers 0.250 / 0.243,
    // sparse r = 0.1 0.243 / 0.265 — profiles/r05_s51_wait_ab.txt)
    int wait() {
        if (++r_->tcp_epoch == 0) r_->tcp_epoch = 1;
        ONO_HIP(stream_wait(s_, r_->tcp_word, r_->tcp_word_dev, r_->tcp_epoch));
        return ONO_OK;
    }
    // D2H of `bytes` from device `src` into r->tx + 12: one piece is copied and waited for here
    // (pieces = 0: the frame is complete); a larger frame goes in pieces with events, which the sender
    // waits for one by one while the rest is still coming down
    int stage_down(const void *src, size_t bytes, size_t &pieces) {
        const size_t blk = r_->tcp_block;
        if (bytes <= blk) {
            pieces = 0;
            if (bytes) ONO_HIP(hipMemcpyAsync(r_->tx + 12, src, bytes, hipMemcpyDeviceToHost, s_));
            return wait();
        }
        pieces = (bytes + blk - 1) / blk;
        int rc = ensure_tx_events(r_, pieces);
        if (rc) return rc;
        for (size_t b = 0; b < pieces; b++) {
            const size_t o = b * blk, c = std::min(blk, bytes - o);
            ONO_HIP(hipMemcpyAsync(r_->tx + 12 + o, static_cast<const uint8_t *>(src) + o, c, hipMemcpyDeviceToHost,
                                   s_));
            ONO_HIP(hipEventRecord(r_->tx_ev[b], s_));
        }
        return ONO_OK;
    }
    // the receive buffers are free once the stream work before this hop ran (a one-piece frame was
    // waited for whole in stage_down)
    int settle(const Outgoing &o) {
        if (o.pieces) ONO_HIP(hipEventSynchronize(r_->tx_ev[0]));  // everything enqueued before the D2H
        return ONO_OK;
    }

    // Base serializer: DenseGrad of the f16 payload already in slot(b, c)
    int out_dense(int b, int c, Outgoing &o) {
        const size_t bytes = 2 * len(c);
        o = Outgoing{};
        o.payload = bytes;
        if (zc_) {  // the codec kernel wrote the payload in place; the header goes just before it
            uint8_t *f = reinterpret_cast<uint8_t *>(slot(b, c)) - 12;
            put_header(f, bytes, KIND_DENSE);
            o.frame = f;
            if (dn_sig_) {  // the stream's last kernel signals its end (dense_done)
                ONO_HIP(stream_spin(s_, r_->tcp_word + 1, dn_sig_));
                dn_sig_ = 0;
            } else {
                ONO_HIP(hipStreamSynchronize(s_));
            }
            return ONO_OK;
        }
        int rc = grow_pinned(&r_->tx, &r_->tx_cap, 12 + bytes);
        if (rc) return rc;
        put_header(r_->tx, bytes, KIND_DENSE);
        o.frame = r_->tx;
        if ((rc = stage_down(slot(b, c), bytes, o.pieces))) return rc;
        return settle(o);
    }

    // SparseCapable serializer, Compressor::compress (compressor.rs:71-98):
    // t = calculate_threshold(chunk, r), the grad_drop stream of the chunk;
    // a SparseGrad if the stream is at most 2 bytes per value (:79), else the
    // DenseGrad of f16(chunk) (:84-89) — encoded into slot(0, c) and, in the
    // scatter (zero_chunk), fused with the dense branch's chunks[i].fill(0.0)
    // (worker_ring.rs:133).  sparse = push_grad's Some(t) / None.
    int out_sparse(float *chunk, int c, bool zero_chunk, float &t, bool &sparse, Outgoing &o) {
        const size_t L = len(c);
        (void)t;  // (the threshold stays on the device: r_->sp_t_dev)
        const size_t k_push = push_k_++;
        int rc = codec([&] { return threshold(chunk, L, k_push); });
        if (rc) return rc;
        if (clk_) clk_->step(0);
        const size_t cap = ono_sparse_max_bytes(L);
        const bool zc = cap <= kSparseZeroCopy;
        uint8_t *dst = nullptr;
        if (zc) {  // payload at +16 (the header's 12 bytes just before it), coherent: the device writes it
            if ((rc = grow_pinned(&r_->sp_tx, &r_->sp_tx_cap, 16 + cap, hipHostMallocCoherent))) return rc;
            dst = r_->sp_tx + 16;
        } else {
            if (r_->sp_dev_cap < cap) {
                (void)hipFree(r_->sp_dev);
                r_->sp_dev = nullptr;
                r_->sp_dev_cap = 0;
                ONO_HIP(hipMalloc((void **)&r_->sp_dev, cap + 8));
                r_->sp_dev_cap = cap;
            }
            dst = r_->sp_dev;
        }
        size_t nb = 0;
        if ((rc = codec([&] { return sparse_drop_tdev(dst, cap, &nb, chunk, L, r_->sp_t_dev, s_); }))) return rc;
        if (clk_) clk_->step(1);
        sparse = nb <= 2 * L;
        if (!sparse) {
            if (zero_chunk) ONO_K(r_, s_, launch_encode_zero<uint16_t>(slot(0, c), chunk, L, s_));
            else ONO_K(r_, s_, launch_encode<uint16_t>(slot(0, c), chunk, L, s_));
            return out_dense(0, c, o);
        }
        o = Outgoing{};
        o.payload = nb;
        if (zc) {  // complete: the drop returned after its last write (and every earlier stream work) landed
            put_header(r_->sp_tx + 4, nb, KIND_SPARSE);
            o.frame = r_->sp_tx + 4;
            return ONO_OK;
        }
        if ((rc = grow_pinned(&r_->tx, &r_->tx_cap, 12 + nb))) return rc;
        put_header(r_->tx, nb, KIND_SPARSE);
        o.frame = r_->tx;
        if ((rc = stage_down(r_->sp_dev, nb, o.pieces))) return rc;
        return settle(o);
    }

    // The push's sample: the caller's sampler, or the default one's queue (or an inline draw when the queue
    // does not hold this push's), or none when the chunk is its own sample (at most SAMPLE_SIZE values).
    // *idx_dev: device-visible indices (NULL: none); *offs_dev: the draw's 256-value block offsets when the
    // queue bucketed it (launch_hop_post can then gather the keys); *m: the sample's size.
    int take_sample(size_t L, size_t k_push, uint32_t **idx_dev_out, const uint32_t **offs_dev_out, size_t *m_out) {
        const size_t m = std::min(L, kSampleMax);
        *m_out = m;
        *idx_dev_out = nullptr;
        *offs_dev_out = nullptr;
        bool sampled = false, in_hbm = false;
        uint32_t *idx_host = r_->sample_idx, *idx_hbm = nullptr, *offs_host = nullptr;
        if (r_->sampler) {
            if (r_->sampler(r_->sampler_ctx, L, r_->sample_idx, m) != 0)
                return set_error(ONO_E_OTHER, "the sampler failed for a chunk of %zu values", L);
            sampled = L > kSampleMax;
        } else if (L > kSampleMax) {
            if (!r_->ahead) {
                auto *a = new SampleAhead();
                a->device = r_->device;
                a->upload = thr_hbm();
                bool ok = hipStreamCreateWithFlags(&a->ust, hipStreamNonBlocking) == hipSuccess;
                for (auto &sl : a->slot)
                    ok = ok &&
                         hipHostMalloc((void **)&sl.buf, kSampleMax * sizeof(uint32_t), hipHostMallocDefault) ==
                             hipSuccess &&
                         hipHostMalloc((void **)&sl.offs, kFuseOffs * sizeof(uint32_t), hipHostMallocDefault) ==
                             hipSuccess &&
                         hipMalloc((void **)&sl.dbuf, kSampleMax * sizeof(uint32_t)) == hipSuccess;
                if (!ok) {
                    sample_ahead_free(a);
                    return set_error(ONO_E_HIP, "sample buffers");
                }
                static const int nthreads = [] {
                    const char *e = getenv("ONO_SAMPLER_THREADS");
                    const int v = e ? atoi(e) : 2;
                    return v < 1 ? 1 : v > SampleAhead::kDepth ? SampleAhead::kDepth : v;
                }();
                for (int t = 0; t < nthreads; t++) a->th.emplace_back([a] { a->loop(); });
                r_->ahead = a;
            }
            uint32_t *qi = nullptr, *qd = nullptr;
            const auto tk0 = std::chrono::steady_clock::now();
            const bool took = r_->ahead->take(&r_->sample_state, L, m, &qi, &qd, &in_hbm, &offs_host);
            if (trace_on()) {
                g_hop_trace.take_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                                           std::chrono::steady_clock::now() - tk0).count();
                g_hop_trace.takes++;
            }
            if (took) {
                idx_host = qi;
                idx_hbm = qd;
            } else {  // not the queue's next draw: drawn here, and the queue re-planned from the state after it
                int rc = ono_sparse_sample_default(&r_->sample_state, L, r_->sample_idx, m);
                if (rc) return rc;
                in_hbm = false;
                offs_host = nullptr;
                r_->ahead->plan(r_->sample_state, push_len_, k_push + 1);
            }
            sampled = true;
        }
        if (clk_) clk_->step(6);  // (the sample: taken from the queue or drawn here)
        if (sampled && r_->sampler)  // a caller's indices are checked; the default sampler's are in range
            for (size_t i = 0; i < m; i++)
                if (r_->sample_idx[i] >= L) return set_error(ONO_E_ARG, "sample index %u out of %zu", r_->sample_idx[i], L);
        if (!sampled) return ONO_OK;
        // the kernels read the pinned indices in place (an upload by the copy engine cost ~30 us of
        // cross-engine hand-off per push); the buffer is not rewritten before this push's drop returns — unless
        // the helper thread already put the draw in HBM, where the gather reads it
        if (in_hbm && thr_hbm()) *idx_dev_out = idx_hbm;
        else ONO_HIP(hipHostGetDevicePointer((void **)idx_dev_out, idx_host, 0));
        if (offs_host) ONO_HIP(hipHostGetDevicePointer((void **)offs_dev_out, offs_host, 0));
        return ONO_OK;
    }
    // calculate_threshold over the sample (take_sample), into r->sp_t_dev in stream order: the drop and the
    // masks read it there (no host round trip; the host never needs the value).  A push whose sample the
    // previous hop took early (pre_) uses it — and when that hop's add / copy gathered the keys, only the
    // select is launched.
    int threshold(const float *chunk, size_t L, size_t k_push) {
        if (pre_.on && pre_.k_push == k_push && pre_.L == L) {
            pre_.on = false;
            if (clk_) clk_->step(6);
            if (pre_.keys_ready) return sparse_select_keys_dev(r_->sp_t_dev, r_->sp_idx_dev, pre_.m, r_->sparse_r, s_);
            return sparse_threshold_dev(r_->sp_t_dev, chunk, L, pre_.idx_dev, r_->sp_idx_dev, pre_.m, r_->sparse_r, s_);
        }
        pre_.on = false;
        uint32_t *idx_dev = nullptr;
        const uint32_t *offs_dev = nullptr;
        size_t m = 0;
        int rc = take_sample(L, k_push, &idx_dev, &offs_dev, &m);
        if (rc) return rc;
        return sparse_threshold_dev(r_->sp_t_dev, chunk, L, idx_dev, r_->sp_idx_dev, m, r_->sparse_r, s_);
    }
    // The hop after its exchange, when the received values went into the chunk the next push sends
    // (cr): that push's sample taken now, and — when it comes bucketed — its keys gathered by the same launch
    // as the add / copy and the push's mask (launch_hop_post; ONO_TCP_FUSE_KEYS=0 keeps the gather launch).
    int hop_post(float *dst, const float *src, size_t k, int add, float *mg, size_t mn, int zero_kept, size_t L,
                 bool next_push) {
        static const bool fuse_keys = env_on("ONO_TCP_FUSE_KEYS");
        uint32_t *keys = nullptr;
        if (next_push && fuse_keys && !r_->sampler && L > kSampleMax && L <= kFuseKeysMax) {
            PreSample p;
            int rc = take_sample(L, push_k_, &p.idx_dev, &p.offs_dev, &p.m);
            if (rc) return rc;
            p.on = true;
            p.k_push = push_k_;
            p.L = L;
            p.keys_ready = p.idx_dev && p.offs_dev;
            if (p.keys_ready) keys = r_->sp_idx_dev;
            pre_ = p;
        }
        if (!keys && !mn) {  // nothing fused: the add or the copy alone
            if (add) ONO_K(r_, s_, launch_acc(dst, src, k, s_, true));
            else ONO_HIP(dev_copy(dst, src, k * sizeof(float), s_));
            return ONO_OK;
        }
        ONO_K(r_, s_, launch_hop_post(dst, src, k, add, mg, mn, r_->sp_t_dev, zero_kept, s_, L, pre_.idx_dev,
                                      pre_.offs_dev, keys));
        return ONO_OK;
    }
    struct PreSample {
        bool on = false, keys_ready = false;
        size_t k_push = 0, L = 0, m = 0;
        uint32_t *idx_dev = nullptr;
        const uint32_t *offs_dev = nullptr;
    };

    Incoming in_for(int c, int b) const {
        Incoming in;
        in.dense_bytes = 2 * len(c);
        if (zc_) {
            in.dense_host = reinterpret_cast<uint8_t *>(slot(b, c));
        } else {
            in.dense_host = r_->rx + 12;
            in.dense_dev = reinterpret_cast<uint8_t *>(slot(b, c));
        }
        return in;
    }
    int ensure_rx() {
        return grow_pinned(&r_->rx, &r_->rx_cap, 12 + 2 * (r_->maxc + 4));
    }
    // scratch of at least `elems` values at every 4-element phase
    int tmp(size_t elems) {
        if (r_->sp_tmp_cap >= elems + 4) return ONO_OK;
        (void)hipFree(r_->sp_tmp);
        r_->sp_tmp = nullptr;
        r_->sp_tmp_cap = 0;
        const size_t cap = std::max(elems, r_->maxc) + 4;
        ONO_HIP(hipMalloc((void **)&r_->sp_tmp, cap * sizeof(float)));
        r_->sp_tmp_cap = cap;
        return ONO_OK;
    }
    // phase-matched scratch for chunk c
    float *tmp_for(int c) const { return r_->sp_tmp + ph(off(c)); }

    // An incoming frame that is not a whole-chunk DenseGrad, as the reference
    // hands it to the hop (WorkerHandle::recv_event, handles/worker.rs:82-130):
    // its values in device memory, vals[0, k).  A non-gradient message fails
    // with recv_event's / the ring's error.  The scatter adds over the shorter
    // of the two lengths (the zip, worker_ring.rs:141-143); the gather needs
    // the hop's chunk length exactly (copy_from_slice, :200, panics on any other).
    int incoming(const Incoming &in, int c, bool gather, const float **vals, size_t *k) {
        const size_t L = len(c);
        if (in.kind != KIND_DENSE_OTHER && in.kind != KIND_SPARSE)
            return worker_event_check(in.kind, r_->sp_rx, in.bytes);
        if (in.kind == KIND_DENSE_OTHER) {
            const size_t m = in.bytes / 2;
            if (gather)
                return set_error(ONO_E_PROTO, "Received an invalid worker event (a gradient of %zu values for a chunk "
                                 "of %zu; the reference's copy_from_slice panics)", m, L);
            *k = std::min(m, L);
            int rc = tmp(L);
            if (rc) return rc;
            uint16_t *h = slot(1, c);  // free: the stream work that read it has run
            if (zc_) memcpy(h, r_->sp_rx, 2 * *k);
            else ONO_HIP(hipMemcpyAsync(h, r_->sp_rx, 2 * *k, hipMemcpyHostToDevice, s_));
            ONO_K(r_, s_, launch_decode_scale<uint16_t>(tmp_for(c), h, *k, 1.0f, s_));
            *vals = tmp_for(c);
            return ONO_OK;
        }
        uint64_t total = 0;  // SparseGrad: grad_lift_into resizes to the stream's total (protocol.rs:102-106)
        for (int q = 0; q < 8 && q < (int)in.bytes; q++) total |= (uint64_t)r_->sp_rx[q] << (8 * q);
        if (in.bytes >= 8 && gather && total != L)
            return set_error(ONO_E_PROTO, "Received an invalid worker event (a gradient of %llu values for a chunk "
                             "of %zu; the reference's copy_from_slice panics)", (unsigned long long)total, L);
        if (in.bytes >= 8 && total > (uint64_t(1) << 36))
            return set_error(ONO_E_IO, "sparse gradient of %llu values: capacity overflow", (unsigned long long)total);
        int rc = tmp(L);  // a frame's claimed total never sizes device memory
        if (rc) return rc;
        size_t got = 0;
        if (in.bytes >= 8 && total > L) {  // scatter: only [0, L) is added (the zip); validate all, keep L
            std::vector<float> h(L);
            rc = sparse_lift_prefix_host(r_->sp_rx, in.bytes, h.data(), L, &got);
            if (rc == ONO_E_PROTO) return set_error(ONO_E_IO, "%s", ono_last_error());
            if (rc) return rc;
            *k = std::min(got, L);
            ONO_HIP(hipMemcpyAsync(tmp_for(c), h.data(), *k * sizeof(float), hipMemcpyHostToDevice, s_));
            ONO_HIP(hipStreamSynchronize(s_));  // h is released on return
            *vals = tmp_for(c);
            return ONO_OK;
        }
        const size_t cap = in.bytes >= 8 ? (size_t)total : 0;
        rc = codec([&] { return lift(tmp_for(c), cap, &got, in.bytes, in.sparse_dev); });
        // a malformed stream is the lift's io::Error (protocol.rs:96-144) on the reference's recv_event
        if (rc == ONO_E_PROTO) return set_error(ONO_E_IO, "%s", ono_last_error());
        if (rc) return rc;
        *k = std::min(got, L);
        *vals = tmp_for(c);
        return ONO_OK;
    }

    // grad_lift_into of the received stream (r->sp_rx, pinned host): the stream-ordered lift
    // (ono_sparse_lift_dev_async: the pattern path, one or two launches) reads the frame in place through
    // its device mapping — no copy of the frame into HBM in the hop; a stream it refuses (not drop-shaped,
    // malformed) goes up to HBM and to the blocking device lift, which parses anything and returns the
    // reference's errors.  *got = the stream's total.  The one-launch lift stores the ring's word itself when
    // it is done (no signal launch behind it; ONO_LIFT_SIGNAL=0 keeps the signal kernel, measurement).
    // (Round 6 also measured the hop pipelined — the add / copy and the next push's threshold enqueued behind
    // a lift not waited for, replayed after a refusal: no gain, profiles/r06_s20, r06_s22, r06_s23)
    int lift(float *out, size_t cap, size_t *got, size_t nbytes, bool in_dev) {
        if (nbytes < 8) return ono_sparse_lift(out, cap, got, r_->sp_rx, nbytes, s_);
        const uint8_t *src = in_dev ? r_->sp_rx_dev : nullptr;
        if (!in_dev) {
            ONO_HIP(hipHostGetDevicePointer((void **)&src, r_->sp_rx, 0));
            if (!lift_pinned()) {
                int rc = up_frame(nbytes);
                if (rc) return rc;
                src = r_->sp_rx_dev;
            }
        }
        uint64_t total = 0;
        memcpy(&total, r_->sp_rx, 8);  // (little endian, protocol.rs:102-106)
        uint64_t ticket = 0;
        LiftDone d;
        static const bool in_kernel = env_on("ONO_LIFT_SIGNAL");
        if (in_kernel) {
            if (++r_->tcp_epoch == 0) r_->tcp_epoch = 1;
            d.word_host = lift_word();
            d.word_dev = r_->tcp_word_dev + 2;
            d.sig = r_->tcp_epoch;
        }
        const auto t0 = std::chrono::steady_clock::now();
        int rc = lift_dev_async(out, cap, src, nbytes, r_->sp_status, &ticket, s_, in_kernel ? &d : nullptr);
        if (rc) return rc;
        const auto t1 = std::chrono::steady_clock::now();
        if (d.in_kernel) ONO_HIP(stream_spin(s_, lift_word(), d.sig));
        else if ((rc = wait())) return rc;
        if (trace_on()) {
            g_hop_trace.lifts++;
            g_hop_trace.lift_call_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
            g_hop_trace.lift_wait_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                                            std::chrono::steady_clock::now() - t1).count();
        }
        if (__atomic_load_n(r_->sp_status, __ATOMIC_ACQUIRE) != ticket) {
            *got = (size_t)total;
            return ONO_OK;
        }
        return lift_fallback(out, cap, got, nbytes, in_dev);
    }
    // the received frame's whole words into r->sp_rx_dev by the library's copy kernel (in stream order)
    int up_frame(size_t nbytes) {
        const uint8_t *src = nullptr;
        ONO_HIP(hipHostGetDevicePointer((void **)&src, r_->sp_rx, 0));
        const size_t words = (nbytes + 3) & ~size_t(3);
        if (r_->sp_rx_dev_cap < words) {
            (void)hipFree(r_->sp_rx_dev);
            r_->sp_rx_dev = nullptr;
            r_->sp_rx_dev_cap = 0;
            const size_t c2 = std::max(words, ono_sparse_max_bytes(r_->maxc) + 8);
            ONO_HIP(hipMalloc((void **)&r_->sp_rx_dev, c2));
            r_->sp_rx_dev_cap = c2;
        }
        ONO_HIP(dev_copy(r_->sp_rx_dev, src, words, s_));
        return ONO_OK;
    }
    // a stream the pattern path refused: the blocking device lift from HBM (it parses anything, with the
    // reference's errors); a frame lifted from its pinned mapping goes up first
    int lift_fallback(float *out, size_t cap, size_t *got, size_t nbytes, bool in_dev) {
        if (!in_dev && lift_pinned()) {
            int rc = up_frame(nbytes);
            if (rc) return rc;
        }
        return ono_sparse_lift_dev(out, cap, got, r_->sp_rx_dev, nbytes, s_);
    }

    // The dense hop's last kernel before a zero-copy frame leaves, launched to signal its own end
    // (KernelDone): out_dense then spins on the ring's word 1 instead of synchronizing the stream, whose
    // wake-up after the kernel was most of the ~15 us a config-1 frame took to be ready (r06_s42);
    // ONO_TCP_DENSE_SIGNAL=0 keeps the synchronisation (measurement).  NULL when not zero-copy.
    KernelDone *dense_done() {
        static const bool on = env_on("ONO_TCP_DENSE_SIGNAL");
        dn_sig_ = 0;
        if (!on || !zc_) return nullptr;
        if (!r_->dn_arrive) {
            if (hipMalloc((void **)&r_->dn_arrive, 128) != hipSuccess) return nullptr;
            if (hipMemsetAsync(r_->dn_arrive, 0, 128, s_) != hipSuccess) return nullptr;
            r_->dn_base = 0;
        }
        if (++r_->tcp_epoch == 0) r_->tcp_epoch = 1;
        *(volatile uint64_t *)(r_->tcp_word + 1) = 0;
        kd_.word_dev = r_->tcp_word_dev + 1;
        kd_.arrive = r_->dn_arrive;
        kd_.base = r_->dn_base;
        kd_.sig = r_->tcp_epoch;
        return &kd_;
    }
    // after a launch given dense_done(): the counter's new base, and the tag out_dense waits for
    void dense_launched(const KernelDone *d) {
        if (!d) return;
        r_->dn_base = d->base;
        dn_sig_ = d->sig;
    }

    // ---- Base serializer: the fused codec kernels (ono_ring.cpp's hop ring);
    // an incoming frame that is not a whole-chunk DenseGrad is taken apart first.
    int pull_dense(float *res, float *grad) {
        int rc = ensure_rx();
        if (rc) return rc;
        const float fn = (float)n_;
        // scatter: out slot 0, in slot 1
        {
            KernelDone *d = dense_done();
            ONO_K(r_, s_, launch_encode_zero<uint16_t>(slot(0, pos_), res + off(pos_), len(pos_), s_, d));
            dense_launched(d);
        }
        for (int st = 0; st < n_ - 1; st++) {
            const int cs = mod(pos_ - st), cr = mod(pos_ - st - 1);
            Outgoing o;
            Incoming in = in_for(cr, 1);
            HopClock clk;  // (ONO_TCP_TRACE: "drop" = the frame ready, "add" = the hop's kernel launched)
            if ((rc = out_dense(0, cs, o))) return rc;
            clk.step(1);
            if ((rc = xchg(o, in))) return rc;
            clk.step(3);
            const bool last = st == n_ - 2;
            if (in.kind == KIND_DENSE) {
                KernelDone *d = dense_done();
                if (!last)
                    ONO_K(r_, s_, launch_add_encode_zero<uint16_t>(slot(0, cr), res + off(cr), slot(1, cr), len(cr), s_,
                                                                   d));
                else
                    ONO_K(r_, s_, launch_add_finish<uint16_t>(grad + off(cr), slot(0, cr), res + off(cr), slot(1, cr),
                                                              len(cr), fn, s_, d));
                dense_launched(d);
                clk.step(5);
                clk.done();
                continue;
            }
            const float *v = nullptr;
            size_t k = 0;
            if ((rc = incoming(in, cr, false, &v, &k))) return rc;
            ONO_K(r_, s_, launch_acc(res + off(cr), v, k, s_, true));  // :141-143
            if (!last) {
                ONO_K(r_, s_, launch_encode_zero<uint16_t>(slot(0, cr), res + off(cr), len(cr), s_));
            } else {  // grad = x / n, the f16 message, residual = 0 (add_finish without the add)
                const float *ins[1] = {res + off(cr)};
                ONO_K(r_, s_, launch_direct<uint16_t>(grad + off(cr), slot(0, cr), ins, 1, len(cr), fn, true, s_));
            }
        }
        // gather: forward what arrived, alternate the two slots
        int bo = 0, bi = 1;
        for (int j = 0; j < n_ - 1; j++) {
            const int cs = mod(pos_ + 1 - j), cr = mod(pos_ - j);
            Outgoing o;
            Incoming in = in_for(cr, bi);
            HopClock clk;
            if ((rc = out_dense(bo, cs, o))) return rc;
            clk.step(1);
            if ((rc = xchg(o, in))) return rc;
            clk.step(3);
            if (in.kind == KIND_DENSE) {
                KernelDone *d = j + 1 < n_ - 1 ? dense_done() : nullptr;  // (a next gather frame waits for it)
                ONO_K(r_, s_, launch_decode_scale<uint16_t>(grad + off(cr), slot(bi, cr), len(cr), fn, s_, d));
                dense_launched(d);
                clk.step(5);
                clk.done();
            } else {  // :200 copies the received chunk; the next hop forwards its f16 image
                const float *v = nullptr;
                size_t k = 0;
                if ((rc = incoming(in, cr, true, &v, &k))) return rc;
                ONO_K(r_, s_, launch_scale_zero(grad + off(cr), v, len(cr), fn, nullptr, s_));
                ONO_K(r_, s_, launch_encode<uint16_t>(slot(bi, cr), v, len(cr), s_));
            }
            std::swap(bo, bi);
        }
        return ONO_OK;
    }

    // ---- SparseCapable serializer (worker_ring.rs:112-204 with the branches
    // push_grad's result selects): unfused — each push's threshold is taken
    // over the chunk as the reference holds it, so the division by n waits
    // for the end (:101-105).
    int pull_sparse(float *res, float *grad) {
        int rc = ensure_rx();
        if (rc) return rc;
        // the chunk lengths of this round's pushes in order (the next round's first follows the last)
        push_len_.clear();
        for (int st = 0; st < n_ - 1; st++) push_len_.push_back(len(mod(pos_ - st)));
        for (int j = 0; j < n_ - 1; j++) push_len_.push_back(len(mod(pos_ + 1 - j)));
        push_k_ = 0;
        float t = 0.0f;
        bool sparse = false;
        for (int st = 0; st < n_ - 1; st++) {  // scatter (:112-147)
            const int cs = mod(pos_ - st), cr = mod(pos_ - st - 1);
            Outgoing o;
            Incoming in = in_for(cr, 1);
            // :126-132 sent values leave; a dense push (:133) zeroed the chunk in its encoder (mask_at: where)
            const int mat = mask_at();
            HopClock clk;
            clk_ = &clk;
            if ((rc = out_sparse(res + off(cs), cs, true, t, sparse, o))) return rc;
            if (mat == MASK_EARLY && sparse && (rc = mask(res + off(cs), len(cs), 1))) return rc;
            clk.step(2);
            if ((rc = xchg(o, in))) return rc;
            clk.step(3);
            if (mat == MASK_LATE && sparse && (rc = mask(res + off(cs), len(cs), 1))) return rc;
            const bool fuse = mat == MASK_FUSED && sparse;
            if (in.kind == KIND_DENSE) {
                if (fuse && (rc = mask(res + off(cs), len(cs), 1))) return rc;
                ONO_K(r_, s_, launch_decode_add<uint16_t>(res + off(cr), slot(1, cr), len(cr), s_));
            } else {
                const float *v = nullptr;
                size_t k = 0;
                if ((rc = incoming(in, cr, false, &v, &k))) return rc;
                clk.step(4);
                // :141-143, with the push's mask; the next push sends chunk cr (the next scatter hop's, or the
                // gather's first: the owned chunk, which the last scatter hop received)
                if (mat == MASK_FUSED) {
                    if ((rc = hop_post(res + off(cr), v, k, 1, res + off(cs), fuse ? len(cs) : 0, 1, len(cr),
                                       st < n_ - 2 || mod(pos_ + 1) == cr)))
                        return rc;
                } else {
                    ONO_K(r_, s_, launch_acc(res + off(cr), v, k, s_, true));
                }
            }
            clk.step(5);
            clk.done();
            clk_ = nullptr;
        }
        const int own = mod(pos_ + 1);  // gather (:155-204)
        ONO_HIP(dev_copy(grad + off(own), res + off(own), len(own) * sizeof(float), s_));  // :166
        for (int j = 0; j < n_ - 1; j++) {
            const int cs = mod(pos_ + 1 - j), cr = mod(pos_ - j);
            Outgoing o;
            Incoming in = in_for(cr, 1);
            const int mat = mask_at();
            HopClock clk;
            clk_ = &clk;
            if ((rc = out_sparse(grad + off(cs), cs, false, t, sparse, o))) return rc;
            if (mat == MASK_EARLY && sparse && (rc = mask(grad + off(cs), len(cs), 0))) return rc;
            clk.step(2);
            if ((rc = xchg(o, in))) return rc;
            clk.step(3);
            // :177-190: a sparse push keeps only the sent values; the owned residual stays (:178-184 commented out)
            if (mat == MASK_LATE && sparse && (rc = mask(grad + off(cs), len(cs), 0))) return rc;
            if (!sparse && j == 0) ONO_HIP(dev_zero(res + off(own), len(own) * sizeof(float), s_));  // :191-193
            const bool fuse = mat == MASK_FUSED && sparse;
            if (in.kind == KIND_DENSE) {
                if (fuse && (rc = mask(grad + off(cs), len(cs), 0))) return rc;
                ONO_K(r_, s_, launch_decode_scale<uint16_t>(grad + off(cr), slot(1, cr), len(cr), 1.0f, s_));
            } else {
                const float *v = nullptr;
                size_t k = 0;
                if ((rc = incoming(in, cr, true, &v, &k))) return rc;
                clk.step(4);
                // :200, with the push's mask; the next gather push (if any this round) sends chunk cr
                if (mat == MASK_FUSED) {
                    if ((rc = hop_post(grad + off(cr), v, len(cr), 0, grad + off(cs), fuse ? len(cs) : 0, 0, len(cr),
                                       j + 1 <= n_ - 2)))
                        return rc;
                } else {
                    ONO_HIP(dev_copy(grad + off(cr), v, len(cr) * sizeof(float), s_));
                }
            }
            clk.step(5);
            clk.done();
            clk_ = nullptr;
        }
        ONO_K(r_, s_, launch_scale_zero(grad, grad, r_->size, (float)n_, nullptr, s_));  // :101-105
        return ONO_OK;
    }

    int xchg(const Outgoing &o, Incoming &in) {
        return timed(r_, s_, ONO_PHASE_RCCL, [&]() -> int { return tcp_exchange(r_, o, in, s_); });
    }
    // the sparse codec's calls, as a phase of their own (ono_ring_timing_phases)
    template <class F> int codec(F &&f) { return timed(r_, s_, ONO_PHASE_SPARSE_CODEC, f); }
    // worker_ring.rs:126-132 (zero_kept) / :177-190, with the push's threshold where the device left it
    int mask(float *g, size_t n, int zero_kept) {
        return codec([&]() -> int {
            ONO_HIP(launch_sparse_mask_tdev(g, n, r_->sp_t_dev, zero_kept, s_));
            return ONO_OK;
        });
    }

    uint64_t *lift_word() const { return r_->tcp_word + 2; }  // (the in-kernel completion of a waited lift)

    ono_ring *r_;
    hipStream_t s_;
    int n_, pos_;
    bool zc_;
    std::vector<size_t> push_len_;
    size_t push_k_ = 0;
    HopClock *clk_ = nullptr;  // (ONO_TCP_TRACE: the hop in progress)
    PreSample pre_;            // the next push's sample, taken by the hop before it
    KernelDone kd_;            // the dense hop's signalling launch (dense_done)
    uint32_t dn_sig_ = 0;      // its tag, until out_dense has waited for it
};

}  // namespace

namespace ono {
int tcp_pull_grads(ono_ring *r, float *res, float *grad, hipStream_t s) {
    TcpRing t(r, s);
    return t.pull_grads(res, grad);
}
}  // namespace ono

extern "C" {

// The reference's ring over its own TCP connections (builder.rs:272-311 hands
// the worker an accepted `prev` and a connected `next` stream): f16 wire, hop
// schedule, the arithmetic in HBM, the frames on the caller's sockets.
int ono_ring_create_tcp(ono_ring **out, int pos, int nranks, size_t size, int device, int fd_prev,
                        int fd_next) {
    if (!out) return set_error(ONO_E_ARG, "out is NULL");
    *out = nullptr;
    if (nranks < 1 || pos < 0 || pos >= nranks) return set_error(ONO_E_ARG, "pos=%d nranks=%d", pos, nranks);
    if (size < (size_t)nranks)
        return set_error(ONO_E_SIZE, "bucket of %zu elements cannot be split over %d ranks", size, nranks);
    if (nranks > 1 && (fd_prev < 0 || fd_next < 0)) return set_error(ONO_E_ARG, "sockets required for nranks > 1");
    // reuse the common allocation path (nranks == 1 needs neither sockets nor an id)
    static const uint8_t no_uid[ONO_UID_BYTES] = {0};
    int rc = ono_ring_create(out, 0, 1, size, device, no_uid, ONO_WIRE_F16);
    if (rc) return rc;
    ono_ring *r = *out;
    if ((rc = alloc_sample(r))) {
        ono_ring_destroy(r);
        *out = nullptr;
        return rc;
    }
    if (nranks == 1) return ONO_OK;
    *out = nullptr;
    r->n = nranks;
    r->pos = pos;
    r->off = split_chunks(size, (size_t)nranks);
    r->maxc = r->off[1] - r->off[0];
    r->algo = ONO_ALGO_HOPS;
    r->fd_prev = fd_prev;
    r->fd_next = fd_next;
    DeviceGuard g(device);
    hipError_t e;
    for (int b = 0; b < 2; b++)
        if ((e = hipMalloc(&r->wbuf[b], (r->maxc + 4) * sizeof(float))) != hipSuccess) {
            ono_ring_destroy(r);
            return hip_error(e, "wire buffer allocation", __FILE__, __LINE__);
        }
    // zero-copy frames up to ONO_TCP_ZEROCOPY KiB of payload (default 256; 0 = off)
    const char *zc_env = getenv("ONO_TCP_ZEROCOPY");
    const size_t zc_max = zc_env ? (size_t)atol(zc_env) << 10 : kTcpInline;
    if (2 * (r->maxc + 4) <= zc_max)
        for (int b = 0; b < 2; b++)
            if ((e = hipHostMalloc((void **)&r->zc[b], 16 + 2 * (r->maxc + 4), hipHostMallocCoherent)) != hipSuccess) {
                ono_ring_destroy(r);
                return hip_error(e, "zero-copy frame allocation", __FILE__, __LINE__);
            }
    r->tcp_block = tcp_block_bytes();
    // (word 0: the hops' waits; word 2: the SparseCapable hop's lift completion)
    if ((e = hipHostMalloc((void **)&r->tcp_word, 4 * sizeof(uint64_t), hipHostMallocMapped | hipHostMallocCoherent)) !=
            hipSuccess ||
        (e = hipHostGetDevicePointer((void **)&r->tcp_word_dev, r->tcp_word, 0)) != hipSuccess) {
        ono_ring_destroy(r);
        return hip_error(e, "TCP ring wait word", __FILE__, __LINE__);
    }
    if ((rc = grow_pinned(&r->tx, &r->tx_cap, 12 + 2 * (r->maxc + 4))) ||
        (rc = grow_pinned(&r->rx, &r->rx_cap, 12 + 2 * (r->maxc + 4))) ||
        (rc = ensure_tx_events(r, (2 * (r->maxc + 4) + r->tcp_block - 1) / r->tcp_block))) {
        ono_ring_destroy(r);
        return rc;
    }
    *out = r;
    return ONO_OK;
}

int ono_ring_set_sparse(ono_ring *r, float ratio, uint64_t seed) {
    if (!r) return set_error(ONO_E_ARG, "ring is NULL");
    if (!(ratio == 0.0f || (ratio > 0.0f && ratio <= 1.0f)))
        return set_error(ONO_E_ARG, "ratio %g: SparseCapable keeps a fraction in (0, 1], 0 = the Base serializer",
                         (double)ratio);
    if (ratio > 0.0f && r->n > 1 && r->fd_next < 0)
        return set_error(ONO_E_ARG, "the SparseCapable serializer is a TCP-wire format: TCP rings only");
    std::lock_guard<std::mutex> lk(r->mu);
    if (int rc = alloc_sample(r)) return rc;
    // the SparseGrad receive frame at the size no sparse push exceeds (a stream above 2 bytes per value goes
    // dense: compressor.rs:79), pinned once here rather than re-pinned as the hops' frames grow
    if (ratio > 0.0f && r->fd_prev >= 0) {
        DeviceGuard g(r->device);
        if (int rc = grow_pinned(&r->sp_rx, &r->sp_rx_cap, 2 * (r->maxc + 4) + 64)) return rc;
    }
    r->sparse_r = ratio;
    r->sample_state = seed;
    return ONO_OK;
}

int ono_ring_set_sampler(ono_ring *r, ono_sample_fn fn, void *ctx) {
    if (!r) return set_error(ONO_E_ARG, "ring is NULL");
    std::lock_guard<std::mutex> lk(r->mu);
    r->sampler = fn;
    r->sampler_ctx = ctx;
    return ONO_OK;
}

// Floyd's algorithm over a splitmix64 stream: `amount` distinct indices of
// [0, len), in draw order.  Not rand 0.9.4's index::sample (StdRng is ChaCha12
// and is not restated here): it is the deterministic stand-in both this
// library and the CPU oracle use when no sampler is installed.
int ono_sparse_sample_default(uint64_t *state, size_t len, uint32_t *idx, size_t amount) {
    if (!state || (amount && !idx)) return set_error(ONO_E_ARG, "NULL argument");
    if (len > 0xFFFFFFFFull) return set_error(ONO_E_ARG, "sample indices are u32");
    if (amount > len) return set_error(ONO_E_ARG, "sample of %zu from %zu values", amount, len);
    if (amount == len) {  // the whole chunk: no draws
        for (size_t i = 0; i < len; i++) idx[i] = (uint32_t)i;
        return ONO_OK;
    }
    // membership as a bitmap over [0, len) (thread-local, cleared through the drawn indices afterwards):
    // the same draws and the same indices as a hash set, without its allocation and probing (round 5:
    // the set took 579 us of a 54,693-value push, most of a config-1 SparseCapable round)
    thread_local std::vector<uint64_t> bits;
    if (bits.size() < (len + 63) / 64) bits.assign((len + 63) / 64, 0);
    size_t c = 0;
    for (size_t j = len - amount; j < len; j++) {
        const uint32_t t = (uint32_t)(sm_next(*state) % (uint64_t)(j + 1));
        const uint32_t x = (bits[t >> 6] >> (t & 63)) & 1u ? (uint32_t)j : t;
        bits[x >> 6] |= 1ull << (x & 63);
        idx[c++] = x;
    }
    for (size_t i = 0; i < c; i++) bits[idx[i] >> 6] = 0;
    return ONO_OK;
}

}  // extern "C"
