// ono_internal.h — shared internals of libono_reduce.so (not part of the ABI).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ono_reduce.h"

namespace ono {

// Records a thread-local error message and returns `code`.
int set_error(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
int hip_error(hipError_t e, const char *what, const char *file, int line);
// WorkerHandle::recv_event's verdict on a frame of this kind (ono_msg.cpp):
// ONO_OK for a gradient (kinds 1-4), else the reference's error class
int worker_event_check(uint32_t kind, const uint8_t *payload, size_t n);

#define ONO_HIP(expr)                                                                  \
    do {                                                                               \
        hipError_t ono_e_ = (expr);                                                    \
        if (ono_e_ != hipSuccess) return ::ono::hip_error(ono_e_, #expr, __FILE__, __LINE__); \
    } while (0)

// Division by a run-time divisor d, bit-exact with IEEE `x / d`:
//  NONE  d == 1 (the reference skips the division, param_manager.rs:183-188)
//  RECIP d = 2^k: x * 2^-k is the same single rounding of the same real value
//  DIV   everything else: correctly rounded v_div sequence
enum ScaleMode { SCALE_NONE = 0, SCALE_RECIP = 1, SCALE_DIV = 2 };
struct Scale {
    ScaleMode mode;
    float v;
};
Scale make_scale(float divisor);

// split_chunks (worker/src/middlewares/mod.rs:15-59): offsets of min(len, n) chunks
std::vector<size_t> split_chunks(size_t len, size_t n);
inline size_t ph(size_t off) { return off & 3u; }  // phase-match wire slots to chunk starts

// Events that order a kernel's output before a copy on another stream (D2H by
// a DMA engine, which reads memory past the GPU's L2): recorded with an
// explicit system-scope release, so the kernel's dirty L2 lines are written
// back before the copy starts whatever the runtime's default release scope.
// ONO_COPY_EVENT_RELEASE=default leaves the scope to the runtime (measurement).
inline unsigned copy_event_flags() {
    static const unsigned f = [] {
        const char *e = getenv("ONO_COPY_EVENT_RELEASE");
        return e && !strcmp(e, "default") ? (unsigned)hipEventDisableTiming
                                          : (unsigned)(hipEventDisableTiming | hipEventReleaseToSystem);
    }();
    return f;
}

// ---- kernel launchers (ono_kernels.hip); return hipSuccess or the launch error
hipError_t launch_sum_scale(float *out, const float *const *ins, int k, size_t n, float divisor,
                            hipStream_t s);
// keep: the accumulator is re-read soon (the ring's residual): cacheable loads
hipError_t launch_acc(float *acc, const float *in, size_t n, hipStream_t s, bool keep = false);
hipError_t launch_scale_zero(float *dst, const float *src, size_t n, float divisor, float *zero,
                             hipStream_t s);
hipError_t launch_synth(float *out, size_t n, uint64_t seed, uint64_t rank, size_t offset,
                        hipStream_t s);
// The TCP ring's SparseCapable push in stream order (ono_sparse.hip): the
// threshold of the sample (idx: the m indices in device memory or a pinned
// host buffer the kernel reads in place, keys: m device words of scratch; or
// idx NULL = the whole chunk) into t_dev, the drop (blocking for its length,
// as ono_sparse_drop) and the masks reading the threshold there.
int sparse_threshold_dev(float *t_dev, const float *g, size_t n, const uint32_t *idx, uint32_t *keys, size_t m, float r,
                         hipStream_t s);
int sparse_drop_tdev(uint8_t *buf, size_t cap, size_t *nbytes, const float *g, size_t n, const float *t_dev,
                     hipStream_t s);
hipError_t launch_sparse_mask_tdev(float *g, size_t n, const float *t_dev, int zero_kept, hipStream_t s);
// one launch: dst[0, k) += src (add) or = src (copy), and the mask of mg[0, mn) (sp_mask's zero_kept form)
// with the threshold at t_dev — the SparseCapable hop's work after its exchange; keys != NULL: also the keys
// |dst[idx[j]]| of the next push's sample (dst, L values), idx bucketed by 256-value blocks (offs: L / 256 + 1)
hipError_t launch_hop_post(float *dst, const float *src, size_t k, int add, float *mg, size_t mn, const float *t_dev,
                           int zero_kept, hipStream_t s, size_t L = 0, const uint32_t *idx = nullptr,
                           const uint32_t *offs = nullptr, uint32_t *keys = nullptr);
// the threshold's select alone over m keys already in device memory (launch_hop_post gathered them)
int sparse_select_keys_dev(float *t_dev, const uint32_t *keys, size_t m, float r, hipStream_t s);
// Wait for everything enqueued on s so far by spinning on a host-mapped word
// that a one-lane kernel sets to `epoch` (a stream synchronisation's wake-up
// costs several microseconds more; used on the TCP ring's hops).
hipError_t stream_wait(hipStream_t s, uint64_t *word_host, uint64_t *word_dev, uint32_t epoch);
// the spin of stream_wait alone, on a word the stream's own kernel stores
hipError_t stream_spin(hipStream_t s, uint64_t *word_host, uint32_t epoch);
// ono_sparse_lift_dev_async with an in-kernel completion: when the lift is one launch its last workgroup
// stores `sig` into the host-mapped word (word_host / word_dev) and in_kernel is set; else the caller waits
struct LiftDone {
    uint64_t *word_host = nullptr, *word_dev = nullptr;
    uint32_t sig = 0;
    bool in_kernel = false;
};
int lift_dev_async(float *g, size_t cap, const uint8_t *buf_dev, size_t nbytes, uint64_t *status, uint64_t *ticket,
                   hipStream_t s, LiftDone *done);
// a SparseGrad's values [0, min(total, L)) on the host after the reference's
// sequential parse of the whole stream (ono_sparse.hip); *got = its total
int sparse_lift_prefix_host(const uint8_t *buf, size_t nbytes, float *out, size_t L, size_t *got);
// the library's own pure streams (T = float or uint16_t): dst = src, dst = value
template <class T> hipError_t launch_copy(T *dst, const T *src, size_t n, hipStream_t s);
template <class T> hipError_t launch_fill(T *dst, T value, size_t n, hipStream_t s);
// device copies / zero fills of any alignment on those streams (ono_ring.cpp)
hipError_t dev_copy(void *dst, const void *src, size_t bytes, hipStream_t s);
hipError_t dev_zero(void *dst, size_t bytes, hipStream_t s);

// a launch that tells the host it is done: its last wave stores `sig` into the host-mapped word (word_dev is
// its device address); arrive is a device counter that only grows, base the waves launched on it so far
// (the launch adds its own)
struct KernelDone {
    uint64_t *word_dev = nullptr, *arrive = nullptr;
    uint64_t base = 0;
    uint32_t sig = 0;
};
// wire-templated hop kernels: W = uint16_t (f16 wire) or float (f32 wire)
template <class W> hipError_t launch_encode(W *out, const float *in, size_t n, hipStream_t s);
template <class W> hipError_t launch_decode_scale(float *out, const W *in, size_t n, float divisor,
                                                  hipStream_t s, KernelDone *done = nullptr);
template <class W> hipError_t launch_encode_zero(W *out, float *chunk, size_t n, hipStream_t s,
                                                 KernelDone *done = nullptr);
template <class W> hipError_t launch_decode_add(float *acc, const W *in, size_t n, hipStream_t s);
template <class W> hipError_t launch_add_encode_zero(W *out, float *acc, const W *in, size_t n,
                                                     hipStream_t s, KernelDone *done = nullptr);
// last scatter hop of the chunk owner: x = acc + in; grad = x / d; out = x; acc = 0
template <class W> hipError_t launch_add_finish(float *grad, W *out, float *acc, const W *in,
                                                size_t n, float divisor, hipStream_t s, KernelDone *done = nullptr);

// Chunk owner's reduction of the direct schedule (ono_kernels.hip DirectOp):
// ins[k] = rank (c+k)'s slice of chunk c (owner's own residual last);
// grad = chain(ins) / divisor; out = wire(chain) (f16 wire) or a copy of grad
// (f32 wire; NULL = none);
// zero the last input, or every input when zero_all.
template <class W>
hipError_t launch_direct(float *grad, W *out, const float *const *ins, int k, size_t n, float divisor,
                         bool zero_all, hipStream_t s);
// the same with nout copies of the result (e.g. straight into every peer's gather
// slot: sys_out = system-coherent stores for peer HBM)
template <class W>
hipError_t launch_direct_multi(float *grad, W *const *outs, int nout, bool sys_out, const float *const *ins, int k,
                               size_t n, float divisor, bool zero_all, hipStream_t s);

// ---- xGMI peer-access schedule (ono_xgmi.hip) ----
// One peer's part of a push or pull launch: n elements from src to dst.
// head = scalar elements before the first 16-B vector (all operands share the
// phase), or kScalarOnly when their phases differ.  tiles is filled in by the
// launcher.
constexpr uint32_t kScalarOnly = 0xFFFFFFFFu;
struct XSeg {
    const void *src;  // push: local slice (f32; a ring residual is zeroed after the read); pull: peer obuf
    void *dst;        // push: peer receive slot (f32); pull: local grad (f32)
    uint64_t n;
    uint32_t head;
    uint32_t tiles;
};
struct XSegs {
    XSeg s[ONO_MAX_INPUTS];
    int nseg;
};
struct XBarrier {
    uint64_t *peer_flags[ONO_MAX_INPUTS];  // peer q's flag array (mapped), this rank writes slot `pos`
    uint64_t *my_flags;                    // this rank's flag array, slot q written by peer q
    uint32_t *err;                         // host-mapped error word, set on timeout
    uint64_t epoch, timeout_ticks;
    int n, pos;
};
hipError_t launch_xgmi_push(const XSegs &g, bool zero_src, hipStream_t s);
hipError_t launch_xgmi_pull(const XSegs &g, bool f16, float divisor, hipStream_t s);
// host-fed input: segment j copies n f32 from host memory (read sc0 sc1) into HBM
hipError_t launch_xgmi_host_in(const XSegs &g, hipStream_t s, bool sys = true);
hipError_t launch_xgmi_barrier(const XBarrier &b, hipStream_t s);
// A system-scope fence on every XCD (host-fed rounds, around the copies): L2
// write-back, then (acquire) L2 invalidate.
hipError_t launch_xgmi_fence_all(hipStream_t s, bool acquire);
// Connect verification (ono_xgmi.cpp): stamp the ring id at the start of every
// page of a region (page 0: at id_off), and read them back through an import
// (bad[p] = 1 where page p shows anything else).
hipError_t launch_xgmi_stamp(uint8_t *region, size_t npages, size_t id_off, uint64_t id, hipStream_t s);
hipError_t launch_xgmi_verify(const uint8_t *region, size_t npages, size_t id_off, uint64_t id, uint8_t *bad,
                              hipStream_t s);
// Teardown markers: lane q != pos stores peer_id[q] into peer_done[q][pos].
struct XSignal {
    uint64_t *peer_done[ONO_MAX_INPUTS];
    uint64_t peer_id[ONO_MAX_INPUTS];
    int n, pos;
};
hipError_t launch_xgmi_signal(const XSignal &sig, hipStream_t s);
// Release bookkeeping (ono_xgmi_pool.h): one system-scope atomic add of 1 to a
// u64 counter of a region (through a peer mapping), completed before the wave ends.
hipError_t launch_xgmi_bump(uint64_t *counter, hipStream_t s);

// PS shard update (storage/blocking/shard.rs:74-92 + optimization/*.rs), fused:
//   g /= nworkers (if > 1); optimizer step on w (state v, s); g = 0 when zero_grad
struct OptLaunch {
    int kind;        // ono_opt_kind
    float lr, momentum, beta1, beta2, eps;
    float step_size; // Adam: lr * (sqrt(1 - beta2^t) / (1 - beta1^t)), computed on the host in f32
    float nworkers;  // divisor (1 = none)
    // Store/PS accumulators start at +0 (shard.rs:41-44), so a summed
    // gradient is never -0; a reduce-scatter of all -0 inputs is.  When set,
    // the update adds +0 first (identity except -0 -> +0).  Wild (raw
    // per-worker gradient, wild/shard.rs:43-58) leaves it clear.
    bool plus_zero = true;
};
hipError_t launch_opt_update(const OptLaunch &o, float *g, float *w, float *v, float *s_,
                             size_t n, bool zero_grad, hipStream_t st, float *w_copy = nullptr,
                             bool copy_for_peers = false);  // w_copy read by other ranks after a barrier

}  // namespace ono
