// ono_store.cpp — the parameter-server store and synchronizers on one device.
//
// BlockingStore (parameter_server/src/storage/blocking/{store,shard}.rs):
// double-buffered gradient accumulators + parameters + optimizer state live in
// HBM; accumulate = one fused `acc[active] += g` kernel; update_params = the
// CAS guard, the active-buffer flip, and ONE fused kernel per store doing
// g /= nworkers, the optimizer step and g = 0 (the reference does the same per
// shard on rayon threads).  Shards only bound the per-shard optimizer state in
// the reference; every shard steps together, so one flat launch is the same
// arithmetic.  WildStore (wild/{store,shard}.rs) applies the optimizer to
// every incoming gradient; its unsynchronised races become stream order here.
//
// BarrierSync / NoBlockingSync / DynBarrier (synchronization/*.rs) are host
// logic, restated on std::mutex + std::condition_variable.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <mutex>

#include "ono_internal.h"

using namespace ono;

namespace {
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
}  // namespace

struct ono_store {
    int kind = ONO_STORE_BLOCKING, device = 0;
    size_t nparams = 0, shard_size = 0, nworkers = 1;
    float *grads[2] = {nullptr, nullptr};
    float *params = nullptr, *v = nullptr, *s = nullptr, *scratch = nullptr;
    OptLaunch opt{};
    float beta1_t = 1.0f, beta2_t = 1.0f;
    std::atomic<int> active_idx{0};
    std::atomic<bool> updating{false};
    std::mutex mu;  // orders submissions on `stream` (the reference's shard mutexes)
    hipStream_t stream = nullptr;
};

static void adam_advance(ono_store *st) {  // adam.rs:76-80, f32 on the host
    if (st->opt.kind != ONO_OPT_ADAM) return;
    st->beta1_t *= st->opt.beta1;
    st->beta2_t *= st->opt.beta2;
    float bc1 = 1.0f - st->beta1_t, bc2 = 1.0f - st->beta2_t;
    st->opt.step_size = st->opt.lr * (std::sqrt(bc2) / bc1);
}

extern "C" {

int ono_store_create(ono_store **out, int kind, const float *init, size_t nparams,
                     size_t shard_size, size_t nworkers, const ono_opt_spec *opt, int device) {
    if (!out || (!init && nparams) || !opt) return set_error(ONO_E_ARG, "NULL argument");
    *out = nullptr;
    if (kind != ONO_STORE_BLOCKING && kind != ONO_STORE_WILD) return set_error(ONO_E_ARG, "store kind %d", kind);
    if (opt->kind < ONO_OPT_GD || opt->kind > ONO_OPT_ADD) return set_error(ONO_E_ARG, "optimizer kind %d", opt->kind);
    if (shard_size == 0) return set_error(ONO_E_ARG, "shard_size must be non-zero (NonZeroUsize)");
    DeviceGuard g(device);
    ono_store *st = new ono_store();
    st->kind = kind; st->device = device; st->nparams = nparams; st->shard_size = shard_size;
    st->nworkers = nworkers ? nworkers : 1;  // NonZeroUsize::new(..).unwrap_or(MIN), builder.rs:164
    st->opt = OptLaunch{opt->kind, opt->lr, opt->momentum, opt->beta1, opt->beta2, opt->eps, 0.0f, 1.0f};
    const size_t b = (nparams ? nparams : 1) * sizeof(float);
    auto fail = [&](hipError_t e) { ono_store_destroy(st); return hip_error(e, "store allocation", __FILE__, __LINE__); };
    hipError_t e;
    if ((e = hipSetDevice(device)) != hipSuccess) return fail(e);
    if ((e = hipStreamCreateWithFlags(&st->stream, hipStreamNonBlocking)) != hipSuccess) return fail(e);
    for (float **p : {&st->grads[0], &st->grads[1], &st->params, &st->v, &st->s, &st->scratch}) {
        if ((e = hipMalloc((void **)p, b)) != hipSuccess) return fail(e);
        if ((e = hipMemset(*p, 0, b)) != hipSuccess) return fail(e);
    }
    if (nparams && (e = hipMemcpy(st->params, init, nparams * sizeof(float), hipMemcpyHostToDevice)) != hipSuccess)
        return fail(e);
    // the zero fills ran on the null stream, which the store's non-blocking stream is not ordered with:
    // complete before the store is handed out (as the ring's buckets)
    if ((e = hipStreamSynchronize(nullptr)) != hipSuccess) return fail(e);
    *out = st;
    return ONO_OK;
}

int ono_store_destroy(ono_store *st) {
    if (!st) return ONO_OK;
    {
        DeviceGuard g(st->device);
        if (st->stream) (void)hipStreamSynchronize(st->stream);
        for (float *p : {st->grads[0], st->grads[1], st->params, st->v, st->s, st->scratch}) (void)hipFree(p);
        if (st->stream) (void)hipStreamDestroy(st->stream);
    }
    delete st;
    return ONO_OK;
}

size_t ono_store_len(const ono_store *st) { return st ? st->nparams : 0; }

static int accumulate(ono_store *st, const float *grad, size_t n, hipMemcpyKind kind) {
    if (!st || (!grad && n)) return set_error(ONO_E_ARG, "NULL argument");
    if (n != st->nparams) return set_error(ONO_E_SIZE, "gradient of %zu elements, store of %zu", n, st->nparams);
    std::lock_guard<std::mutex> lk(st->mu);
    DeviceGuard g(st->device);
    hipStream_t s = st->stream;
    if (n == 0) return ONO_OK;
    ONO_HIP(hipMemcpyAsync(st->scratch, grad, n * sizeof(float), kind, s));
    if (st->kind == ONO_STORE_WILD) {
        // wild/store.rs:77-91: the optimizer consumes every gradient as it arrives
        adam_advance(st);
        OptLaunch o = st->opt;
        o.nworkers = 1.0f;
        o.plus_zero = false;  // the raw incoming gradient, as WildShard::update_params
        ONO_HIP(launch_opt_update(o, st->scratch, st->params, st->v, st->s, n, false, s));
    } else {
        // store.rs:84-91: the active index is read once per accumulate
        int active = st->active_idx.load(std::memory_order_acquire);
        ONO_HIP(launch_acc(st->grads[active], st->scratch, n, s, true));
    }
    ONO_HIP(hipStreamSynchronize(s));
    return ONO_OK;
}

// The reference's wire form: the worker sends its gradient as f16
// (ParamServerHandle::push_grad, comms/src/handles/parameter_server.rs:92-107)
// and the server decodes it on the CPU before accumulating
// (WorkerHandle::recv_event, handles/worker.rs:82-101).  Here the f16 payload
// itself crosses PCIe (half the bytes) and the decode is fused into the
// accumulate kernel: acc += f32(h), exact widening with half 2.7.1's NaN rule.
static int accumulate_f16(ono_store *st, const uint16_t *grad, size_t n, hipMemcpyKind kind) {
    if (!st || (!grad && n)) return set_error(ONO_E_ARG, "NULL argument");
    if (n != st->nparams) return set_error(ONO_E_SIZE, "gradient of %zu elements, store of %zu", n, st->nparams);
    std::lock_guard<std::mutex> lk(st->mu);
    DeviceGuard g(st->device);
    hipStream_t s = st->stream;
    if (n == 0) return ONO_OK;
    uint16_t *h = reinterpret_cast<uint16_t *>(st->scratch);  // 4N bytes hold the 2N-byte payload
    ONO_HIP(hipMemcpyAsync(h, grad, n * sizeof(uint16_t), kind, s));
    if (st->kind == ONO_STORE_WILD) {
        adam_advance(st);
        OptLaunch o = st->opt;
        o.nworkers = 1.0f;
        o.plus_zero = false;
        float *g32 = st->grads[0];  // unused by the wild store: the decoded gradient
        ONO_HIP(launch_decode_scale<uint16_t>(g32, h, n, 1.0f, s));
        ONO_HIP(launch_opt_update(o, g32, st->params, st->v, st->s, n, false, s));
    } else {
        int active = st->active_idx.load(std::memory_order_acquire);
        ONO_HIP(launch_decode_add<uint16_t>(st->grads[active], h, n, s));
    }
    ONO_HIP(hipStreamSynchronize(s));
    return ONO_OK;
}

int ono_store_accumulate(ono_store *st, const float *grad, size_t n) {
    return accumulate(st, grad, n, hipMemcpyHostToDevice);
}
int ono_store_accumulate_dev(ono_store *st, const float *grad, size_t n) {
    return accumulate(st, grad, n, hipMemcpyDeviceToDevice);
}

int ono_store_accumulate_f16(ono_store *st, const uint16_t *grad, size_t n) {
    return accumulate_f16(st, grad, n, hipMemcpyHostToDevice);
}
int ono_store_accumulate_f16_dev(ono_store *st, const uint16_t *grad, size_t n) {
    return accumulate_f16(st, grad, n, hipMemcpyDeviceToDevice);
}

int ono_store_update_params(ono_store *st) {
    if (!st) return set_error(ONO_E_ARG, "store is NULL");
    if (st->kind == ONO_STORE_WILD) return ONO_OK;  // wild/store.rs:94: no-op
    bool expected = false;
    if (!st->updating.compare_exchange_strong(expected, true, std::memory_order_acq_rel,
                                              std::memory_order_relaxed))
        return ONO_OK;  // store.rs:94-99: somebody else is updating
    int rc = ONO_OK;
    {
        std::lock_guard<std::mutex> lk(st->mu);
        DeviceGuard g(st->device);
        int frozen = st->active_idx.fetch_xor(1, std::memory_order_acq_rel);
        adam_advance(st);
        OptLaunch o = st->opt;
        o.nworkers = (float)st->nworkers;  // shard.rs:80-83, factor = nworkers as f32
        hipError_t e = launch_opt_update(o, st->grads[frozen], st->params, st->v, st->s,
                                         st->nparams, true, st->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(st->stream);
        if (e != hipSuccess) rc = hip_error(e, "update_params", __FILE__, __LINE__);
    }
    st->updating.store(false, std::memory_order_release);
    return rc;
}

static int pull(ono_store *st, float *out, size_t n, hipMemcpyKind kind) {
    if (!st || (!out && n)) return set_error(ONO_E_ARG, "NULL argument");
    if (n != st->nparams) return set_error(ONO_E_SIZE, "buffer of %zu elements, store of %zu", n, st->nparams);
    std::lock_guard<std::mutex> lk(st->mu);
    DeviceGuard g(st->device);
    if (n == 0) return ONO_OK;
    ONO_HIP(hipMemcpyAsync(out, st->params, n * sizeof(float), kind, st->stream));
    ONO_HIP(hipStreamSynchronize(st->stream));
    return ONO_OK;
}

int ono_store_pull_params(ono_store *st, float *out, size_t n) { return pull(st, out, n, hipMemcpyDeviceToHost); }
int ono_store_pull_params_dev(ono_store *st, float *out, size_t n) { return pull(st, out, n, hipMemcpyDeviceToDevice); }

int ono_store_active_idx(const ono_store *st) { return st ? st->active_idx.load() : -1; }
int ono_store_set_updating(ono_store *st, int u) {
    if (!st) return set_error(ONO_E_ARG, "store is NULL");
    st->updating.store(u != 0);
    return ONO_OK;
}

}  // extern "C"

// ------------------------------------------------------------ DynBarrier ----
// synchronization/dyn_barrier.rs:47-106, restated.  The leader closure runs
// with the state lock held, exactly as in the reference.
struct ono_barrier {
    std::mutex mu;
    std::condition_variable cv;
    size_t generation = 0, leader_gen = 0, remaining = 0, size = 0;

    void advance() {
        generation += 1;
        remaining = size;
        if (remaining > 1) cv.notify_all();
    }
    template <class F> void wait_with(F &&leader) {
        std::unique_lock<std::mutex> lk(mu);
        remaining -= 1;
        bool is_leader;
        if (remaining > 0) {
            size_t local = generation;
            cv.wait(lk, [&] { return generation != local; });
            is_leader = leader_gen < generation;
        } else {
            is_leader = true;
        }
        if (is_leader) {
            leader();
            leader_gen += 1;
            if (leader_gen > generation) advance();
        }
    }
    void acquire() {
        std::lock_guard<std::mutex> lk(mu);
        remaining -= 1;
        size -= 1;
        if (remaining == 0) advance();
    }
};

extern "C" {

int ono_barrier_create(ono_barrier **out, size_t size) {
    if (!out || size == 0) return set_error(ONO_E_ARG, "size must be non-zero");
    ono_barrier *b = new ono_barrier();
    b->remaining = b->size = size;
    *out = b;
    return ONO_OK;
}
int ono_barrier_destroy(ono_barrier *b) {
    delete b;
    return ONO_OK;
}
int ono_barrier_wait_with(ono_barrier *b, ono_leader_fn f, void *ctx) {
    if (!b) return set_error(ONO_E_ARG, "barrier is NULL");
    b->wait_with([&] { if (f) f(ctx); });
    return ONO_OK;
}
int ono_barrier_acquire(ono_barrier *b) {
    if (!b) return set_error(ONO_E_ARG, "barrier is NULL");
    b->acquire();
    return ONO_OK;
}

}  // extern "C"

// ----------------------------------------------------------- Synchronizer ---
struct ono_sync {
    int kind = ONO_SYNC_BARRIER;
    ono_barrier barrier;
    std::atomic<int> refs{1};  // Arc strong count of the BarrierSync clones
};

extern "C" {

int ono_sync_create(ono_sync **out, int kind, size_t barrier_size) {
    if (!out) return set_error(ONO_E_ARG, "out is NULL");
    if (kind != ONO_SYNC_BARRIER && kind != ONO_SYNC_NONBLOCKING) return set_error(ONO_E_ARG, "sync kind %d", kind);
    if (kind == ONO_SYNC_BARRIER && barrier_size == 0) return set_error(ONO_E_ARG, "barrier size must be non-zero");
    ono_sync *s = new ono_sync();
    s->kind = kind;
    s->barrier.remaining = s->barrier.size = barrier_size ? barrier_size : 1;
    *out = s;
    return ONO_OK;
}

int ono_sync_clone(ono_sync *s) {
    if (!s) return set_error(ONO_E_ARG, "sync is NULL");
    s->refs.fetch_add(1);
    return ONO_OK;
}

int ono_sync_release(ono_sync *s) {
    if (!s) return set_error(ONO_E_ARG, "sync is NULL");
    // barrier.rs:30-38: a dropped clone shrinks the barrier while others remain
    int before = s->refs.fetch_sub(1);
    if (before > 1) {
        if (s->kind == ONO_SYNC_BARRIER) s->barrier.acquire();
    } else {
        delete s;
    }
    return ONO_OK;
}

static int sync_step(ono_sync *s, ono_store *st, const void *grad, bool f16, float *params, size_t n) {
    if (!s || !st) return set_error(ONO_E_ARG, "NULL argument");
    int rc = f16 ? ono_store_accumulate_f16(st, static_cast<const uint16_t *>(grad), n)
                 : ono_store_accumulate(st, static_cast<const float *>(grad), n);
    if (rc) return rc;
    if (s->kind == ONO_SYNC_BARRIER) {
        int urc = ONO_OK;
        s->barrier.wait_with([&] { urc = ono_store_update_params(st); });
        if (urc) return urc;
    } else {
        rc = ono_store_update_params(st);
        if (rc) return rc;
    }
    return ono_store_pull_params(st, params, n);
}

int ono_sync_step(ono_sync *s, ono_store *st, const float *grad, float *params, size_t n) {
    return sync_step(s, st, grad, false, params, n);
}
int ono_sync_step_f16(ono_sync *s, ono_store *st, const uint16_t *grad, float *params, size_t n) {
    return sync_step(s, st, grad, true, params, n);
}

}  // extern "C"
