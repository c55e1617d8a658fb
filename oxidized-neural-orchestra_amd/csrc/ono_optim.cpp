// ono_optim.cpp — the all-reduce consumer.
//
// After pull_grads the reference worker runs (worker/src/workers/all_reduce.rs:126-132)
//   Trainer::optimize -> ParamManager::optimize -> Optimizer::update_params(grad, params)
//   param_manager.zero_grad()
//   optimization_params.copy_from_slice(&params)
// i.e. three passes over N floats.  Here they are one fused gfx950 kernel
// (OptOp with a second parameter output): read grad, params (+ optimizer state),
// write params, the params copy, grad = 0 (+ state).  The gradient is used as
// the ring produced it — no averaging (pull_grads already divided) and no +0
// canonicalisation (a ring sum can legitimately be -0).
#include <hip/hip_runtime.h>

#include <cmath>
#include <mutex>

#include "ono_internal.h"

using namespace ono;

struct ono_optimizer {
    int device = 0;
    size_t n = 0;
    OptLaunch o{};
    float beta1_t = 1.0f, beta2_t = 1.0f;  // adam.rs:39-40
    float *v = nullptr, *s = nullptr;
    std::mutex mu;
};

extern "C" {

int ono_optimizer_create(ono_optimizer **out, const ono_opt_spec *opt, size_t n, int device) {
    if (!out || !opt) return set_error(ONO_E_ARG, "NULL argument");
    *out = nullptr;
    if (opt->kind < ONO_OPT_GD || opt->kind > ONO_OPT_ADD) return set_error(ONO_E_ARG, "optimizer kind %d", opt->kind);
    int prev = -1;
    (void)hipGetDevice(&prev);
    ONO_HIP(hipSetDevice(device));
    ono_optimizer *p = new ono_optimizer();
    p->device = device;
    p->n = n;
    p->o = OptLaunch{opt->kind, opt->lr, opt->momentum, opt->beta1, opt->beta2, opt->eps, 0.0f, 1.0f};
    p->o.plus_zero = false;
    const size_t b = (n ? n : 1) * sizeof(float);
    hipError_t e = hipSuccess;
    if (opt->kind == ONO_OPT_MOMENTUM || opt->kind == ONO_OPT_ADAM) {
        if ((e = hipMalloc((void **)&p->v, b)) == hipSuccess) e = hipMemset(p->v, 0, b);
    }
    if (e == hipSuccess && opt->kind == ONO_OPT_ADAM) {
        if ((e = hipMalloc((void **)&p->s, b)) == hipSuccess) e = hipMemset(p->s, 0, b);
    }
    // the zero fills ran on the null stream; the caller's stream may be a non-blocking one: complete them here
    if (e == hipSuccess) e = hipStreamSynchronize(nullptr);
    if (prev >= 0) (void)hipSetDevice(prev);
    if (e != hipSuccess) {
        (void)hipFree(p->v);
        (void)hipFree(p->s);
        delete p;
        return hip_error(e, "optimizer state allocation", __FILE__, __LINE__);
    }
    *out = p;
    return ONO_OK;
}

int ono_optimizer_destroy(ono_optimizer *p) {
    if (!p) return ONO_OK;
    (void)hipFree(p->v);
    (void)hipFree(p->s);
    delete p;
    return ONO_OK;
}

int ono_optimizer_step(ono_optimizer *p, float *params, float *grad, float *params_copy, size_t n,
                       void *stream) {
    if (!p || (n && (!params || !grad))) return set_error(ONO_E_ARG, "NULL argument");
    if (n != p->n) return set_error(ONO_E_SIZE, "buffers of %zu elements, optimizer of %zu", n, p->n);
    std::lock_guard<std::mutex> lk(p->mu);
    if (p->o.kind == ONO_OPT_ADAM) {  // adam.rs:76-80, f32 on the host
        p->beta1_t *= p->o.beta1;
        p->beta2_t *= p->o.beta2;
        float bc1 = 1.0f - p->beta1_t, bc2 = 1.0f - p->beta2_t;
        p->o.step_size = p->o.lr * (std::sqrt(bc2) / bc1);
    }
    ONO_HIP(launch_opt_update(p->o, grad, params, p->v, p->s, n, true, reinterpret_cast<hipStream_t>(stream),
                              params_copy));
    return ONO_OK;
}

}  // extern "C"
