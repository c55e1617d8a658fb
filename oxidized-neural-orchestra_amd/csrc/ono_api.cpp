// ono_api.cpp — C ABI entry points: errors and the elementwise kernel surface.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <string>

#include "ono_internal.h"

namespace ono {

static thread_local std::string g_err;

int set_error(int code, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

int hip_error(hipError_t e, const char *what, const char *file, int line) {
    return set_error(ONO_E_HIP, "%s failed: %s (%s:%d)", what, hipGetErrorString(e), file, line);
}

}  // namespace ono

using namespace ono;

#define ONO_LAUNCH(expr)                                                            \
    do {                                                                            \
        hipError_t ono_e_ = (expr);                                                 \
        if (ono_e_ != hipSuccess) return hip_error(ono_e_, #expr, __FILE__, __LINE__); \
        return ONO_OK;                                                              \
    } while (0)

static inline hipStream_t S(void *s) { return reinterpret_cast<hipStream_t>(s); }

extern "C" {

const char *ono_last_error(void) { return g_err.c_str(); }
int ono_abi_version(void) { return ONO_ABI_VERSION; }

int ono_device_count(int *count) {
    if (!count) return set_error(ONO_E_ARG, "count is NULL");
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *count = c;
    return ONO_OK;
}

int ono_sum_scale_f32(float *out, const float *const *ins, int k, size_t n, float divisor,
                      void *stream) {
    if (k < 1 || k > ONO_MAX_INPUTS) return set_error(ONO_E_ARG, "k=%d outside [1, %d]", k, ONO_MAX_INPUTS);
    if (n && (!out || !ins)) return set_error(ONO_E_ARG, "NULL pointer");
    for (int j = 0; n && j < k; j++)
        if (!ins[j]) return set_error(ONO_E_ARG, "ins[%d] is NULL", j);
    ONO_LAUNCH(launch_sum_scale(out, ins, k, n, divisor, S(stream)));
}

int ono_acc_f32(float *acc, const float *in, size_t n, void *stream) {
    if (n && (!acc || !in)) return set_error(ONO_E_ARG, "NULL pointer");
    ONO_LAUNCH(launch_acc(acc, in, n, S(stream)));
}

int ono_scale_zero_f32(float *dst, const float *src, size_t n, float divisor, float *zero,
                       void *stream) {
    if (n && (!dst || !src)) return set_error(ONO_E_ARG, "NULL pointer");
    ONO_LAUNCH(launch_scale_zero(dst, src, n, divisor, zero, S(stream)));
}

int ono_copy_f32(float *dst, const float *src, size_t n, void *stream) {
    if (n && (!dst || !src)) return set_error(ONO_E_ARG, "NULL pointer");
    ONO_LAUNCH(launch_copy<float>(dst, src, n, S(stream)));
}

int ono_fill_f32(float *dst, float value, size_t n, void *stream) {
    if (n && !dst) return set_error(ONO_E_ARG, "NULL pointer");
    ONO_LAUNCH(launch_fill<float>(dst, value, n, S(stream)));
}

int ono_f16_encode(uint16_t *out, const float *in, size_t n, void *stream) {
    if (n && (!out || !in)) return set_error(ONO_E_ARG, "NULL pointer");
    ONO_LAUNCH(launch_encode<uint16_t>(out, in, n, S(stream)));
}

int ono_f16_decode(float *out, const uint16_t *in, size_t n, void *stream) {
    if (n && (!out || !in)) return set_error(ONO_E_ARG, "NULL pointer");
    ONO_LAUNCH(launch_decode_scale<uint16_t>(out, in, n, 1.0f, S(stream)));
}

int ono_f16_encode_zero(uint16_t *out, float *chunk, size_t n, void *stream) {
    if (n && (!out || !chunk)) return set_error(ONO_E_ARG, "NULL pointer");
    ONO_LAUNCH(launch_encode_zero<uint16_t>(out, chunk, n, S(stream)));
}

int ono_f16_decode_add(float *acc, const uint16_t *in, size_t n, void *stream) {
    if (n && (!acc || !in)) return set_error(ONO_E_ARG, "NULL pointer");
    ONO_LAUNCH(launch_decode_add<uint16_t>(acc, in, n, S(stream)));
}

int ono_f16_add_encode_zero(uint16_t *out, float *acc, const uint16_t *in, size_t n, void *stream) {
    if (n && (!out || !acc || !in)) return set_error(ONO_E_ARG, "NULL pointer");
    ONO_LAUNCH(launch_add_encode_zero<uint16_t>(out, acc, in, n, S(stream)));
}

int ono_f16_decode_scale(float *out, const uint16_t *in, size_t n, float divisor, void *stream) {
    if (n && (!out || !in)) return set_error(ONO_E_ARG, "NULL pointer");
    ONO_LAUNCH(launch_decode_scale<uint16_t>(out, in, n, divisor, S(stream)));
}

int ono_direct_chain(float *grad, void *out, const float *const *ins, int k, size_t n, float divisor, int wire,
                     int zero_all, void *stream) {
    if (k < 1 || k > ONO_MAX_INPUTS) return set_error(ONO_E_ARG, "k=%d outside [1, %d]", k, ONO_MAX_INPUTS);
    if (wire != ONO_WIRE_F32 && wire != ONO_WIRE_F16) return set_error(ONO_E_ARG, "wire=%d", wire);
    if (n && (!grad || !ins)) return set_error(ONO_E_ARG, "NULL pointer");
    for (int j = 0; n && j < k; j++)
        if (!ins[j]) return set_error(ONO_E_ARG, "ins[%d] is NULL", j);
    if (wire == ONO_WIRE_F16)
        ONO_LAUNCH(launch_direct<uint16_t>(grad, static_cast<uint16_t *>(out), ins, k, n, divisor, zero_all != 0,
                                           S(stream)));
    ONO_LAUNCH(launch_direct<float>(grad, static_cast<float *>(out), ins, k, n, divisor, zero_all != 0, S(stream)));
}

int ono_synth_f32(float *out, size_t n, uint64_t seed, uint64_t rank, size_t offset, void *stream) {
    if (n && !out) return set_error(ONO_E_ARG, "NULL pointer");
    ONO_LAUNCH(launch_synth(out, n, seed, rank, offset, S(stream)));
}

}  // extern "C"
