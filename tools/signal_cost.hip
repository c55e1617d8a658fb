// signal_cost — what a host wait on stream completion costs (round 5, the TCP ring's hop):
// after one small kernel, the host learns that the stream reached that point by
//   (a) a one-wave kernel storing an epoch to a host-mapped word, host spin (the library's host_wait)
//   (b) hipStreamWriteValue64 of the epoch to the host-mapped word, host spin
//   (c) hipEventRecord + spin on hipEventQuery
//   (d) hipStreamSynchronize
//   (e) the small kernel itself storing the epoch when done (one workgroup: no completion count)
// Prints the median wall time per (kernel + wait) over 2000 iterations for each.
//   make -C tools signal_cost && tools/signal_cost
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
            return 2;                                                                     \
        }                                                                                 \
    } while (0)

__global__ void work(float *x, int n, uint64_t *word, uint64_t epoch) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) x[i] = x[i] * 0.5f + 1.0f;
    if (word) {
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence_system();
            __hip_atomic_store(word, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}
__global__ void signal(uint64_t *word, uint64_t epoch) {
    if (threadIdx.x == 0) __hip_atomic_store(word, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    float *x;
    CK(hipMalloc((void **)&x, 256 * sizeof(float)));
    uint64_t *wh, *wd;
    CK(hipHostMalloc((void **)&wh, 64, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer((void **)&wd, wh, 0));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    const char *names[] = {"signal_kernel_spin", "stream_write_value_spin", "event_query_spin", "stream_synchronize",
                           "in_kernel_store_spin"};
    uint64_t epoch = 0;
    for (int form = 0; form < 5; form++) {
        std::vector<double> ts;
        for (int it = 0; it < 2200; it++) {
            ++epoch;
            volatile uint64_t *w = wh;
            const auto t0 = std::chrono::steady_clock::now();
            hipLaunchKernelGGL(work, dim3(1), dim3(256), 0, s, x, 256, form == 4 ? wd : nullptr, epoch);
            if (form == 0) {
                hipLaunchKernelGGL(signal, dim3(1), dim3(64), 0, s, wd, epoch);
                while (*w != epoch) {}
            } else if (form == 1) {
                CK(hipStreamWriteValue64(s, wd, epoch, 0));
                while (*w != epoch) {}
            } else if (form == 2) {
                CK(hipEventRecord(ev, s));
                while (hipEventQuery(ev) == hipErrorNotReady) {}
            } else if (form == 3) {
                CK(hipStreamSynchronize(s));
            } else {
                while (*w != epoch) {}
            }
            const auto t1 = std::chrono::steady_clock::now();
            if (it >= 200) ts.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
        }
        std::sort(ts.begin(), ts.end());
        printf("{\"form\": \"%s\", \"us_p50\": %.2f, \"us_p10\": %.2f, \"us_p90\": %.2f}\n", names[form], ts[ts.size() / 2],
               ts[ts.size() / 10], ts[ts.size() * 9 / 10]);
        fflush(stdout);
    }
    return 0;
}
