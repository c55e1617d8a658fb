// xcd_balance.hip — one A/B session for BASELINE config 2:
// does balancing the work across the XCDs at run time beat the one-shot grid
// whose XCDs finish 1.2-3.9 us apart?
//   A  the library's ono_sum_scale_f32 (one-shot grid, one 16-B vector per lane)
//   B  a resident grid (CUs x W workgroups of 256 threads); each XCD owns 1/8 of
//      the pieces (P elements each) and takes them with a per-XCD counter
//      (its XCC id from HW_REG_XCC_ID); a workgroup whose XCD's share is gone
//      takes pieces of the other XCDs — so a slow XCD's tail is done by the rest
// Both: out = (sum of k inputs) / k, 64 MiB per buffer, rotating sets (> 1.5 GiB)
// so the Infinity Cache cannot serve re-reads, HIP events around 20 launches,
// median of 5 passes.  Prints one JSON line per k.
//   make -C tools xcd_balance && tools/xcd_balance
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ono_reduce.h"

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
            exit(2);                                                                      \
        }                                                                                 \
    } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int kT = 256;
constexpr int kV = 4;                      // vectors per lane per piece
constexpr int kPiece = kT * kV * 4;        // elements per piece (4096)

struct Ins {
    const float *p[8];
};

template <int K>
__global__ __launch_bounds__(kT) void sum_dyn(float *out, Ins in, uint32_t pieces, float d, unsigned *ctr) {
    __shared__ uint32_t s_piece;
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    x &= 7u;
    const uint32_t per = (pieces + 7) / 8;
    uint32_t y = x, tried = 0;
    for (;;) {
        if (threadIdx.x == 0) {
            uint32_t p = 0xFFFFFFFFu;
            while (tried < 8) {
                const uint32_t q = atomicAdd(ctr + 32 * y, 1u);  // (one 128-B line per counter)
                const uint32_t lo = y * per, hi = min(pieces, lo + per);
                if (lo + q < hi) {
                    p = lo + q;
                    break;
                }
                y = (y + 1) & 7u;
                tried++;
            }
            s_piece = p;
        }
        __syncthreads();
        const uint32_t p = s_piece;
        __syncthreads();
        if (p == 0xFFFFFFFFu) return;
        const size_t base = (size_t)p * kPiece / 4;  // in vectors
        f4 acc[kV];
#pragma unroll
        for (int v = 0; v < kV; v++) acc[v] = __builtin_nontemporal_load((const f4 *)in.p[0] + base + v * kT + threadIdx.x);
#pragma unroll
        for (int k = 1; k < K; k++)
#pragma unroll
            for (int v = 0; v < kV; v++)
                acc[v] += __builtin_nontemporal_load((const f4 *)in.p[k] + base + v * kT + threadIdx.x);
#pragma unroll
        for (int v = 0; v < kV; v++) __builtin_nontemporal_store(acc[v] / d, (f4 *)out + base + v * kT + threadIdx.x);
    }
}

int main(int argc, char **argv) {
    const size_t n = (size_t)16 << 20;  // 64 MiB of f32
    const int W = argc > 1 ? atoi(argv[1]) : 8;  // resident workgroups per CU for B
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int sets = 4, launches = 20, passes = 5;
    const uint32_t pieces = (uint32_t)(n / kPiece);
    for (int K : {2, 4, 8}) {
        std::vector<float *> bufs((size_t)sets * (K + 1));
        for (auto &b : bufs) {
            CK(hipMalloc(&b, n * 4));
            CK(ono_synth_f32(b, n, 7, (uint64_t)(&b - bufs.data()), 0, nullptr) == ONO_OK ? hipSuccess : hipErrorUnknown);
        }
        unsigned *ctr = nullptr;
        const size_t nctr = (size_t)launches * 8 * 32;
        CK(hipMalloc(&ctr, nctr * 4));
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        std::vector<double> ta, tb;
        for (int pass = 0; pass < passes; pass++) {
            for (int form = 0; form < 2; form++) {
                CK(hipMemset(ctr, 0, nctr * 4));
                CK(hipDeviceSynchronize());
                for (int w = 0; w < 3; w++) {  // warm-up launches (their own counters: the last ones)
                    float **s = &bufs[(size_t)(w % sets) * (K + 1)];
                    if (form == 0) (void)ono_sum_scale_f32(s[K], (const float *const *)s, K, n, (float)K, nullptr);
                }
                CK(hipEventRecord(e0, nullptr));
                for (int l = 0; l < launches; l++) {
                    float **s = &bufs[(size_t)(l % sets) * (K + 1)];
                    if (form == 0) {
                        (void)ono_sum_scale_f32(s[K], (const float *const *)s, K, n, (float)K, nullptr);
                    } else {
                        Ins in{};
                        for (int k = 0; k < K; k++) in.p[k] = s[k];
                        unsigned *c = ctr + (size_t)l * 8 * 32;
                        dim3 g((unsigned)(cus * W)), b(kT);
                        if (K == 2) hipLaunchKernelGGL(sum_dyn<2>, g, b, 0, 0, s[K], in, pieces, (float)K, c);
                        else if (K == 4) hipLaunchKernelGGL(sum_dyn<4>, g, b, 0, 0, s[K], in, pieces, (float)K, c);
                        else hipLaunchKernelGGL(sum_dyn<8>, g, b, 0, 0, s[K], in, pieces, (float)K, c);
                    }
                }
                CK(hipEventRecord(e1, nullptr));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                (form == 0 ? ta : tb).push_back(ms * 1e3 / launches);
            }
        }
        std::sort(ta.begin(), ta.end());
        std::sort(tb.begin(), tb.end());
        const double bytes = (double)(K + 1) * n * 4;
        printf("{\"k\": %d, \"resident_wg_per_cu\": %d, \"oneshot_us\": %.2f, \"oneshot_frac\": %.4f, \"balanced_us\": %.2f, "
               "\"balanced_frac\": %.4f}\n",
               K, W, ta[passes / 2], bytes / (ta[passes / 2] * 1e-6) / 8e12, tb[passes / 2],
               bytes / (tb[passes / 2] * 1e-6) / 8e12);
        fflush(stdout);
        for (auto &b : bufs) CK(hipFree(b));
        CK(hipFree(ctr));
    }
    return 0;
}
