// thr_bench — the TCP ring's threshold for a config-1 push (measurement build, not the product).
//
// The push's threshold is two launches: sp_gather_keys (the 16384 sampled |g| keys) and sp_threshold (the
// bit-sliced select in one workgroup).  This tool times them over a config-1 chunk (54,693 values of the
// bench's synthetic distribution, 16384 sampled indices in HBM or pinned host memory):
//   * back to back (K pairs between two events): the kernels' own cost, launch gaps included;
//   * one pair at a time, synchronized (event pair around each): the latency a push sees;
//   * a stamped copy of sp_threshold (wall clock, 100 MHz, thread 0): start -> keys loaded -> transposed ->
//     end, so the select's own phases are known;
//   * variants of the select, each checked against the library's result.
//
// usage: thr_bench [K=200]
#include "../oxidized-neural-orchestra_amd/csrc/ono_sparse.hip"

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <random>
#include <vector>

namespace ono {
int set_error(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    fprintf(stderr, "error %d: ", code);
    vfprintf(stderr, fmt, ap);
    fprintf(stderr, "\n");
    va_end(ap);
    return code;
}
int hip_error(hipError_t e, const char *what, const char *file, int line) {
    fprintf(stderr, "%s: %s (%s:%d)\n", what, hipGetErrorString(e), file, line);
    return ONO_E_HIP;
}
}  // namespace ono

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

namespace {

// sp_threshold with stamps: st[0..3] = start, keys in registers, transposed, end (thread 0's wall clock)
__global__ __launch_bounds__(kThrT) void thr_stamped(const uint32_t *keys, uint32_t m, uint32_t k, float *t_out,
                                                     uint64_t *st) {
    __shared__ uint32_t wc[2][kThrT / 64][2];
    const uint64_t t0 = wall_clock64();
    const int wave = threadIdx.x / 64;
    uint32_t A[32], C = 0;
#pragma unroll
    for (int q = 0; q < kThrK; q++) {
        const uint32_t i = threadIdx.x + (uint32_t)q * kThrT;
        A[q] = i < m ? keys[i] : 0u;
        C |= i < m ? 1u << (31 - q) : 0u;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const uint64_t t1 = wall_clock64();
    transpose32(A);
    __syncthreads();
    const uint64_t t2 = wall_clock64();
    uint32_t prefix = 0, kk = k;
#pragma unroll
    for (int s = 0; s < 16; s++) {
        const int hi = 30 - 2 * s, lo = hi - 1;
        const uint32_t P1 = A[31 - hi], P0 = lo >= 0 ? A[31 - lo] : 0u;
        const uint32_t c0 = C & ~P1;
        const uint32_t x = (uint32_t)__popc(c0 & ~P0) | (uint32_t)__popc(c0 & P0) << 16;
        const uint32_t y = (uint32_t)__popc(C & P1 & ~P0);
        const uint32_t X = wsum(x), Y = lo >= 0 ? wsum(y) : 0u;
        const int par = s & 1;
        if ((threadIdx.x & 63) == 0) {
            wc[par][wave][0] = X;
            wc[par][wave][1] = Y;
        }
        __syncthreads();
        uint32_t sx = 0, sy = 0;
#pragma unroll
        for (int w = 0; w < kThrT / 64; w++) {
            sx += wc[par][w][0];
            sy += wc[par][w][1];
        }
        const uint32_t n00 = sx & 0xFFFFu, n01 = sx >> 16, n10 = sy;
        uint32_t d;
        if (lo < 0) {
            d = kk < n00 ? 0u : 1u;
            if (d) kk -= n00;
            C &= d ? P1 : ~P1;
            prefix |= d;
        } else {
            if (kk < n00) d = 0;
            else if (kk < n00 + n01) { d = 1; kk -= n00; }
            else if (kk < n00 + n01 + n10) { d = 2; kk -= n00 + n01; }
            else { d = 3; kk -= n00 + n01 + n10; }
            C &= (d & 2 ? P1 : ~P1) & (d & 1 ? P0 : ~P0);
            prefix |= d << lo;
        }
    }
    if (threadIdx.x == 0) {
        const float mp = 6.103515625e-05f;
        const float t = __builtin_bit_cast(float, prefix);
        t_out[0] = prefix > 0x7F800000u ? mp : (t > mp ? t : mp);
        st[0] = t0;
        st[1] = t1;
        st[2] = t2;
        st[3] = wall_clock64();
    }
}

// variant E: sp_threshold that stops once the chosen digit leaves one candidate (the answer is that key,
// read back from its bit planes by the lane that holds it)
__global__ __launch_bounds__(kThrT) void thr_early(const uint32_t *keys, uint32_t m, uint32_t k, float *t_out) {
    __shared__ uint32_t wc[2][kThrT / 64][2];
    const int wave = threadIdx.x / 64;
    uint32_t A[32], C = 0;
#pragma unroll
    for (int q = 0; q < kThrK; q++) {
        const uint32_t i = threadIdx.x + (uint32_t)q * kThrT;
        A[q] = i < m ? keys[i] : 0u;
        C |= i < m ? 1u << (31 - q) : 0u;
    }
    transpose32(A);
    uint32_t prefix = 0, kk = k, cand = m;
    bool one = false;
#pragma unroll
    for (int s = 0; s < 16; s++) {
        const int hi = 30 - 2 * s, lo = hi - 1;
        const uint32_t P1 = A[31 - hi], P0 = lo >= 0 ? A[31 - lo] : 0u;
        const uint32_t c0 = C & ~P1;
        const uint32_t x = (uint32_t)__popc(c0 & ~P0) | (uint32_t)__popc(c0 & P0) << 16;
        const uint32_t y = (uint32_t)__popc(C & P1 & ~P0);
        const uint32_t X = wsum(x), Y = lo >= 0 ? wsum(y) : 0u;
        const int par = s & 1;
        if ((threadIdx.x & 63) == 0) {
            wc[par][wave][0] = X;
            wc[par][wave][1] = Y;
        }
        __syncthreads();
        uint32_t sx = 0, sy = 0;
#pragma unroll
        for (int w = 0; w < kThrT / 64; w++) {
            sx += wc[par][w][0];
            sy += wc[par][w][1];
        }
        const uint32_t n00 = sx & 0xFFFFu, n01 = sx >> 16, n10 = sy;
        uint32_t d, nd;
        if (lo < 0) {
            d = kk < n00 ? 0u : 1u;
            nd = d ? cand - n00 : n00;
            if (d) kk -= n00;
            C &= d ? P1 : ~P1;
            prefix |= d;
        } else {
            if (kk < n00) { d = 0; nd = n00; }
            else if (kk < n00 + n01) { d = 1; kk -= n00; nd = n01; }
            else if (kk < n00 + n01 + n10) { d = 2; kk -= n00 + n01; nd = n10; }
            else { d = 3; kk -= n00 + n01 + n10; nd = cand - n00 - n01 - n10; }
            C &= (d & 2 ? P1 : ~P1) & (d & 1 ? P0 : ~P0);
            prefix |= d << lo;
        }
        cand = nd;
        if (cand == 1 && lo > 0) {  // (uniform) one key left: its lane writes it
            one = true;
            break;
        }
    }
    const float mp = 6.103515625e-05f;
    if (one) {
        if (C) {
            const int q = __builtin_clz(C);  // bit 31 - q
            uint32_t key = 0;
#pragma unroll
            for (int p = 0; p < 31; p++) key |= ((A[31 - p] >> (31 - q)) & 1u) << p;
            const float t = __builtin_bit_cast(float, key);
            t_out[0] = key > 0x7F800000u ? mp : (t > mp ? t : mp);
        }
        return;
    }
    if (threadIdx.x == 0) {
        const float t = __builtin_bit_cast(float, prefix);
        t_out[0] = prefix > 0x7F800000u ? mp : (t > mp ? t : mp);
    }
}

// variant W: four waves, 64 keys per lane (two 32 x 32 transposes), so each step sums four waves' counts
__global__ __launch_bounds__(256) void thr_w4(const uint32_t *keys, uint32_t m, uint32_t k, float *t_out) {
    __shared__ uint32_t wc[2][4][2];
    const int wave = threadIdx.x / 64;
    uint32_t A[32], B[32], CA = 0, CB = 0;
#pragma unroll
    for (int q = 0; q < 32; q++) {
        const uint32_t i = threadIdx.x + (uint32_t)q * 256, j = i + 32 * 256;
        A[q] = i < m ? keys[i] : 0u;
        B[q] = j < m ? keys[j] : 0u;
        CA |= i < m ? 1u << (31 - q) : 0u;
        CB |= j < m ? 1u << (31 - q) : 0u;
    }
    transpose32(A);
    transpose32(B);
    uint32_t prefix = 0, kk = k;
#pragma unroll
    for (int s = 0; s < 16; s++) {
        const int hi = 30 - 2 * s, lo = hi - 1;
        const uint32_t PA1 = A[31 - hi], PA0 = lo >= 0 ? A[31 - lo] : 0u;
        const uint32_t PB1 = B[31 - hi], PB0 = lo >= 0 ? B[31 - lo] : 0u;
        const uint32_t a0 = CA & ~PA1, b0 = CB & ~PB1;
        const uint32_t x = (uint32_t)(__popc(a0 & ~PA0) + __popc(b0 & ~PB0)) |
                           (uint32_t)(__popc(a0 & PA0) + __popc(b0 & PB0)) << 16;
        const uint32_t y = (uint32_t)(__popc(CA & PA1 & ~PA0) + __popc(CB & PB1 & ~PB0));
        const uint32_t X = wsum(x), Y = lo >= 0 ? wsum(y) : 0u;
        const int par = s & 1;
        if ((threadIdx.x & 63) == 0) {
            wc[par][wave][0] = X;
            wc[par][wave][1] = Y;
        }
        __syncthreads();
        uint32_t sx = 0, sy = 0;
#pragma unroll
        for (int w = 0; w < 4; w++) {
            sx += wc[par][w][0];
            sy += wc[par][w][1];
        }
        const uint32_t n00 = sx & 0xFFFFu, n01 = sx >> 16, n10 = sy;
        uint32_t d;
        if (lo < 0) {
            d = kk < n00 ? 0u : 1u;
            if (d) kk -= n00;
            CA &= d ? PA1 : ~PA1;
            CB &= d ? PB1 : ~PB1;
            prefix |= d;
        } else {
            if (kk < n00) d = 0;
            else if (kk < n00 + n01) { d = 1; kk -= n00; }
            else if (kk < n00 + n01 + n10) { d = 2; kk -= n00 + n01; }
            else { d = 3; kk -= n00 + n01 + n10; }
            CA &= (d & 2 ? PA1 : ~PA1) & (d & 1 ? PA0 : ~PA0);
            CB &= (d & 2 ? PB1 : ~PB1) & (d & 1 ? PB0 : ~PB0);
            prefix |= d << lo;
        }
    }
    if (threadIdx.x == 0) {
        const float mp = 6.103515625e-05f;
        const float t = __builtin_bit_cast(float, prefix);
        t_out[0] = prefix > 0x7F800000u ? mp : (t > mp ? t : mp);
    }
}

// variant D: four bits a step (8 steps, the last re-deciding bit 3), 16 bucket counts per lane packed two to a
// word (8 wave sums a step), early exit at one candidate
__device__ __forceinline__ void select4(uint32_t (&A)[32], uint32_t C, uint32_t m, uint32_t k, float *t_out,
                                        uint32_t (*wc)[kThrT / 64][8]) {
    const int wave = threadIdx.x / 64;
    uint32_t prefix = 0, kk = k, cand = m;
    bool one = false;
#pragma unroll
    for (int s = 0; s < 8; s++) {
        const int hi = s < 7 ? 30 - 4 * s : 3, lo = hi - 3;
        const uint32_t P3 = A[31 - hi], P2 = A[31 - (hi - 1)], P1 = A[31 - (hi - 2)], P0 = A[31 - lo];
        uint32_t msk[16];
#pragma unroll
        for (int d = 0; d < 16; d++)
            msk[d] = C & (d & 8 ? P3 : ~P3) & (d & 4 ? P2 : ~P2) & (d & 2 ? P1 : ~P1) & (d & 1 ? P0 : ~P0);
        uint32_t w[8];
#pragma unroll
        for (int j = 0; j < 8; j++) w[j] = wsum((uint32_t)__popc(msk[2 * j]) | (uint32_t)__popc(msk[2 * j + 1]) << 16);
        const int par = s & 1;
        if ((threadIdx.x & 63) == 0) {
#pragma unroll
            for (int j = 0; j < 8; j++) wc[par][wave][j] = w[j];
        }
        __syncthreads();
        uint32_t tot[8];
#pragma unroll
        for (int j = 0; j < 8; j++) tot[j] = 0;
#pragma unroll
        for (int q = 0; q < kThrT / 64; q++) {
            const uint4 a = *(const uint4 *)&wc[par][q][0], b = *(const uint4 *)&wc[par][q][4];
            tot[0] += a.x; tot[1] += a.y; tot[2] += a.z; tot[3] += a.w;
            tot[4] += b.x; tot[5] += b.y; tot[6] += b.z; tot[7] += b.w;
        }
        uint32_t d = 15, cum = 0, nd = 0;
        bool found = false;
#pragma unroll
        for (int q = 0; q < 16; q++) {
            const uint32_t c = q & 1 ? tot[q / 2] >> 16 : tot[q / 2] & 0xFFFFu;
            if (!found && kk < cum + c) { d = (uint32_t)q; nd = c; found = true; kk -= cum; }
            cum += c;
        }
        C = msk[0];
#pragma unroll
        for (int q = 1; q < 16; q++) C = d == (uint32_t)q ? msk[q] : C;
        prefix |= d << lo;
        cand = nd;
        if (cand == 1) {
            one = true;
            break;
        }
    }
    const float mp = 6.103515625e-05f;
    if (one) {
        if (C) {
            const int q = __builtin_clz(C);
            uint32_t key = 0;
#pragma unroll
            for (int p = 0; p < 31; p++) key |= ((A[31 - p] >> (31 - q)) & 1u) << p;
            const float t = __builtin_bit_cast(float, key);
            t_out[0] = key > 0x7F800000u ? mp : (t > mp ? t : mp);
        }
        return;
    }
    if (threadIdx.x == 0) {
        const float t = __builtin_bit_cast(float, prefix);
        t_out[0] = prefix > 0x7F800000u ? mp : (t > mp ? t : mp);
    }
}
__global__ __launch_bounds__(kThrT) void thr_d4(const uint32_t *keys, uint32_t m, uint32_t k, float *t_out) {
    __shared__ __attribute__((aligned(16))) uint32_t wc[2][kThrT / 64][8];
    uint32_t A[32], C = 0;
#pragma unroll
    for (int q = 0; q < kThrK; q++) {
        const uint32_t i = threadIdx.x + (uint32_t)q * kThrT;
        A[q] = i < m ? keys[i] : 0u;
        C |= i < m ? 1u << (31 - q) : 0u;
    }
    transpose32(A);
    select4(A, C, m, k, t_out, wc);
}
// variant F: the gather and the select in one launch — 32 workgroups gather 512 keys each, count themselves in
// after a device-scope fence; the last to arrive selects (D's select) over all the keys (counter: monotonic,
// the host passes the value the last arrival sees)
__global__ __launch_bounds__(kThrT) void thr_fused(const float *g, const uint32_t *idx, uint32_t *keys, uint32_t m,
                                                   uint32_t k, float *t_out, uint32_t *count, uint32_t last) {
    __shared__ __attribute__((aligned(16))) uint32_t wc[2][kThrT / 64][8];
    __shared__ uint32_t s_last;
    const uint32_t i = blockIdx.x * kThrT + threadIdx.x;
    if (i < m) keys[i] = abs_key(g[idx[i]]);
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) s_last = atomicAdd(count, 1u) == last ? 1u : 0u;
    __syncthreads();
    if (!s_last) return;
    __threadfence();
    uint32_t A[32], C = 0;
#pragma unroll
    for (int q = 0; q < kThrK; q++) {
        const uint32_t j = threadIdx.x + (uint32_t)q * kThrT;
        A[q] = j < m ? __hip_atomic_load(keys + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
        C |= j < m ? 1u << (31 - q) : 0u;
    }
    transpose32(A);
    select4(A, C, m, k, t_out, wc);
}

__global__ void synth_vals(float *g, size_t n, uint32_t seed) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    // Box-Muller over a hash: N(0, 1)-like values, as the bench's gradients
    uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull ^ seed;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    const float u1 = ((uint32_t)z + 1.0f) * 2.3283064e-10f, u2 = (uint32_t)(z >> 32) * 2.3283064e-10f;
    g[i] = sqrtf(-2.0f * logf(u1)) * cosf(6.2831853f * u2);
}

}  // namespace

int main(int argc, char **argv) {
    const int K = argc > 1 ? atoi(argv[1]) : 200;
    const size_t n = 54693, m = kSampleMax;
    const uint32_t k = (uint32_t)threshold_rank(m, 0.1f);
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    float *g, *t_dev, *t_host;
    uint32_t *idx_dev, *idx_host, *keys;
    uint64_t *st;
    CK(hipMalloc((void **)&g, n * sizeof(float)));
    CK(hipMalloc((void **)&t_dev, 16 * sizeof(float)));
    CK(hipMalloc((void **)&idx_dev, m * sizeof(uint32_t)));
    CK(hipMalloc((void **)&keys, m * sizeof(uint32_t)));
    CK(hipMalloc((void **)&st, 8 * sizeof(uint64_t)));
    CK(hipHostMalloc((void **)&idx_host, m * sizeof(uint32_t), hipHostMallocDefault));
    CK(hipHostMalloc((void **)&t_host, 16 * sizeof(float), hipHostMallocDefault));
    hipLaunchKernelGGL(synth_vals, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, g, n, 7u);
    std::mt19937_64 rng(11);
    std::vector<uint32_t> perm(n);
    for (size_t i = 0; i < n; i++) perm[i] = (uint32_t)i;
    std::shuffle(perm.begin(), perm.end(), rng);
    for (size_t i = 0; i < m; i++) idx_host[i] = perm[i];
    CK(hipMemcpyAsync(idx_dev, idx_host, m * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    uint32_t *idx_mapped = nullptr;
    CK(hipHostGetDevicePointer((void **)&idx_mapped, idx_host, 0));
    CK(hipStreamSynchronize(s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto gather = [&](const uint32_t *idx) {
        hipLaunchKernelGGL(sp_gather_keys, dim3((unsigned)((m + kGatherT - 1) / kGatherT)), dim3(kGatherT), 0, s, g,
                           idx, keys, (uint32_t)m);
    };
    uint32_t *count = nullptr, fused_calls = 0;
    CK(hipMalloc((void **)&count, 64));
    CK(hipMemsetAsync(count, 0, 64, s));
    const uint32_t G = (uint32_t)((m + kThrT - 1) / kThrT);
    auto select = [&](int v, float *out) {
        if (v == 4)
            hipLaunchKernelGGL(thr_d4, dim3(1), dim3(kThrT), 0, s, (const uint32_t *)keys, (uint32_t)m, k, out);
        else if (v == 0)
            hipLaunchKernelGGL(sp_threshold, dim3(1), dim3(kThrT), 0, s, (const uint32_t *)keys, (const float *)g,
                               (uint32_t)m, k, out);
        else if (v == 1)
            hipLaunchKernelGGL(thr_early, dim3(1), dim3(kThrT), 0, s, (const uint32_t *)keys, (uint32_t)m, k, out);
        else if (v == 2)
            hipLaunchKernelGGL(thr_w4, dim3(1), dim3(256), 0, s, (const uint32_t *)keys, (uint32_t)m, k, out);
        else
            hipLaunchKernelGGL(thr_stamped, dim3(1), dim3(kThrT), 0, s, (const uint32_t *)keys, (uint32_t)m, k, out,
                               st);
    };
    const char *names[] = {"sp_threshold (library)", "early exit at one candidate", "four waves, 64 keys a lane",
                           "stamped copy", "four bits a step, early exit", "gather + select in one launch (4 bits)"};
    auto fused = [&](const uint32_t *idx, float *out) {
        fused_calls++;
        hipLaunchKernelGGL(thr_fused, dim3(G), dim3(kThrT), 0, s, (const float *)g, idx, keys, (uint32_t)m, k, out,
                           count, fused_calls * G - 1);
    };
    printf("{\"workload\": \"config-1 push threshold: %zu values, %zu sampled, k = %u\", \"K\": %d", n, m, k, K);
    // the library's result
    gather(idx_dev);
    select(0, t_dev);
    CK(hipMemcpyAsync(t_host, t_dev, sizeof(float), hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    const float want = t_host[0];
    printf(", \"t\": %.9g", (double)want);
    for (int src = 0; src < 2; src++) {
        const uint32_t *idx = src ? idx_mapped : idx_dev;
        printf(", \"%s\": {", src ? "idx_pinned" : "idx_hbm");
        for (int v = 0; v < 6; v++) {
            if (v == 5) {  // one launch: the pair only
                fused(idx, t_dev + 1);
                CK(hipMemcpyAsync(t_host, t_dev + 1, sizeof(float), hipMemcpyDeviceToHost, s));
                CK(hipStreamSynchronize(s));
                const bool ok = t_host[0] == want;
                for (int w = 0; w < 10; w++) fused(idx, t_dev + 1);
                CK(hipEventRecord(e0, s));
                for (int i = 0; i < K; i++) fused(idx, t_dev + 1);
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float bb = 0;
                CK(hipEventElapsedTime(&bb, e0, e1));
                std::vector<float> xs;
                for (int i = 0; i < K / 4 + 5; i++) {
                    CK(hipEventRecord(e0, s));
                    fused(idx, t_dev + 1);
                    CK(hipEventRecord(e1, s));
                    CK(hipEventSynchronize(e1));
                    float x = 0;
                    CK(hipEventElapsedTime(&x, e0, e1));
                    xs.push_back(x);
                }
                std::sort(xs.begin(), xs.end());
                printf(", \"%s\": {\"ok\": %s, \"pair_us_back_to_back\": %.2f, \"pair_us\": %.2f}", names[v],
                       ok ? "true" : "false", bb * 1e3 / K, xs[xs.size() / 2] * 1e3);
                continue;
            }
            // check
            gather(idx);
            select(v, t_dev + 1);
            CK(hipMemcpyAsync(t_host, t_dev + 1, sizeof(float), hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
            const bool ok = t_host[0] == want;
            // back to back
            for (int w = 0; w < 10; w++) { gather(idx); select(v, t_dev + 1); }
            CK(hipEventRecord(e0, s));
            for (int i = 0; i < K; i++) { gather(idx); select(v, t_dev + 1); }
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float bb = 0;
            CK(hipEventElapsedTime(&bb, e0, e1));
            // one at a time: gather alone, select alone, the pair
            double lat[3] = {0, 0, 0};
            for (int part = 0; part < 3; part++) {
                std::vector<float> xs;
                for (int i = 0; i < K / 4 + 5; i++) {
                    if (part == 1) { gather(idx); CK(hipStreamSynchronize(s)); }
                    CK(hipEventRecord(e0, s));
                    if (part != 1) gather(idx);
                    if (part != 0) select(v, t_dev + 1);
                    CK(hipEventRecord(e1, s));
                    CK(hipEventSynchronize(e1));
                    float x = 0;
                    CK(hipEventElapsedTime(&x, e0, e1));
                    xs.push_back(x);
                }
                std::sort(xs.begin(), xs.end());
                lat[part] = xs[xs.size() / 2] * 1e3;
            }
            printf("%s\"%s\": {\"ok\": %s, \"pair_us_back_to_back\": %.2f, \"gather_us\": %.2f, \"select_us\": %.2f, "
                   "\"pair_us\": %.2f",
                   v ? ", " : "", names[v], ok ? "true" : "false", bb * 1e3 / K, lat[0], lat[1], lat[2]);
            if (v == 3) {
                uint64_t h[4];
                std::vector<double> a, b, c;
                for (int i = 0; i < 41; i++) {
                    gather(idx);
                    select(3, t_dev + 1);
                    CK(hipMemcpyAsync(h, st, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
                    CK(hipStreamSynchronize(s));
                    a.push_back((h[1] - h[0]) * 0.01);
                    b.push_back((h[2] - h[1]) * 0.01);
                    c.push_back((h[3] - h[2]) * 0.01);
                }
                std::sort(a.begin(), a.end());
                std::sort(b.begin(), b.end());
                std::sort(c.begin(), c.end());
                printf(", \"stamps_us\": {\"load\": %.2f, \"transpose\": %.2f, \"steps\": %.2f}", a[20], b[20], c[20]);
            }
            printf("}");
        }
        printf("}");
    }
    printf("}\n");
    return 0;
}
