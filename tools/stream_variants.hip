// stream_variants.hip — HBM streaming micro-benchmarks on gfx950 (measurement tool,
// not part of the product).  Picks the store policy, unroll and grid shape for
// the reduction path's elementwise kernels and records the copy ceiling.
//
// Each timed launch works on a different buffer set (ROT sets rotating through
// > 1.5 GiB), so the 256 MiB Infinity Cache cannot serve re-reads: the numbers
// are HBM numbers.  Data is random (non-zero).
//
//   hipcc --offload-arch=gfx950 -O3 -o stream_variants stream_variants.hip
//   ./stream_variants [n_elems]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
    } while (0)

constexpr int ROT = 6;      // buffer sets rotated between launches
constexpr int MAXK = 8;

template <bool NTS> __device__ __forceinline__ void st(f4 *p, f4 v) {
    if constexpr (NTS) __builtin_nontemporal_store(v, p);
    else *p = v;
}

struct Args {
    const f4 *in[MAXK];
    f4 *out;
    f4 *zero;
};

// out = (sum of K inputs) (* 0.5); zero[] = 0 if ZERO
template <int K, bool ZERO, int U, bool NTS>
__global__ __launch_bounds__(256) void k_red(Args a, size_t nvec) {
    size_t tid = (size_t)blockIdx.x * 256 + threadIdx.x, stride = (size_t)gridDim.x * 256;
    size_t v = tid;
    for (; v + (U - 1) * stride < nvec; v += U * stride) {
        f4 r[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            r[u] = a.in[0][v + u * stride];
#pragma unroll
            for (int j = 1; j < K; j++) r[u] += a.in[j][v + u * stride];
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            st<NTS>(a.out + v + u * stride, K > 1 ? r[u] * 0.5f : r[u]);
            if constexpr (ZERO) st<NTS>(a.zero + v + u * stride, f4{0, 0, 0, 0});
        }
    }
    for (; v < nvec; v += stride) {
        f4 r = a.in[0][v];
#pragma unroll
        for (int j = 1; j < K; j++) r += a.in[j][v];
        st<NTS>(a.out + v, K > 1 ? r * 0.5f : r);
        if constexpr (ZERO) st<NTS>(a.zero + v, f4{0, 0, 0, 0});
    }
}


template <bool NTL> __device__ __forceinline__ f4 ldv(const f4 *p) {
    if constexpr (NTL) return __builtin_nontemporal_load(p);
    else return *p;
}

// one-shot, B threads per block, VPT adjacent 16-B vectors per thread
template <int K, bool ZERO, int B, int VPT, bool NTL>
__global__ __launch_bounds__(B) void k_red2(Args a, size_t nvec) {
    size_t base = ((size_t)blockIdx.x * B) * VPT + threadIdx.x;
    f4 r[VPT];
#pragma unroll
    for (int u = 0; u < VPT; u++) {
        size_t v = base + (size_t)u * B;
        if (v < nvec) {
            r[u] = ldv<NTL>(a.in[0] + v);
#pragma unroll
            for (int j = 1; j < K; j++) r[u] += ldv<NTL>(a.in[j] + v);
        }
    }
#pragma unroll
    for (int u = 0; u < VPT; u++) {
        size_t v = base + (size_t)u * B;
        if (v < nvec) {
            st<true>(a.out + v, K > 1 ? r[u] * 0.5f : r[u]);
            if constexpr (ZERO) st<true>(a.zero + v, f4{0, 0, 0, 0});
        }
    }
}

__global__ void k_fill(f4 *p, size_t nvec, unsigned seed) {
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    for (; i < nvec; i += (size_t)gridDim.x * 256) {
        unsigned h = (unsigned)i * 2654435761u ^ seed;
        p[i] = f4{(float)(h & 0xFFFF), (float)(h >> 16), (float)(h & 0xFF), 1.0f} * 1e-4f;
    }
}

struct Pool {
    std::vector<f4 *> bufs;  // ROT * (MAXK + 2) buffers
    size_t nvec;
};

template <int K, bool ZERO, int U, bool NTS>
void row(Pool &P, int cus, int bpc, hipStream_t s, const char *name) {
    int blocks = bpc > 0 ? cus * bpc : (int)((P.nvec + 256 * U - 1) / (256 * U));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> t;
    for (int r = 0; r < 2 * ROT + 2; r++) {
        int set = r % ROT;
        Args a{};
        for (int j = 0; j < K; j++) a.in[j] = P.bufs[set * (MAXK + 2) + j];
        a.out = P.bufs[set * (MAXK + 2) + MAXK];
        a.zero = ZERO ? (f4 *)a.in[0] : nullptr;  // zero the first input (pull_grads: residual)
        CK(hipEventRecord(e0, s));
        hipLaunchKernelGGL((k_red<K, ZERO, U, NTS>), dim3(blocks), dim3(256), 0, s, a, P.nvec);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 2) t.push_back(ms);
        if (ZERO) hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, s, (f4 *)a.in[0], P.nvec, 77u + r);
    }
    std::sort(t.begin(), t.end());
    double ms = t[t.size() / 2];
    double bytes = (double)(K + 1 + (ZERO ? 1 : 0)) * 16 * P.nvec;
    double gbs = bytes / (ms * 1e-3) / 1e9;
    printf("%-14s U=%d nts=%d bpc=%-3d blocks=%-7d %9.2f us %8.1f GB/s  %.3f of 8000\n", name, U, NTS, bpc, blocks,
           ms * 1e3, gbs, gbs / 8000.0);
    fflush(stdout);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

template <int K, bool ZERO>
void sweep(Pool &P, int cus, hipStream_t s, const char *name) {
    row<K, ZERO, 1, true>(P, cus, 0, s, name);
    row<K, ZERO, 2, true>(P, cus, 0, s, name);
    row<K, ZERO, 4, true>(P, cus, 0, s, name);
    row<K, ZERO, 1, false>(P, cus, 0, s, name);
    row<K, ZERO, 4, false>(P, cus, 0, s, name);
    row<K, ZERO, 1, true>(P, cus, 8, s, name);
    row<K, ZERO, 4, true>(P, cus, 8, s, name);
    row<K, ZERO, 4, true>(P, cus, 16, s, name);
    row<K, ZERO, 2, true>(P, cus, 32, s, name);
}


template <int K, bool ZERO, int B, int VPT, bool NTL>
void row2(Pool &P, hipStream_t s, const char *name) {
    int blocks = (int)((P.nvec + (size_t)B * VPT - 1) / ((size_t)B * VPT));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> t;
    for (int r = 0; r < 2 * ROT + 2; r++) {
        int set = r % ROT;
        Args a{};
        for (int j = 0; j < K; j++) a.in[j] = P.bufs[set * (MAXK + 2) + j];
        a.out = P.bufs[set * (MAXK + 2) + MAXK];
        a.zero = ZERO ? (f4 *)a.in[0] : nullptr;
        CK(hipEventRecord(e0, s));
        hipLaunchKernelGGL((k_red2<K, ZERO, B, VPT, NTL>), dim3(blocks), dim3(B), 0, s, a, P.nvec);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 2) t.push_back(ms);
        if (ZERO) hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, s, (f4 *)a.in[0], P.nvec, 77u + r);
    }
    std::sort(t.begin(), t.end());
    double ms = t[t.size() / 2];
    double bytes = (double)(K + 1 + (ZERO ? 1 : 0)) * 16 * P.nvec;
    double gbs = bytes / (ms * 1e-3) / 1e9;
    printf("%-14s B=%-4d VPT=%d ntl=%d blocks=%-7d %9.2f us %8.1f GB/s  %.3f of 8000\n", name, B, VPT, NTL, blocks,
           ms * 1e3, gbs, gbs / 8000.0);
    fflush(stdout);
}

template <int K, bool ZERO>
void sweep2(Pool &P, hipStream_t s, const char *name) {
    row2<K, ZERO, 256, 1, false>(P, s, name);
    row2<K, ZERO, 512, 1, false>(P, s, name);
    row2<K, ZERO, 1024, 1, false>(P, s, name);
    row2<K, ZERO, 256, 2, false>(P, s, name);
    row2<K, ZERO, 256, 4, false>(P, s, name);
    row2<K, ZERO, 128, 1, false>(P, s, name);
    row2<K, ZERO, 64, 1, false>(P, s, name);
    row2<K, ZERO, 256, 1, true>(P, s, name);
}

// pull_grads(n=1) shape: residual (rotating, fresh) -> grad (FIXED or rotating), residual = 0.
// Back-to-back launches timed as one span (like bench.py) or one event pair per launch.
void pull_shape(Pool &P, hipStream_t s, bool fixed_out, bool per_launch_events, int B) {
    const int L = 12;
    int blocks = (int)((P.nvec + B - 1) / B);
    hipEvent_t ev[2 * L + 2];
    for (int q = 0; q < 2 * L + 2; q++) CK(hipEventCreate(&ev[q]));
    for (int r = 0; r < ROT; r++) hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, s, (f4 *)P.bufs[r * (MAXK + 2)], P.nvec, 5u + r);
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(ev[0], s));
    for (int i = 0; i < L; i++) {
        int set = i % ROT;
        Args a{};
        a.in[0] = P.bufs[set * (MAXK + 2)];
        a.out = fixed_out ? P.bufs[MAXK] : P.bufs[set * (MAXK + 2) + MAXK];
        a.zero = (f4 *)a.in[0];
        if (per_launch_events) CK(hipEventRecord(ev[2 + 2 * i], s));
        if (B == 256) hipLaunchKernelGGL((k_red2<1, true, 256, 1, false>), dim3(blocks), dim3(256), 0, s, a, P.nvec);
        else hipLaunchKernelGGL((k_red2<1, true, 64, 1, false>), dim3(blocks), dim3(64), 0, s, a, P.nvec);
        if (per_launch_events) CK(hipEventRecord(ev[3 + 2 * i], s));
        if (i == ROT - 1) {  // refill the residuals for the second lap (untimed in per-launch mode)
        }
    }
    CK(hipEventRecord(ev[1], s));
    CK(hipStreamSynchronize(s));
    float total;
    CK(hipEventElapsedTime(&total, ev[0], ev[1]));
    double per = total / L, sum = 0;
    if (per_launch_events) {
        for (int i = 0; i < L; i++) { float m; CK(hipEventElapsedTime(&m, ev[2 + 2 * i], ev[3 + 2 * i])); sum += m; }
    }
    double bytes = 12.0 * 4 * P.nvec;
    printf("pull n=1 B=%-3d out=%s events=%s  span/launch %8.2f us %7.1f GB/s", B, fixed_out ? "fixed" : "rotating",
           per_launch_events ? "per-launch" : "span", per * 1e3, bytes / (per * 1e-3) / 1e9);
    if (per_launch_events) printf("  | event avg %8.2f us %7.1f GB/s", sum / L * 1e3, bytes / (sum / L * 1e-3) / 1e9);
    printf("\n");
    fflush(stdout);
    for (int q = 0; q < 2 * L + 2; q++) CK(hipEventDestroy(ev[q]));
}

// The pull shape launched in isolation: a host wait before every launch (the
// GPU idles ~10-20 us between kernels) vs the same launches back to back —
// separates a kernel's burst rate from the sustained streaming rate.
void pull_isolated(Pool &P, hipStream_t s, bool idle_between, int L) {
    const int B = 64;
    int blocks = (int)((P.nvec + B - 1) / B);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> t;
    for (int r = 0; r < ROT; r++) hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, s, (f4 *)P.bufs[r * (MAXK + 2)], P.nvec, 9u + r);
    CK(hipStreamSynchronize(s));
    for (int i = 0; i < L; i++) {
        int set = i % ROT;
        Args a{};
        a.in[0] = P.bufs[set * (MAXK + 2)];
        a.out = P.bufs[set * (MAXK + 2) + MAXK];
        a.zero = (f4 *)a.in[0];
        if (idle_between) CK(hipStreamSynchronize(s));
        CK(hipEventRecord(e0, s));
        hipLaunchKernelGGL((k_red2<1, true, 64, 1, false>), dim3(blocks), dim3(64), 0, s, a, P.nvec);
        CK(hipEventRecord(e1, s));
        if (idle_between) {
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t.push_back(ms);
        }
        if (i % ROT == ROT - 1) {  // refill the residuals the lap zeroed (outside the timed launches)
            if (!idle_between) CK(hipStreamSynchronize(s));
            for (int r = 0; r < ROT; r++)
                hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, s, (f4 *)P.bufs[r * (MAXK + 2)], P.nvec, 9u + r + i);
            CK(hipStreamSynchronize(s));
        }
    }
    CK(hipStreamSynchronize(s));
    if (!idle_between) {  // back to back inside each lap: time one lap as a span
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < ROT; i++) {
            Args a{};
            a.in[0] = P.bufs[i * (MAXK + 2)];
            a.out = P.bufs[i * (MAXK + 2) + MAXK];
            a.zero = (f4 *)a.in[0];
            hipLaunchKernelGGL((k_red2<1, true, 64, 1, false>), dim3(blocks), dim3(64), 0, s, a, P.nvec);
        }
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t.push_back(ms / ROT);
    }
    std::sort(t.begin(), t.end());
    double ms = t[t.size() / 2];
    double bytes = 12.0 * 4 * P.nvec;
    printf("pull n=1 B=64 %-26s %9.2f us %8.1f GB/s  %.3f of 8000\n", idle_between ? "isolated (host wait before)"
           : "back-to-back lap of 6", ms * 1e3, bytes / (ms * 1e-3) / 1e9, bytes / (ms * 1e-3) / 1e9 / 8000.0);
    fflush(stdout);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

__global__ void k_empty(int *p) {
    if (p && threadIdx.x == 0 && blockIdx.x == 0) p[0] = 0;
}

// What precedes a timed pull-shape launch (host wait between pairs):
//   0 nothing | 1 fill of another 256 MiB buffer | 2 empty kernel |
//   3 fill of 16 MiB | 4 a pull-shape launch on another set | 5 fill 64 MiB
void pull_after(Pool &P, hipStream_t s, int what, int L) {
    const int B = 64;
    int blocks = (int)((P.nvec + B - 1) / B);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> t;
    for (int r = 0; r < ROT; r++) hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, s, (f4 *)P.bufs[r * (MAXK + 2)], P.nvec, 3u + r);
    CK(hipStreamSynchronize(s));
    for (int i = 0; i < L; i++) {
        const int set = i % ROT, other = (i + 3) % ROT;
        Args a{};
        a.in[0] = P.bufs[set * (MAXK + 2)];
        a.out = P.bufs[set * (MAXK + 2) + MAXK];
        a.zero = (f4 *)a.in[0];
        f4 *scratch = P.bufs[other * (MAXK + 2) + 1];  // an input slot the pull shape never touches
        if (what == 1) hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, s, scratch, P.nvec, 1u + i);
        if (what == 2) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, (int *)nullptr);
        if (what == 3) hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, s, scratch, P.nvec / 16, 1u + i);
        if (what == 5) hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, s, scratch, P.nvec / 4, 1u + i);
        if (what == 4) {
            Args b{};
            b.in[0] = P.bufs[other * (MAXK + 2) + 1];
            b.out = P.bufs[other * (MAXK + 2) + 2];
            b.zero = nullptr;
            hipLaunchKernelGGL((k_red2<1, false, 64, 1, false>), dim3(blocks), dim3(64), 0, s, b, P.nvec);
        }
        CK(hipEventRecord(e0, s));
        hipLaunchKernelGGL((k_red2<1, true, 64, 1, false>), dim3(blocks), dim3(64), 0, s, a, P.nvec);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t.push_back(ms);
        hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, s, (f4 *)a.in[0], P.nvec, 11u + i);  // refill what it zeroed
        CK(hipStreamSynchronize(s));
    }
    std::sort(t.begin(), t.end());
    double ms = t[t.size() / 2];
    double bytes = 12.0 * 4 * P.nvec;
    static const char *nm[] = {"nothing", "fill 256 MiB other", "empty kernel", "fill 16 MiB", "copy 256 MiB other",
                               "fill 64 MiB"};
    printf("pull after %-20s %9.2f us %8.1f GB/s  %.3f of 8000\n", nm[what], ms * 1e3,
           bytes / (ms * 1e-3) / 1e9, bytes / (ms * 1e-3) / 1e9 / 8000.0);
    fflush(stdout);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

// Cache-policy variants of the pull shape (buffer loads / stores with explicit
// sc0 / sc1 / nt bits; aux: sc0 = 1, nt = 2, sc1 = 16), timed as the bench
// runs them: back-to-back launches over freshly filled buffers.
template <int LP, int SP>
__global__ __launch_bounds__(64) void k_pol(const f4 *src, f4 *dst, f4 *zero, unsigned nvec) {
    const unsigned v = blockIdx.x * 64 + threadIdx.x;
    if (v >= nvec) return;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)src, 0, 0x7FFFFFFF, 0x00020000);
    __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void *)dst, 0, 0x7FFFFFFF, 0x00020000);
    __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc((void *)zero, 0, 0x7FFFFFFF, 0x00020000);
    f4 x = __builtin_amdgcn_raw_buffer_load_b128(rs, v * 16, 0, LP);
    __builtin_amdgcn_raw_buffer_store_b128(x, rd, v * 16, 0, SP);
    __builtin_amdgcn_raw_buffer_store_b128(f4{0, 0, 0, 0}, rz, v * 16, 0, SP);
}

template <int LP, int SP>
void pol_row(Pool &P, hipStream_t s, const char *name) {
    const unsigned nvec = (unsigned)P.nvec;
    const int blocks = (int)((P.nvec + 63) / 64);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> t;
    for (int lap = 0; lap < 4; lap++) {
        for (int r = 0; r < ROT; r++)
            hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, s, (f4 *)P.bufs[r * (MAXK + 2)], P.nvec, 21u + r + lap);
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < ROT; i++) {
            f4 *in = P.bufs[i * (MAXK + 2)], *out = P.bufs[i * (MAXK + 2) + MAXK];
            if (LP < 0) {
                Args a{};
                a.in[0] = in;
                a.out = out;
                a.zero = in;
                hipLaunchKernelGGL((k_red2<1, true, 64, 1, false>), dim3(blocks), dim3(64), 0, s, a, P.nvec);
            } else {
                hipLaunchKernelGGL((k_pol<LP < 0 ? 0 : LP, SP>), dim3(blocks), dim3(64), 0, s, in, out, in, nvec);
            }
        }
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (lap) t.push_back(ms / ROT);
    }
    std::sort(t.begin(), t.end());
    double ms = t[t.size() / 2];
    double bytes = 12.0 * 4 * P.nvec;
    printf("pull b2b %-32s %9.2f us %8.1f GB/s  %.3f of 8000\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9,
           bytes / (ms * 1e-3) / 1e9 / 8000.0);
    fflush(stdout);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

// kR1W (sum_scale shape) with explicit load / store cache policies
template <int K, int LP, int SP>
__global__ __launch_bounds__(64) void k_polk(Args a, unsigned nvec) {
    const unsigned v = blockIdx.x * 64 + threadIdx.x;
    if (v >= nvec) return;
    f4 r = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < K; j++) {
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)a.in[j], 0, 0x7FFFFFFF, 0x00020000);
        r += __builtin_amdgcn_raw_buffer_load_b128(rs, v * 16, 0, LP);
    }
    __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void *)a.out, 0, 0x7FFFFFFF, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(r * 0.5f, rd, v * 16, 0, SP);
}

template <int K, int LP, int SP>
void polk_row(Pool &P, hipStream_t s, const char *name) {
    const int blocks = (int)((P.nvec + 63) / 64);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> t;
    for (int lap = 0; lap < 5; lap++) {
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < ROT; i++) {
            Args a{};
            for (int j = 0; j < K; j++) a.in[j] = P.bufs[i * (MAXK + 2) + j];
            a.out = P.bufs[i * (MAXK + 2) + MAXK];
            hipLaunchKernelGGL((k_polk<K, LP, SP>), dim3(blocks), dim3(64), 0, s, a, (unsigned)P.nvec);
        }
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (lap) t.push_back(ms / ROT);
    }
    std::sort(t.begin(), t.end());
    double ms = t[t.size() / 2];
    double bytes = (double)(K + 1) * 16 * P.nvec;
    printf("sum%d b2b %-28s %9.2f us %8.1f GB/s  %.3f of 8000\n", K, name, ms * 1e3, bytes / (ms * 1e-3) / 1e9,
           bytes / (ms * 1e-3) / 1e9 / 8000.0);
    fflush(stdout);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

template <int K> void polk_sweep(Pool &P, hipStream_t s) {
    polk_row<K, 0, 2>(P, s, "ld - / st nt");
    polk_row<K, 2, 2>(P, s, "ld nt / st nt (product)");
    polk_row<K, 2, 18>(P, s, "ld nt / st nt sc1");
    polk_row<K, 18, 2>(P, s, "ld nt sc1 / st nt");
    polk_row<K, 18, 18>(P, s, "ld nt sc1 / st nt sc1");
    polk_row<K, 16, 2>(P, s, "ld sc1 / st nt");
    polk_row<K, 3, 2>(P, s, "ld sc0 nt / st nt");
    polk_row<K, 2, 0>(P, s, "ld nt / st -");
}

// The training regime: ONE residual bucket reused every step — acc_residual
// (res += g, 1 launch per local batch) then pull (grad = res, res = 0) —
// with the pull's cache policy varied: is the bench's fresh-bucket gain real
// when the same 256 MiB lines come back every step?
template <int LP, int SP>
__global__ __launch_bounds__(64) void k_acc(f4 *res, const f4 *g, unsigned nvec) {
    const unsigned v = blockIdx.x * 64 + threadIdx.x;
    if (v >= nvec) return;
    __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc((void *)res, 0, 0x7FFFFFFF, 0x00020000);
    __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc((void *)g, 0, 0x7FFFFFFF, 0x00020000);
    f4 a = __builtin_amdgcn_raw_buffer_load_b128(rr, v * 16, 0, LP);
    f4 b = __builtin_amdgcn_raw_buffer_load_b128(rg, v * 16, 0, 2);
    __builtin_amdgcn_raw_buffer_store_b128(a + b, rr, v * 16, 0, SP);
}

template <int LP, int SP, int PLP = LP, int PSP = SP>
void train_row(Pool &P, hipStream_t s, const char *name, int acc_per_step) {
    const int blocks = (int)((P.nvec + 63) / 64);
    f4 *res = P.bufs[0], *grad = P.bufs[MAXK];
    hipEvent_t e0, e1, p0, p1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreate(&p0));
    CK(hipEventCreate(&p1));
    std::vector<float> t, tp;
    for (int it = 0; it < 12; it++) {
        CK(hipEventRecord(e0, s));
        for (int a = 0; a < acc_per_step; a++)
            hipLaunchKernelGGL((k_acc<LP, SP>), dim3(blocks), dim3(64), 0, s, res, (const f4 *)P.bufs[1 + (a % 4)],
                               (unsigned)P.nvec);
        CK(hipEventRecord(p0, s));
        hipLaunchKernelGGL((k_pol<PLP, PSP>), dim3(blocks), dim3(64), 0, s, (const f4 *)res, grad, res, (unsigned)P.nvec);
        CK(hipEventRecord(p1, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms, mp;
        CK(hipEventElapsedTime(&ms, e0, e1));
        CK(hipEventElapsedTime(&mp, p0, p1));
        if (it >= 2) { t.push_back(ms); tp.push_back(mp); }
    }
    std::sort(t.begin(), t.end());
    std::sort(tp.begin(), tp.end());
    printf("train step (%d acc + pull) %-22s step %8.2f us   pull %8.2f us (%.3f of 8000)\n", acc_per_step, name,
           t[t.size() / 2] * 1e3, tp[tp.size() / 2] * 1e3, 12.0 * 4 * P.nvec / (tp[tp.size() / 2] * 1e-3) / 1e9 / 8000.0);
    fflush(stdout);
}

// f16 decode shape (8 B in, 16 B out per lane) with explicit policies
template <int LP, int SP>
__global__ __launch_bounds__(64) void k_dec(const unsigned short *in, f4 *out, unsigned nvec) {
    const unsigned v = blockIdx.x * 64 + threadIdx.x;
    if (v >= nvec) return;
    __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc((void *)in, 0, 0x7FFFFFFF, 0x00020000);
    __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void *)out, 0, 0x7FFFFFFF, 0x00020000);
    typedef unsigned u2 __attribute__((ext_vector_type(2)));
    u2 h = __builtin_bit_cast(u2, __builtin_amdgcn_raw_buffer_load_b64(ri, v * 8, 0, LP));
    f4 r = {(float)__builtin_bit_cast(_Float16, (unsigned short)(h.x & 0xFFFF)),
            (float)__builtin_bit_cast(_Float16, (unsigned short)(h.x >> 16)),
            (float)__builtin_bit_cast(_Float16, (unsigned short)(h.y & 0xFFFF)),
            (float)__builtin_bit_cast(_Float16, (unsigned short)(h.y >> 16))};
    __builtin_amdgcn_raw_buffer_store_b128(r * 0.125f, ro, v * 16, 0, SP);
}

template <int LP, int SP>
void dec_row(Pool &P, hipStream_t s, const char *name) {
    const int blocks = (int)((P.nvec + 63) / 64);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> t;
    for (int lap = 0; lap < 5; lap++) {
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < ROT; i++)
            hipLaunchKernelGGL((k_dec<LP, SP>), dim3(blocks), dim3(64), 0, s,
                               (const unsigned short *)P.bufs[i * (MAXK + 2)], P.bufs[i * (MAXK + 2) + MAXK],
                               (unsigned)P.nvec);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (lap) t.push_back(ms / ROT);
    }
    std::sort(t.begin(), t.end());
    double ms = t[t.size() / 2];
    double bytes = 24.0 * P.nvec;
    printf("decode b2b %-24s %9.2f us %8.1f GB/s  %.3f of 8000\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9,
           bytes / (ms * 1e-3) / 1e9 / 8000.0);
    fflush(stdout);
}

int main(int argc, char **argv) {
    size_t n = argc > 1 ? strtoull(argv[1], 0, 10) : (size_t)1 << 24;  // 64 MiB per buffer
    Pool P;
    P.nvec = n / 4;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    for (int i = 0; i < ROT * (MAXK + 2); i++) {
        f4 *p;
        CK(hipMalloc(&p, n * 4));
        hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, s, p, P.nvec, (unsigned)i);
        P.bufs.push_back(p);
    }
    CK(hipStreamSynchronize(s));
    printf("n=%zu (%.0f MiB per buffer), %d rotating sets, CUs=%d\n", n, n * 4.0 / (1 << 20), ROT, cus);
    const char *mode = argc > 2 ? argv[2] : "all";
    if (mode[0] == 'd') {
        for (int rep = 0; rep < 2; rep++) {
            dec_row<2, 2>(P, s, "ld nt / st nt (product)");
            dec_row<0, 2>(P, s, "ld - / st nt");
            dec_row<2, 0>(P, s, "ld nt / st -");
            dec_row<2, 18>(P, s, "ld nt / st nt sc1");
            dec_row<18, 18>(P, s, "ld nt sc1 / st nt sc1");
            dec_row<2, 3>(P, s, "ld nt / st sc0 nt");
            dec_row<2, 16>(P, s, "ld nt / st sc1");
        }
    } else if (mode[0] == 't') {
        for (int rep = 0; rep < 2; rep++)
            for (int A : {0, 1, 4}) {
                train_row<0, 2>(P, s, "ld - / st nt", A);
                train_row<2, 2>(P, s, "ld nt / st nt", A);
                train_row<2, 18>(P, s, "ld nt / st nt sc1", A);
                train_row<0, 2, 2, 18>(P, s, "acc -/nt, pull nt/nt sc1", A);
                train_row<0, 2, 2, 2>(P, s, "acc -/nt, pull nt/nt", A);
                train_row<0, 0, 0, 2>(P, s, "acc -/-, pull -/nt", A);
            }
    } else if (mode[0] == 'k' && mode[1] == 'c') {
        for (int rep = 0; rep < 2; rep++) {
            polk_sweep<2>(P, s);
            polk_sweep<4>(P, s);
            polk_sweep<8>(P, s);
        }
    } else if (mode[0] == 'c') {
        for (int rep = 0; rep < 2; rep++) {
            pol_row<-1, 0>(P, s, "global ld / nt st (product)");
            pol_row<0, 2>(P, s, "ld - / st nt");
            pol_row<0, 0>(P, s, "ld - / st -");
            pol_row<2, 2>(P, s, "ld nt / st nt");
            pol_row<0, 18>(P, s, "ld - / st nt sc1");
            pol_row<0, 16>(P, s, "ld - / st sc1");
            pol_row<0, 17>(P, s, "ld - / st sc0 sc1");
            pol_row<0, 19>(P, s, "ld - / st sc0 nt sc1");
            pol_row<0, 3>(P, s, "ld - / st sc0 nt");
            pol_row<16, 2>(P, s, "ld sc1 / st nt");
            pol_row<18, 18>(P, s, "ld nt sc1 / st nt sc1");
            pol_row<17, 19>(P, s, "ld sc0 sc1 / st sc0 nt sc1");
        }
    } else if (mode[0] == 'x') {
        for (int rep = 0; rep < 2; rep++)
            for (int w : {0, 1, 2, 3, 5, 4}) pull_after(P, s, w, 14);
    } else if (mode[0] == 'i') {
        for (int rep = 0; rep < 2; rep++) {
            pull_isolated(P, s, true, 24);
            pull_isolated(P, s, false, 6);
            row2<1, true, 64, 1, false>(P, s, "copy+zero 1R2W");
            row2<1, true, 256, 1, false>(P, s, "copy+zero 1R2W");
        }
    } else if (mode[0] == 'p') {
        for (int rep = 0; rep < 2; rep++)
            for (int B : {256, 64})
                for (bool fx : {true, false})
                    for (bool pe : {false, true}) pull_shape(P, s, fx, pe, B);
    } else if (mode[0] == 'k') {  // sum_scale block size with nt loads (config 2 shape)
        for (int rep = 0; rep < 2; rep++) {
            row2<2, false, 64, 1, true>(P, s, "sum2 2R1W");
            row2<2, false, 128, 1, true>(P, s, "sum2 2R1W");
            row2<2, false, 256, 1, true>(P, s, "sum2 2R1W");
            row2<4, false, 64, 1, true>(P, s, "sum4 4R1W");
            row2<4, false, 128, 1, true>(P, s, "sum4 4R1W");
            row2<4, false, 256, 1, true>(P, s, "sum4 4R1W");
            row2<4, false, 512, 1, true>(P, s, "sum4 4R1W");
            row2<8, false, 64, 1, true>(P, s, "sum8 8R1W");
            row2<8, false, 128, 1, true>(P, s, "sum8 8R1W");
            row2<8, false, 256, 1, true>(P, s, "sum8 8R1W");
            row2<8, false, 512, 1, true>(P, s, "sum8 8R1W");
            row2<8, false, 256, 2, true>(P, s, "sum8 8R1W");
        }
    } else if (mode[0] == 'a') {
        sweep<1, false>(P, cus, s, "copy 1R1W");
        sweep<1, true>(P, cus, s, "copy+zero 1R2W");
        sweep<2, false>(P, cus, s, "sum2 2R1W");
        sweep<4, false>(P, cus, s, "sum4 4R1W");
        sweep<8, false>(P, cus, s, "sum8 8R1W");
    } else {
        sweep2<1, false>(P, s, "copy 1R1W");
        sweep2<1, true>(P, s, "copy+zero 1R2W");
        sweep2<2, false>(P, s, "sum2 2R1W");
        sweep2<4, false>(P, s, "sum4 4R1W");
        sweep2<8, false>(P, s, "sum8 8R1W");
    }
    return 0;
}
