// kernel_variants.hip — measurement tool (not part of the product): shapes of
// the reduction path's HBM streams that round 1 left below 80 % of the 8 TB/s
// roofline, at the bench's 64 MiB size, timed like bench.py (one HIP event pair
// around L back-to-back launches rotating over buffer sets > 1.5 GiB, so the
// Infinity Cache cannot serve re-reads).
//
//   sum<K>   out = (in0 + ... + inK-1) * 0.5            (sum_scale_f32, kR1W)
//   dec      out = f32(in_f16) * 0.125                  (f16_decode_scale, 2 B in / 4 B out)
//   acc      acc = acc + in                             (acc_residual, 2R1W)
//
// Variant axes: workgroup size B, vectors per lane U (each one wave apart, so
// every instruction stays a contiguous 1 KiB; all loads issued before any
// store), XCD-contiguous block mapping (X: workgroup b runs on XCD b % 8, so
// logical block = (b % 8) * (G / 8) + b / 8 gives each XCD a contiguous eighth
// of the buffer), and for dec an LDS transpose: 16-B f16 loads (8 halves per
// lane, 1 KiB per wave-instruction) staged through the wave's own 1 KiB of LDS
// and read back as 8-B slices so each f32 store instruction covers 1 KiB.
//
//   hipcc --offload-arch=gfx950 -O3 -o kernel_variants kernel_variants.hip
//   ./kernel_variants [sum|dec|acc|all]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef uint16_t h4 __attribute__((ext_vector_type(4)));
typedef uint16_t h8 __attribute__((ext_vector_type(8)));

#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e = (x);                                                                       \
        if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
    } while (0)

static size_t N = 16u << 20;  // elements per buffer (default 64 MiB f32; argv[2] = MiB)
constexpr int L = 40;            // timed launches
constexpr int W = 3;             // warmup launches

template <class T> __device__ __forceinline__ T ldn(const T *p) { return __builtin_nontemporal_load(p); }
template <class T> __device__ __forceinline__ void stn(T *p, T v) { __builtin_nontemporal_store(v, p); }

__device__ __forceinline__ size_t logical_block(bool xcd) {
    if (!xcd) return blockIdx.x;
    const size_t G = gridDim.x, b = blockIdx.x;  // G is a multiple of 8 (host pads)
    return (b % 8) * (G / 8) + b / 8;
}

struct SumArgs {
    const f4 *in[8];
    f4 *out;
};
// vector index of lane `l`, unroll u: wave-contiguous 1 KiB per instruction
template <int B, int U>
__device__ __forceinline__ size_t vidx(size_t lb, int u) {
    const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
    return ((lb * (B / 64) + wave) * U + u) * 64 + lane;
}

template <int K, int B, int U, bool X>
__global__ __launch_bounds__(B) void k_sum(SumArgs a, size_t nvec) {
    const size_t lb = logical_block(X);
    f4 r[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t v = vidx<B, U>(lb, u);
        if (v < nvec) {
            r[u] = ldn(a.in[0] + v);
#pragma unroll
            for (int j = 1; j < K; j++) r[u] += ldn(a.in[j] + v);
        }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t v = vidx<B, U>(lb, u);
        if (v < nvec) stn(a.out + v, r[u] * 0.5f);
    }
}

__device__ __forceinline__ float dec1(uint16_t b) { return (float)__builtin_bit_cast(_Float16, b); }
__device__ __forceinline__ f4 dec4(h4 h) { return f4{dec1(h.x), dec1(h.y), dec1(h.z), dec1(h.w)}; }

// current product shape: 8-B f16 loads (4 halves per lane), one f4 store
template <int B, int U, bool X>
__global__ __launch_bounds__(B) void k_dec(const h4 *in, f4 *out, size_t nvec) {
    const size_t lb = logical_block(X);
    h4 h[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t v = vidx<B, U>(lb, u);
        if (v < nvec) h[u] = ldn(in + v);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t v = vidx<B, U>(lb, u);
        if (v < nvec) stn(out + v, dec4(h[u]) * 0.125f);
    }
}

// LDS transpose: lane l loads halves [8l, 8l+8) of the wave's 512 (one 16-B
// load, 1 KiB per instruction), writes them to the wave's LDS row, reads back
// halves [4l, 4l+4) and [256+4l, 256+4l+4) and stores them as two 1-KiB f32
// instructions.  U 16-B loads per lane (2 KiB of f16 per wave per u).
template <int B, int U, bool X>
__global__ __launch_bounds__(B) void k_dec_lds(const h8 *in, f4 *out, size_t n8) {
    __shared__ h4 lds[B / 64][U][128];
    const size_t lb = logical_block(X);
    const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
    h8 h[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t v = vidx<B, U>(lb, u);
        if (v < n8) h[u] = ldn(in + v);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        lds[wave][u][2 * lane] = h4{h[u][0], h[u][1], h[u][2], h[u][3]};
        lds[wave][u][2 * lane + 1] = h4{h[u][4], h[u][5], h[u][6], h[u][7]};
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t v = vidx<B, U>(lb, u);  // this lane's 16-B f16 vector = two f4 outputs
        const size_t wave_base = (v - lane) * 2;   // first f4 of the wave's 128
        h4 a = lds[wave][u][lane], b = lds[wave][u][64 + lane];
        if (wave_base + lane < 2 * n8) stn(out + wave_base + lane, dec4(a) * 0.125f);
        if (wave_base + 64 + lane < 2 * n8) stn(out + wave_base + 64 + lane, dec4(b) * 0.125f);
    }
}

// acc += in
template <int B, int U, bool X, bool NTACC>
__global__ __launch_bounds__(B) void k_acc(f4 *acc, const f4 *in, size_t nvec) {
    const size_t lb = logical_block(X);
    f4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t v = vidx<B, U>(lb, u);
        if (v < nvec) {
            a[u] = NTACC ? ldn(acc + v) : acc[v];
            b[u] = ldn(in + v);
        }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t v = vidx<B, U>(lb, u);
        if (v < nvec) stn(acc + v, a[u] + b[u]);
    }
}


// ---- diagnostics: read-only / write-only ceilings, store policy, persistent pipelined grid
template <int K>
__global__ __launch_bounds__(64) void k_read(SumArgs a, size_t nvec) {
    const size_t v = (size_t)blockIdx.x * 64 + threadIdx.x;
    f4 r = ldn(a.in[0] + v);
#pragma unroll
    for (int j = 1; j < K; j++) r += ldn(a.in[j] + v);
    if (r.x == 1234.5f && r.y == -1.0f) a.out[v] = r;  // never true for the fill data: keeps the loads
}
__global__ __launch_bounds__(64) void k_write(f4 *out, size_t nvec) {
    const size_t v = (size_t)blockIdx.x * 64 + threadIdx.x;
    stn(out + v, f4{0.0f, 1.0f, 2.0f, 3.0f});
}
__device__ __forceinline__ void st_sc1(f4 *p, f4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" : : "v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st_sc01(f4 *p, f4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt\n\ts_nop 1" : : "v"(p), "v"(v) : "memory");
}
// store policy P: 0 nt, 1 nt sc1, 2 sc0 sc1 nt
template <int K, int P>
__global__ __launch_bounds__(64) void k_sum_pol(SumArgs a, size_t nvec) {
    const size_t v = (size_t)blockIdx.x * 64 + threadIdx.x;
    f4 r = ldn(a.in[0] + v);
#pragma unroll
    for (int j = 1; j < K; j++) r += ldn(a.in[j] + v);
    r *= 0.5f;
    if constexpr (P == 0) stn(a.out + v, r);
    else if constexpr (P == 1) st_sc1(a.out + v, r);
    else st_sc01(a.out + v, r);
}
template <int P>
__global__ __launch_bounds__(64) void k_dec_pol(const h4 *in, f4 *out, size_t nvec) {
    const size_t v = (size_t)blockIdx.x * 64 + threadIdx.x;
    f4 r = dec4(ldn(in + v)) * 0.125f;
    if constexpr (P == 0) stn(out + v, r);
    else if constexpr (P == 1) st_sc1(out + v, r);
    else st_sc01(out + v, r);
}
// persistent grid, software pipelined: the loads of iteration i+1 are issued
// before the store of iteration i (B-thread workgroups, G = CUs x WPC)
template <int K, int B>
__global__ __launch_bounds__(B) void k_sum_pipe(SumArgs a, size_t nvec) {
    const size_t stride = (size_t)gridDim.x * B;
    size_t v = (size_t)blockIdx.x * B + threadIdx.x;
    if (v >= nvec) return;
    f4 r = ldn(a.in[0] + v);
#pragma unroll
    for (int j = 1; j < K; j++) r += ldn(a.in[j] + v);
    for (;;) {
        const size_t vn = v + stride;
        f4 q = {0, 0, 0, 0};
        if (vn < nvec) {
            q = ldn(a.in[0] + vn);
#pragma unroll
            for (int j = 1; j < K; j++) q += ldn(a.in[j] + vn);
        }
        stn(a.out + v, r * 0.5f);
        if (vn >= nvec) break;
        v = vn;
        r = q;
    }
}

__global__ void k_fill(f4 *p, size_t nvec, unsigned seed) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (size_t)gridDim.x * 256) {
        unsigned h = (unsigned)i * 2654435761u ^ seed;
        p[i] = f4{(float)(h & 0xFFFF), (float)(h >> 16), (float)(h & 0xFF), 1.0f} * 1e-4f;
    }
}

static unsigned blocks_for(size_t work_vecs, int B, int U, bool X) {
    size_t per = (size_t)B * U;
    size_t g = (work_vecs + per - 1) / per;
    if (X) g = (g + 7) / 8 * 8;
    return (unsigned)g;
}

// time L launches over rotating sets; launch(set) enqueues one launch
template <class F>
static void timeit(const char *name, double bytes, int nsets, hipStream_t s, F launch) {
    for (int i = 0; i < W; i++) launch(i % nsets);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < L; i++) launch((W + i) % nsets);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / L, gbs = bytes / (us * 1e-6) / 1e9;
    printf("%-34s %8.2f us %8.1f GB/s  %.3f of 8000\n", name, us, gbs, gbs / 8000.0);
    fflush(stdout);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

static std::vector<f4 *> g_bufs;
static f4 *buf(int i, hipStream_t s) {
    while ((int)g_bufs.size() <= i) {
        f4 *p;
        CK(hipMalloc(&p, N * sizeof(float)));
        hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, s, p, N / 4, 17u + (unsigned)g_bufs.size());
        g_bufs.push_back(p);
    }
    return g_bufs[i];
}

template <int K, int B, int U, bool X>
static void sum_row(hipStream_t s) {
    const int nsets = (1536 / ((K + 1) * 64)) + 2;
    const size_t nvec = N / 4;
    char name[64];
    snprintf(name, sizeof name, "sum k=%d B=%d U=%d X=%d", K, B, U, (int)X);
    const unsigned g = blocks_for(nvec, B, U, X);
    timeit(name, (double)(K + 1) * 4 * N, nsets, s, [&](int set) {
        SumArgs a{};
        for (int j = 0; j < K; j++) a.in[j] = buf(set * (K + 1) + j, s);
        a.out = buf(set * (K + 1) + K, s);
        hipLaunchKernelGGL((k_sum<K, B, U, X>), dim3(g), dim3(B), 0, s, a, nvec);
    });
}

template <int K>
static void sum_sweep(hipStream_t s) {
    sum_row<K, 64, 1, false>(s);  // the product's shape
    sum_row<K, 64, 1, true>(s);
    sum_row<K, 64, 2, false>(s);
    sum_row<K, 64, 2, true>(s);
    sum_row<K, 64, 4, false>(s);
    sum_row<K, 256, 1, false>(s);
    sum_row<K, 256, 1, true>(s);
    sum_row<K, 256, 2, false>(s);
    sum_row<K, 256, 2, true>(s);
    sum_row<K, 256, 4, true>(s);
    sum_row<K, 512, 1, true>(s);
}

template <int B, int U, bool X>
static void dec_row(hipStream_t s) {
    const size_t nvec = N / 4;
    char name[64];
    snprintf(name, sizeof name, "dec h4 B=%d U=%d X=%d", B, U, (int)X);
    const unsigned g = blocks_for(nvec, B, U, X);
    timeit(name, 6.0 * N, 12, s, [&](int set) {
        const h4 *in = (const h4 *)buf(2 * set, s);
        hipLaunchKernelGGL((k_dec<B, U, X>), dim3(g), dim3(B), 0, s, in, buf(2 * set + 1, s), nvec);
    });
}
template <int B, int U, bool X>
static void dec_lds_row(hipStream_t s) {
    const size_t n8 = N / 8;
    char name[64];
    snprintf(name, sizeof name, "dec lds16 B=%d U=%d X=%d", B, U, (int)X);
    const unsigned g = blocks_for(n8, B, U, X);
    timeit(name, 6.0 * N, 12, s, [&](int set) {
        const h8 *in = (const h8 *)buf(2 * set, s);
        hipLaunchKernelGGL((k_dec_lds<B, U, X>), dim3(g), dim3(B), 0, s, in, buf(2 * set + 1, s), n8);
    });
}

template <int B, int U, bool X, bool NTACC>
static void acc_row(hipStream_t s) {
    const size_t nvec = N / 4;
    char name[64];
    snprintf(name, sizeof name, "acc B=%d U=%d X=%d ntacc=%d", B, U, (int)X, (int)NTACC);
    const unsigned g = blocks_for(nvec, B, U, X);
    timeit(name, 12.0 * N, 12, s, [&](int set) {
        hipLaunchKernelGGL((k_acc<B, U, X, NTACC>), dim3(g), dim3(B), 0, s, buf(2 * set, s), buf(2 * set + 1, s),
                           nvec);
    });
}


template <int K>
static void diag_rows(hipStream_t s) {
    const int nsets = (1536 / ((K + 1) * 64)) + 2;
    const size_t nvec = N / 4;
    const unsigned g = (unsigned)(nvec / 64);
    char name[64];
    snprintf(name, sizeof name, "read-only k=%d", K);
    timeit(name, (double)K * 4 * N, nsets, s, [&](int set) {
        SumArgs a{};
        for (int j = 0; j < K; j++) a.in[j] = buf(set * (K + 1) + j, s);
        a.out = buf(set * (K + 1) + K, s);
        hipLaunchKernelGGL((k_read<K>), dim3(g), dim3(64), 0, s, a, nvec);
    });
    for (int P = 0; P < 3; P++) {
        snprintf(name, sizeof name, "sum k=%d st_pol=%d", K, P);
        timeit(name, (double)(K + 1) * 4 * N, nsets, s, [&](int set) {
            SumArgs a{};
            for (int j = 0; j < K; j++) a.in[j] = buf(set * (K + 1) + j, s);
            a.out = buf(set * (K + 1) + K, s);
            if (P == 0) hipLaunchKernelGGL((k_sum_pol<K, 0>), dim3(g), dim3(64), 0, s, a, nvec);
            if (P == 1) hipLaunchKernelGGL((k_sum_pol<K, 1>), dim3(g), dim3(64), 0, s, a, nvec);
            if (P == 2) hipLaunchKernelGGL((k_sum_pol<K, 2>), dim3(g), dim3(64), 0, s, a, nvec);
        });
    }
    for (int wpc : {8, 16, 32}) {
        snprintf(name, sizeof name, "sum k=%d pipe B=256 wgpc=%d", K, wpc / 4);
        timeit(name, (double)(K + 1) * 4 * N, nsets, s, [&](int set) {
            SumArgs a{};
            for (int j = 0; j < K; j++) a.in[j] = buf(set * (K + 1) + j, s);
            a.out = buf(set * (K + 1) + K, s);
            hipLaunchKernelGGL((k_sum_pipe<K, 256>), dim3(256 * wpc / 4), dim3(256), 0, s, a, nvec);
        });
    }
}
static void diag(hipStream_t s) {
    diag_rows<1>(s);
    diag_rows<2>(s);
    diag_rows<8>(s);
    const size_t nvec = N / 4;
    const unsigned g = (unsigned)(nvec / 64);
    timeit("write-only", 4.0 * N, 12, s, [&](int set) {
        hipLaunchKernelGGL(k_write, dim3(g), dim3(64), 0, s, buf(set, s), nvec);
    });
    for (int P = 0; P < 3; P++) {
        char name[64];
        snprintf(name, sizeof name, "dec st_pol=%d", P);
        timeit(name, 6.0 * N, 12, s, [&](int set) {
            const h4 *in = (const h4 *)buf(2 * set, s);
            f4 *o = buf(2 * set + 1, s);
            if (P == 0) hipLaunchKernelGGL(k_dec_pol<0>, dim3(g), dim3(64), 0, s, in, o, nvec);
            if (P == 1) hipLaunchKernelGGL(k_dec_pol<1>, dim3(g), dim3(64), 0, s, in, o, nvec);
            if (P == 2) hipLaunchKernelGGL(k_dec_pol<2>, dim3(g), dim3(64), 0, s, in, o, nvec);
        });
    }
}

// training regime (acc_residual then pull_grads on ONE reused bucket, fresh
// gradients): acc with plain vs nt residual loads, then the product's pull
// shape (nt loads, nt sc1 stores of grad and the zeroed residual)
__global__ __launch_bounds__(64) void k_pull(f4 *grad, f4 *res, size_t nvec) {
    const size_t v = (size_t)blockIdx.x * 64 + threadIdx.x;
    f4 x = ldn(res + v);
    st_sc1(grad + v, x);
    st_sc1(res + v, f4{0, 0, 0, 0});
}
template <bool NTACC>
static void train_row(hipStream_t s, int accs_per_pull) {
    const size_t nvec = N / 4;
    const unsigned g = (unsigned)(nvec / 64);
    f4 *res = buf(0, s), *grad = buf(1, s);
    char name[64];
    snprintf(name, sizeof name, "train acc x%d + pull ntacc=%d", accs_per_pull, (int)NTACC);
    timeit(name, (12.0 * accs_per_pull + 12.0) * N, 10, s, [&](int set) {
        for (int a = 0; a < accs_per_pull; a++)
            hipLaunchKernelGGL((k_acc<64, 1, false, NTACC>), dim3(g), dim3(64), 0, s, res, buf(2 + (set * accs_per_pull + a) % 10, s), nvec);
        hipLaunchKernelGGL(k_pull, dim3(g), dim3(64), 0, s, grad, res, nvec);
    });
}

int main(int argc, char **argv) {
    const char *mode = argc > 1 ? argv[1] : "all";
    if (argc > 2) N = (size_t)atol(argv[2]) << 18;
    const int passes = argc > 3 ? atoi(argv[3]) : 1;
    const bool all = !strcmp(mode, "all");
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    printf("# %s, %d CUs, %zu elements per buffer\n", p.gcnArchName, p.multiProcessorCount, N);
    sum_row<2, 64, 1, false>(s);  // warm the clocks
    for (int pass = 0; pass < passes; pass++) {
    printf("# pass %d\n", pass);
    if (!strcmp(mode, "diag")) diag(s);
    if (!strcmp(mode, "train")) {
        for (int a : {1, 4}) { train_row<false>(s, a); train_row<true>(s, a); }
    }
    if (all || !strcmp(mode, "dec")) {
        dec_row<64, 1, false>(s);  // the product's shape
        dec_row<64, 1, true>(s);
        dec_row<64, 2, false>(s);
        dec_row<64, 4, false>(s);
        dec_row<256, 1, false>(s);
        dec_row<256, 2, true>(s);
        dec_lds_row<64, 1, false>(s);
        dec_lds_row<64, 1, true>(s);
        dec_lds_row<64, 2, false>(s);
        dec_lds_row<256, 1, false>(s);
        dec_lds_row<256, 1, true>(s);
        dec_lds_row<256, 2, false>(s);
        dec_lds_row<512, 1, true>(s);
    }
    if (all || !strcmp(mode, "acc")) {
        acc_row<64, 1, false, false>(s);  // the product's shape
        acc_row<64, 1, false, true>(s);
        acc_row<64, 1, true, false>(s);
        acc_row<64, 2, false, false>(s);
        acc_row<64, 2, false, true>(s);
        acc_row<256, 1, false, false>(s);
        acc_row<256, 1, true, true>(s);
        acc_row<256, 2, false, true>(s);
        acc_row<256, 2, true, true>(s);
        acc_row<512, 1, true, true>(s);
    }
    if (all || !strcmp(mode, "sum")) {
        sum_sweep<2>(s);
        sum_sweep<4>(s);
        sum_sweep<8>(s);
    }
    }
    for (f4 *q : g_bufs) CK(hipFree(q));
    return 0;
}
