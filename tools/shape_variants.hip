// shape_variants.hip — measurement tool (not part of the product): do the two
// levers found for sum_scale in round 3 (one load in flight per wave; a cap on
// one-wave workgroups per CU through unused dynamic LDS) carry over to the
// path's other HBM streams?  Generic shapes at 64 MiB (16 M f32 elements per
// stream), timed like tools/sum_variants.hip (event span over L launches
// rotating over > 1.5 GiB):
//   R reads, W writes per element, 16-B vectors, one per lane, nt loads and
//   nt stores (the product's policies for these ops):
//     1R2W   pull_grads finaliser (scale_zero: grad = res / n; res = 0)
//     2R3W   all-reduce consumer, GD (g, w -> w, g = 0, copy of w)
//     3R4W   consumer, momentum (g, w, v -> v, w, g, copy)
//     4R5W   consumer, Adam (g, w, v, s -> v, s, g, w, copy)
//     8R3W   owner chain at n = 8 (8 slices -> grad, message, own slice = 0)
//   and the f16 gather decode (1 x 8 B read -> 16 B written per lane).
// Variant letters: P (all loads in flight), S (one load in flight), and an
// occupancy cap "_oN" (at most N one-wave workgroups per CU).
//
//   hipcc --offload-arch=gfx950 -O3 -o shape_variants shape_variants.hip
//   ./shape_variants [passes=3]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef uint16_t h4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e = (x);                                                                       \
        if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
    } while (0)

static const size_t N = 16u << 20;
constexpr int L = 30, W = 3;

struct Args {
    f4 *b[16];
    size_t nvec;
};

template <class T> __device__ __forceinline__ T ldn(const T *p) { return __builtin_nontemporal_load(p); }
template <class T> __device__ __forceinline__ void stn(T *p, T v) { __builtin_nontemporal_store(v, p); }

// reads b[0..R), writes b[R..R+W); every output = a different mix of inputs
template <int R, int Wn, bool SER>
__global__ __launch_bounds__(64) void k_shape(Args a) {
    const size_t v = (size_t)blockIdx.x * 64 + threadIdx.x;
    if (v >= a.nvec) return;
    f4 x[R];
#pragma unroll
    for (int j = 0; j < R; j++) {
        x[j] = ldn(a.b[j] + v);
        if constexpr (SER) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    f4 s = x[0];
#pragma unroll
    for (int j = 1; j < R; j++) s = s * 0.5f + x[j];
#pragma unroll
    for (int w = 0; w < Wn; w++) stn(a.b[R + w] + v, s + (float)w);
}

// f16 decode: 8 B in (4 halves) -> 16 B out
__global__ __launch_bounds__(64) void k_dec(Args a) {
    const size_t v = (size_t)blockIdx.x * 64 + threadIdx.x;
    if (v >= a.nvec) return;
    h4 h = ldn((const h4 *)a.b[0] + v);
    f4 x = {(float)__builtin_bit_cast(_Float16, h.x), (float)__builtin_bit_cast(_Float16, h.y),
            (float)__builtin_bit_cast(_Float16, h.z), (float)__builtin_bit_cast(_Float16, h.w)};
    stn(a.b[1] + v, x * 0.125f);
}

// the decode with B threads per workgroup and U vectors per lane (one wave apart: each
// instruction 512 B in, 1 KiB out, contiguous): fewer workgroups for the dispatcher (round 3)
template <int B, int U>
__global__ __launch_bounds__(B) void k_dec_bu(Args a) {
    const size_t base = ((size_t)blockIdx.x * (B / 64) + threadIdx.x / 64) * 64 * U + threadIdx.x % 64;
    h4 h[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t v = base + 64 * u;
        if (v < a.nvec) h[u] = ldn((const h4 *)a.b[0] + v);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t v = base + 64 * u;
        if (v < a.nvec) {
            f4 x = {(float)__builtin_bit_cast(_Float16, h[u].x), (float)__builtin_bit_cast(_Float16, h[u].y),
                    (float)__builtin_bit_cast(_Float16, h[u].z), (float)__builtin_bit_cast(_Float16, h[u].w)};
            stn(a.b[1] + v, x * 0.125f);
        }
    }
}
// the same grid doing nothing but its guard
template <int B, int U>
__global__ __launch_bounds__(B) void k_empty_bu(Args a) {
    const size_t base = ((size_t)blockIdx.x * (B / 64) + threadIdx.x / 64) * 64 * U + threadIdx.x % 64;
    if (base == (size_t)-1) a.b[1][0] = f4{0, 0, 0, 0};
}

__global__ void k_fill(f4 *p, size_t n, unsigned seed) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned h = (unsigned)i * 2654435761u ^ seed;
        p[i] = f4{(float)(h & 1023), (float)((h >> 10) & 1023), 1.0f, -2.0f};
    }
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

template <class F>
static double timeit(int nsets, hipStream_t s, F launch) {
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
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return ms * 1e3 / L;
}

struct Row {
    std::string name;
    double bytes;
    std::vector<double> us;
};
static std::vector<Row> g_rows;
static void record(const std::string &name, double bytes, double us) {
    for (auto &r : g_rows)
        if (r.name == name) { r.us.push_back(us); return; }
    g_rows.push_back({name, bytes, {us}});
}

static unsigned lds_for(int occ) { return occ >= 32 ? 0u : (unsigned)(160 * 1024 * 2 / (2 * occ + 1)); }

static std::vector<int> g_occ_p = {32, 28, 24, 20, 16, 12, 10, 8, 6, 4}, g_occ_s = {32, 24, 20, 16};
template <int R, int Wn>
static void shape(const char *tag, hipStream_t s) {
    const int per = R + Wn, nsets = 1536 / (per * 64) + 2;
    const unsigned g = (unsigned)((N / 4 + 63) / 64);
    for (int occ : {32, 28, 24, 20, 16, 12, 10, 8, 6, 4}) {
        for (int ser = 0; ser < (R > 1 ? 2 : 1); ser++) {
            if (ser && occ < 16) continue;
            const unsigned l = lds_for(occ);
            const double us = timeit(nsets, s, [&](int set) {
                Args a{};
                for (int j = 0; j < per; j++) a.b[j] = buf(set * per + j, s);
                a.nvec = N / 4;
                if (ser) hipLaunchKernelGGL((k_shape<R, Wn, true>), dim3(g), dim3(64), l, s, a);
                else hipLaunchKernelGGL((k_shape<R, Wn, false>), dim3(g), dim3(64), l, s, a);
            });
            char nm[64];
            snprintf(nm, sizeof nm, "%s %s_o%d", tag, ser ? "S" : "P", occ);
            record(nm, (double)per * 4 * N, us);
        }
    }
}

template <int B, int U>
static void dec_bu(hipStream_t s, bool empty) {
    const int nsets = 1536 / (6 * 64 / 4 * 4 / 4) + 2;
    const unsigned g = (unsigned)((N / 4 + 64 * U * (B / 64) - 1) / (64 * U * (B / 64)));
    const double us = timeit(nsets, s, [&](int set) {
        Args a{};
        a.b[0] = buf(set * 2, s);
        a.b[1] = buf(set * 2 + 1, s);
        a.nvec = N / 4;
        if (empty) hipLaunchKernelGGL((k_empty_bu<B, U>), dim3(g), dim3(B), 0, s, a);
        else hipLaunchKernelGGL((k_dec_bu<B, U>), dim3(g), dim3(B), 0, s, a);
    });
    char nm[64];
    snprintf(nm, sizeof nm, "%s B%d U%d", empty ? "empty" : "dec", B, U);
    record(nm, 6.0 * N, us);
}

static void dec(hipStream_t s) {
    const int nsets = 1536 / (6 * 64 / 4 * 4 / 4) + 2;  // 6 B per element
    const unsigned g = (unsigned)((N / 4 + 63) / 64);
    for (int occ : {32, 28}) {
        const unsigned l = lds_for(occ);
        const double us = timeit(nsets, s, [&](int set) {
            Args a{};
            a.b[0] = buf(set * 2, s);
            a.b[1] = buf(set * 2 + 1, s);
            a.nvec = N / 4;
            hipLaunchKernelGGL(k_dec, dim3(g), dim3(64), l, s, a);
        });
        char nm[64];
        snprintf(nm, sizeof nm, "dec P_o%d", occ);
        record(nm, 6.0 * N, us);
    }
}

int main(int argc, char **argv) {
    const int passes = argc > 1 ? atoi(argv[1]) : 3;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    printf("# %s, %d CUs, %zu elements per stream, %d passes, median us per launch\n", p.gcnArchName,
           p.multiProcessorCount, N, passes);
    fflush(stdout);
    for (int pass = 0; pass < passes; pass++) {
        if (!getenv("DEC_BU")) {
            shape<1, 2>("1R2W", s);
            shape<2, 1>("2R1W", s);
            shape<2, 2>("2R2W", s);
            shape<2, 3>("2R3W", s);
            shape<3, 4>("3R4W", s);
            shape<4, 5>("4R5W", s);
            shape<8, 3>("8R3W", s);
        }
        dec(s);
        if (getenv("DEC_BU")) {
            for (bool e : {false, true}) {
                dec_bu<64, 1>(s, e);
                dec_bu<64, 2>(s, e);
                dec_bu<64, 4>(s, e);
                dec_bu<256, 1>(s, e);
                dec_bu<256, 2>(s, e);
                dec_bu<1024, 1>(s, e);
            }
        }
        fprintf(stderr, "pass %d done\n", pass);
    }
    for (auto &r : g_rows) {
        std::sort(r.us.begin(), r.us.end());
        const double us = r.us[r.us.size() / 2];
        printf("%-14s %8.2f us  %7.1f GB/s  %.3f of 8 TB/s\n", r.name.c_str(), us, r.bytes / us / 1e3,
               r.bytes / us / 1e3 / 8000.0);
    }
    for (f4 *q : g_bufs) CK(hipFree(q));
    return 0;
}
