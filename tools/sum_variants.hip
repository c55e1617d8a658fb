// sum_variants.hip — measurement tool (not part of the product): round-3
// variants of the config-2 kernel, out = (in_0 + ... + in_{k-1}) * 0.5 over a
// 64 MiB f32 bucket (sum_scale_f32, kR1W), k = 2, 4, 8, timed like bench.py
// and tools/kernel_variants.hip: one HIP event pair around L back-to-back
// launches rotating over buffer sets > 1.5 GiB (no Infinity-Cache re-reads).
// Round 2 measured workgroup size, vectors per lane, XCD-contiguous block
// order, operand skew, cache policies and a persistent grid (all no better);
// the axes here are the ones it left:
//   P     the product (64-thread workgroups, one 16-B vector per lane and
//         input, nt loads, nt stores)
//   BUF   raw buffer loads: one SGPR resource per input, one VGPR offset for
//         all k (no 64-bit address arithmetic per input), nt
//   GLDS  LDS-DMA: every input's 1 KiB per wave lands in LDS
//         (global_load_lds_dwordx4 nt), one wait, then ds_read_b128 + adds
//   ROT   the k loads of a wave issued starting at input (wave mod k)
//   PRIO  s_setprio 3 around the load burst
//   REV   blocks in reverse address order
//   B128  128-thread workgroups (2 waves)
//   EMPTY the same grid doing nothing but its guard (the launch + drain floor)
//   SER<D> at most D of a wave's K loads in flight (the rotation variants
//         below turned out to serialize their loads through one register set)
//   PSEL  the product's first rotation form (per-wave pointer order)
//   ROTX / ROT3 / HALF / GLDSROT / ROT256  other rotations of the load order
//         (by position within the XCD, by 3 x wave, half the waves by k/2;
//         with LDS-DMA; 256-thread workgroups)
//
//   LIB   the product's ono_sum_scale_f32 (libono_reduce.so) on the same buffers
//
//   hipcc --offload-arch=gfx950 -O3 -I../include -o sum_variants sum_variants.hip \
//         -L../oxidized-neural-orchestra_amd/ono_amd -lono_reduce -Wl,-rpath,...
//   ./sum_variants [MiB=64] [passes=3]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ono_reduce.h"  // LIB: the product's ono_sum_scale_f32 on the same buffers

typedef float f4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e = (x);                                                                       \
        if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
    } while (0)

static size_t N = 16u << 20;
constexpr int L = 40, W = 3;

struct Args {
    const f4 *in[8];
    f4 *out;
    size_t nvec;
};

template <class T> __device__ __forceinline__ T ldn(const T *p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void stn(f4 *p, f4 v) { __builtin_nontemporal_store(v, p); }

enum { P = 0, ROT = 1, PRIO = 2, REV = 3, EMPTY = 4, ROTX = 5, ROT3 = 6, HALF = 7, ROTU = 8 };

// the input a wave loads j-th (ROT family): rotation r of the input order
template <int K, int MODE> __device__ __forceinline__ int rot_of(size_t wave, size_t blk) {
    if constexpr (MODE == ROT) return (int)(wave % K);
    else if constexpr (MODE == ROTX) return (int)((blk / 8) % K);  // by position within the block's XCD
    else if constexpr (MODE == ROT3) return (int)((wave * 3) % K);
    else if constexpr (MODE == HALF) return (int)((wave & 1) * (K / 2));
    else return 0;
}

template <int K, int B, int MODE>
__global__ __launch_bounds__(B) void k_sum(Args a) {
    size_t blk = blockIdx.x;
    if (MODE == REV) blk = gridDim.x - 1 - blk;
    const size_t v = blk * B + threadIdx.x;
    if (v >= a.nvec) return;
    if constexpr (MODE == EMPTY) return;
    f4 x[K];
    if constexpr (MODE == PRIO) __builtin_amdgcn_s_setprio(3);
    if constexpr (MODE == ROT || MODE == ROTX || MODE == ROT3 || MODE == HALF) {
        const int r = rot_of<K, MODE>(blk * (B / 64) + threadIdx.x / 64, blk);
#pragma unroll
        for (int j = 0; j < K; j++) {
            const int q = (j + r) % K;
            x[q] = ldn(a.in[q] + v);  // runtime index: the compiler keeps x in registers via selects
        }
    } else {
#pragma unroll
        for (int j = 0; j < K; j++) x[j] = ldn(a.in[j] + v);
    }
    if constexpr (MODE == PRIO) __builtin_amdgcn_s_setprio(0);
    f4 s = x[0];
#pragma unroll
    for (int j = 1; j < K; j++) s += x[j];
    stn(a.out + v, s * 0.5f);
}

// at most D of a wave's K loads in flight: each load issued once the one D
// places before it has returned (in input order, the fold as usual)
template <int D> __device__ __forceinline__ void wait_vm() {
    if constexpr (D == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (D == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else if constexpr (D == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else if constexpr (D == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
}
template <int K, int D>
__global__ __launch_bounds__(64) void k_sum_ser(Args a) {
    const size_t v = (size_t)blockIdx.x * 64 + threadIdx.x;
    if (v >= a.nvec) return;
    f4 x[K];
#pragma unroll
    for (int j = 0; j < K; j++) {
        if (j >= D) wait_vm<D - 1>();
        x[j] = ldn(a.in[j] + v);
    }
    f4 s = x[0];
#pragma unroll
    for (int j = 1; j < K; j++) s += x[j];
    stn(a.out + v, s * 0.5f);
}

// one input in flight per wave, B threads per workgroup, U vectors per lane
// (one wave apart: every instruction 1 KiB contiguous, the U loads of one
// input in flight together)
template <int K, int B, int U>
__global__ __launch_bounds__(B) void k_sum_seru(Args a) {
    const size_t base = ((size_t)blockIdx.x * (B / 64) + threadIdx.x / 64) * 64 * U + (threadIdx.x % 64);
    f4 acc[U];
#pragma unroll
    for (int j = 0; j < K; j++) {
        f4 x[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const size_t v = base + 64 * u;
            x[u] = v < a.nvec ? ldn(a.in[j] + v) : f4{0, 0, 0, 0};
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int u = 0; u < U; u++) acc[u] = j == 0 ? x[u] : acc[u] + x[u];
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t v = base + 64 * u;
        if (v < a.nvec) stn(a.out + v, acc[u] * 0.5f);
    }
}

// the product's form (round 3): pointer j of an odd wave is input (j + K/2) % K,
// loads in fixed instruction order, the fold in input order by a uniform branch
template <int K>
__global__ __launch_bounds__(64) void k_sum_psel(Args a) {
    const size_t v = (size_t)blockIdx.x * 64 + threadIdx.x;
    if (v >= a.nvec) return;
    constexpr int h = K / 2;
    const bool odd = blockIdx.x & 1;
    f4 y[K];
#pragma unroll
    for (int j = 0; j < K; j++) y[j] = ldn((odd ? a.in[(j + h) % K] : a.in[j]) + v);
    f4 s;
    if (odd) {
        s = y[K - h];
#pragma unroll
        for (int q = 1; q < K; q++) s += y[(q + K - h) % K];
    } else {
        s = y[0];
#pragma unroll
        for (int q = 1; q < K; q++) s += y[q];
    }
    stn(a.out + v, s * 0.5f);
}

// LDS-DMA with the rotated order
template <int K>
__global__ __launch_bounds__(64) void k_sum_glds_rot(Args a) {
    __shared__ f4 lds[K][64];
    const size_t v = (size_t)blockIdx.x * 64 + threadIdx.x;
    const size_t vv = v < a.nvec ? v : a.nvec - 1;
    const int r = (int)(blockIdx.x % K);
#pragma unroll
    for (int j = 0; j < K; j++) {
        const int q = (j + r) % K;
        __builtin_amdgcn_global_load_lds((const void *)(a.in[q] + vv), (__attribute__((address_space(3))) void *)&lds[q][0],
                                         16, 0, 2);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    f4 s = lds[0][threadIdx.x];
#pragma unroll
    for (int j = 1; j < K; j++) s += lds[j][threadIdx.x];
    if (v < a.nvec) stn(a.out + v, s * 0.5f);
}

// raw buffer loads: resource per input (num_records = the bucket's bytes)
template <int K>
__global__ __launch_bounds__(64) void k_sum_buf(Args a) {
    const size_t v = (size_t)blockIdx.x * 64 + threadIdx.x;
    if (v >= a.nvec) return;
    const unsigned off = (unsigned)(v * 16);
    f4 x[K];
#pragma unroll
    for (int j = 0; j < K; j++) {
        __amdgpu_buffer_rsrc_t r =
            __builtin_amdgcn_make_buffer_rsrc((void *)a.in[j], (short)0, (int)(a.nvec * 16 > 0x7FFFFFFF ? 0x7FFFFFFF : a.nvec * 16), 0x00020000);
        x[j] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 2));
    }
    f4 s = x[0];
#pragma unroll
    for (int j = 1; j < K; j++) s += x[j];
    stn(a.out + v, s * 0.5f);
}

// LDS-DMA: input j's 1 KiB of this wave -> lds[j], one wait, LDS reads
template <int K>
__global__ __launch_bounds__(64) void k_sum_glds(Args a) {
    __shared__ f4 lds[K][64];
    const size_t v = (size_t)blockIdx.x * 64 + threadIdx.x;
    const size_t vv = v < a.nvec ? v : a.nvec - 1;
#pragma unroll
    for (int j = 0; j < K; j++)
        __builtin_amdgcn_global_load_lds((const void *)(a.in[j] + vv), (__attribute__((address_space(3))) void *)&lds[j][0],
                                         16, 0, 2);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    f4 s = lds[0][threadIdx.x];
#pragma unroll
    for (int j = 1; j < K; j++) s += lds[j][threadIdx.x];
    if (v < a.nvec) stn(a.out + v, s * 0.5f);
}

// LDS-DMA, U vectors per lane (one wave apart)
template <int K, int U>
__global__ __launch_bounds__(64) void k_sum_glds_u(Args a) {
    __shared__ f4 lds[U][K][64];
    const size_t base = (size_t)blockIdx.x * 64 * U + threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t v = base + 64 * u, vv = v < a.nvec ? v : a.nvec - 1;
#pragma unroll
        for (int j = 0; j < K; j++)
            __builtin_amdgcn_global_load_lds((const void *)(a.in[j] + vv),
                                             (__attribute__((address_space(3))) void *)&lds[u][j][0], 16, 0, 2);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t v = base + 64 * u;
        f4 s = lds[u][0][threadIdx.x];
#pragma unroll
        for (int j = 1; j < K; j++) s += lds[u][j][threadIdx.x];
        if (v < a.nvec) stn(a.out + v, s * 0.5f);
    }
}

__global__ void k_fill(f4 *p, size_t n, unsigned seed) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned h = (unsigned)i * 2654435761u ^ seed;
        p[i] = f4{(float)(h & 1023), (float)((h >> 10) & 1023), 1.0f, -2.0f};
    }
}

static std::vector<f4 *> g_bufs;
static bool g_synth = false;  // argv[3] == "synth": the bench's data (ono_synth_f32, SURVEY §8(d) distribution)
static f4 *buf(int i, hipStream_t s) {
    while ((int)g_bufs.size() <= i) {
        f4 *p;
        CK(hipMalloc(&p, N * sizeof(float)));
        if (g_synth) {
            if (ono_synth_f32((float *)p, N, 0x0402026 + g_bufs.size(), g_bufs.size() % 9, 0, s) != 0) exit(1);
        } else {
            hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, s, p, N / 4, 17u + (unsigned)g_bufs.size());
        }
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
    const char *name;
    int k;
    std::vector<double> us;
};
static std::vector<Row> g_rows;
static Row &row(const char *name, int k) {
    for (auto &r : g_rows)
        if (r.k == k && !strcmp(r.name, name)) return r;
    g_rows.push_back({name, k, {}});
    return g_rows.back();
}

template <int K, class Launch>
static void variant(const char *name, hipStream_t s, Launch launch) {
    const int nsets = 1536 / ((K + 1) * (int)(N >> 18)) + 2;
    const double us = timeit(nsets, s, [&](int set) {
        Args a{};
        for (int j = 0; j < K; j++) a.in[j] = buf(set * (K + 1) + j, s);
        a.out = buf(set * (K + 1) + K, s);
        a.nvec = N / 4;
        launch(a);
    });
    row(name, K).us.push_back(us);
}

template <int K>
static void sweep(hipStream_t s) {
    const unsigned g64 = (unsigned)((N / 4 + 63) / 64), g128 = (unsigned)((N / 4 + 127) / 128);
    variant<K>("P", s, [&](Args a) { hipLaunchKernelGGL((k_sum<K, 64, P>), dim3(g64), dim3(64), 0, s, a); });
    variant<K>("GLDS", s, [&](Args a) { hipLaunchKernelGGL((k_sum_glds<K>), dim3(g64), dim3(64), 0, s, a); });
    variant<K>("EMPTY", s, [&](Args a) { hipLaunchKernelGGL((k_sum<K, 64, EMPTY>), dim3(g64), dim3(64), 0, s, a); });
    variant<K>("SER1", s, [&](Args a) { hipLaunchKernelGGL((k_sum_ser<K, 1>), dim3(g64), dim3(64), 0, s, a); });
    variant<K>("LIB", s, [&](Args a) {
        const float *ins[8];
        for (int j = 0; j < K; j++) ins[j] = (const float *)a.in[j];
        if (ono_sum_scale_f32((float *)a.out, ins, K, N, 2.0f, s) != 0) { fprintf(stderr, "%s\n", ono_last_error()); exit(1); }
    });
    // occupancy limited by dynamic LDS per one-wave workgroup: at most N per CU
    auto lds_for = [](int n) { return (unsigned)(160 * 1024 * 2 / (2 * n + 1)); };
    static char names[256][24];
    static int nn = 0;
    auto name = [&](const char *f, int occ) { char *nm = names[nn++ % 256]; snprintf(nm, 24, f, occ); return (const char *)nm; };
    for (int occ : {20, 24, 28}) {
        const unsigned l = lds_for(occ);
        variant<K>(name("SER1_occ%d", occ), s, [&](Args a) { hipLaunchKernelGGL((k_sum_ser<K, 1>), dim3(g64), dim3(64), l, s, a); });
        variant<K>(name("GLDS_occ%d", occ), s, [&](Args a) { hipLaunchKernelGGL((k_sum_glds<K>), dim3(g64), dim3(64), l, s, a); });
    }
    // U vectors per lane, serialized by input (round 3, session 2): fewer waves, more bytes per load burst
    const unsigned g64u2 = (unsigned)((N / 4 + 127) / 128), g64u4 = (unsigned)((N / 4 + 255) / 256);
    for (int occ : {0, 16, 24}) {
        const unsigned l = occ ? lds_for(occ) : 0u;
        variant<K>(name("SERU2_occ%d", occ), s, [&](Args a) { hipLaunchKernelGGL((k_sum_seru<K, 64, 2>), dim3(g64u2), dim3(64), l, s, a); });
        variant<K>(name("SERU4_occ%d", occ), s, [&](Args a) { hipLaunchKernelGGL((k_sum_seru<K, 64, 4>), dim3(g64u4), dim3(64), l, s, a); });
    }
}

int main(int argc, char **argv) {
    if (argc > 1) N = (size_t)atol(argv[1]) << 18;
    const int passes = argc > 2 ? atoi(argv[2]) : 3;
    g_synth = argc > 3 && !strcmp(argv[3], "synth");
    hipStream_t s = nullptr;  // argv[4] == "null": the legacy default stream
    if (!(argc > 4 && !strcmp(argv[4], "null"))) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    printf("# %s, %d CUs, %zu elements (%zu MiB) per buffer, %d passes, median us per launch\n", p.gcnArchName,
           p.multiProcessorCount, N, N >> 18, passes);
    fflush(stdout);
    for (int pass = 0; pass < passes; pass++) {
        sweep<2>(s);
        sweep<4>(s);
        sweep<8>(s);
        fprintf(stderr, "pass %d done\n", pass);
    }
    for (auto &r : g_rows) {
        std::sort(r.us.begin(), r.us.end());
        const double us = r.us[r.us.size() / 2];
        const double bytes = (double)(r.k + 1) * 4 * N;
        printf("k=%d %-6s %8.2f us  %7.1f GB/s  %.3f of 8 TB/s   (min %.2f max %.2f)\n", r.k, r.name, us,
               bytes / us / 1e3, bytes / us / 1e3 / 8000.0, r.us.front(), r.us.back());
    }
    for (f4 *q : g_bufs) CK(hipFree(q));
    return 0;
}
