// launch_phases.hip — measurement tool (not part of the product): where the
// fixed cost of one back-to-back streaming launch goes.
//
// Every kernel here is the library's skeleton (64-thread workgroups, one
// 16-B vector per lane per stream, a one-shot grid) in a STAMP build: lane 0
// of every workgroup reads the 100 MHz real-time counter at its first
// instruction and again after its own stores have been acknowledged
// (s_waitcnt vmcnt(0)), and writes {start, end, XCC id, HW id} with one
// vector store into a side buffer.  From the stamps of L back-to-back
// launches over rotating buffer sets (> 1.5 GiB, no Infinity-Cache reuse):
//   span    first workgroup start -> last workgroup end of one launch
//   gap     last end of launch i -> first start of launch i+1 (the boundary)
//   steady  the streaming rate R fitted on the 20-80 % completions, and the
//           span that rate would take: ideal = bytes / R
//   ramp    first start -> where the fitted line leaves zero completions
//   drain   where the fitted line reaches all completions -> last end
//   xcd     max - min over the 8 XCDs of their last end (drain imbalance)
// span = ramp + ideal + drain; per launch (events) = span + gap.
//
// The same shapes also run un-stamped (HIP events only, what bench.py times)
// and through the product library (LIB: ono_sum_scale_f32, ono_scale_zero_f32,
// ono_copy_f32, ono_fill_f32, ono_f16_decode_scale on the same buffers).
//
//   ./launch_phases [MiB list, default "64,256"] [launches L = 24]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ono_reduce.h"

typedef float f4 __attribute__((ext_vector_type(4)));
typedef uint16_t h4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e = (x);                                                                       \
        if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
    } while (0)
#define OK(x)                                                                    \
    do {                                                                         \
        if ((x) != 0) { fprintf(stderr, "%s: %s\n", #x, ono_last_error()); exit(1); } \
    } while (0)

struct Stamp {  // 16 B, one per workgroup
    uint32_t t0_lo, t0_hi, dt, ids;  // start (64-bit), end - start, XCC id << 16 | (HW id >> 8 & 0xFFFF)
};

struct Args {
    const f4 *in[8];
    f4 *out[2];
    size_t nvec;
    Stamp *st;
    uint32_t first;  // workgroups that fit the chip at once (CUs x 28)
};

template <class T> __device__ __forceinline__ T ldn(const T *p) { return __builtin_nontemporal_load(p); }
template <class T> __device__ __forceinline__ void stn(T *p, T v) { __builtin_nontemporal_store(v, p); }
__device__ __forceinline__ void st_sc1(f4 *p, f4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" : : "v"(p), "v"(v) : "memory");
}

// store policies for the boundary question: does a kernel that leaves no dirty L2 lines end sooner?
__device__ __forceinline__ void st_sys(f4 *p, f4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" : : "v"(p), "v"(v) : "memory");
}
template <int POL> __device__ __forceinline__ void st_pol(f4 *p, f4 v) {
    if constexpr (POL == 0) stn(p, v);
    else if constexpr (POL == 1) st_sc1(p, v);
    else if constexpr (POL == 2) st_sys(p, v);
    else *p = v;
}

template <bool STAMP> struct Clock {
    uint64_t t0 = 0;
    __device__ __forceinline__ void start() {
        if constexpr (STAMP) t0 = __builtin_amdgcn_s_memrealtime();
    }
    __device__ __forceinline__ void stop(Stamp *st) {
        if constexpr (STAMP) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
            unsigned x, h;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(h));
            if (threadIdx.x == 0) {
                uint4 v = {(unsigned)t0, (unsigned)(t0 >> 32), (unsigned)(t1 - t0), ((x & 0xF) << 16) | ((h >> 8) & 0xFFFF)};
                *(uint4 *)&st[blockIdx.x] = v;
            }
        }
    }
};

enum Shape {
    COPY = 0, COPYZ, FILL, SUM2, SUM4, SUM8, DEC, EMPTY, COPY_SC1, COPY_SYS, SUM2_SC1, SUM2_SYS,
    FILL_SC1, FILL_SYS, FILL_PLAIN, DEC_SC1, DEC_SYS, DEC_PLAIN,
    FILL_U4, FILL_U16, FILL_B256, FILL_GRID, DEC_U2, DEC_U4, DEC_B256, COPY_U2, COPY_B256,
    DEC_B256_SC1, DEC_U2_B256, FILL_U4_B256, COPYZ_OCC24, COPYZ_B256, COPYZ_B256_OCC6, COPYZ_U2_OCC12,
    SUM4_HYB, SUM8_HYB, SUM4_HYB2, SUM8_HYB2, NSHAPES
};
static const char *kName[] = {"copy 1R1W", "copy+zero 1R2W", "fill 0R1W", "sum2 2R1W", "sum4 4R1W", "sum8 8R1W",
                              "f16 decode", "empty", "copy st nt sc1", "copy st sc0sc1", "sum2 st nt sc1",
                              "sum2 st sc0sc1", "fill st nt sc1", "fill st sc0sc1", "fill st plain", "decode st nt sc1",
                              "decode st sc0sc1", "decode st plain", "fill U4/lane", "fill U16/lane",
                              "fill 256-thr wg", "fill grid 4/CU", "decode U2/lane", "decode U4/lane",
                              "decode 256-thr wg", "copy U2/lane", "copy 256-thr wg", "decode 256 nt sc1",
                              "decode U2 256-thr", "fill U4 256-thr", "copy+zero occ24", "copy+zero 256-thr",
                              "copy+zero 256 occ6", "copy+zero U2 occ12", "sum4 parallel head", "sum8 parallel head",
                              "sum4 parallel tail", "sum8 parallel tail"};
static const int kReads[] = {1, 1, 0, 2, 4, 8, 1, 0, 1, 1, 2, 2, 0, 0, 0, 1, 1, 1, 0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 0,
                             1, 1, 1, 1, 4, 8, 4, 8};
static const int kWrites[] = {1, 2, 1, 1, 1, 1, 1, 0, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                              2, 2, 2, 2, 1, 1, 1, 1};
// algorithmic bytes per f32 element
static const double kBytes[] = {8, 12, 4, 12, 20, 36, 6, 0, 8, 8, 12, 12, 4, 4, 4, 6, 6, 6,
                                4, 4, 4, 4, 6, 6, 6, 8, 8, 6, 6, 4, 12, 12, 12, 12, 20, 36, 20, 36};
// workgroups per launch for the shapes that do not use one-wave workgroups of one vector per lane
static size_t grid_of(int shape, size_t nvec, int cus) {
    switch (shape) {
    case FILL_U4: case DEC_U4: return (nvec + 255) / 256;
    case FILL_U16: return (nvec + 1023) / 1024;
    case DEC_U2: case COPY_U2: return (nvec + 127) / 128;
    case FILL_B256: case DEC_B256: case COPY_B256: case DEC_B256_SC1: return (nvec + 255) / 256;
    case DEC_U2_B256: return (nvec + 511) / 512;
    case FILL_U4_B256: return (nvec + 1023) / 1024;
    case COPYZ_B256: case COPYZ_B256_OCC6: return (nvec + 255) / 256;
    case COPYZ_U2_OCC12: return (nvec + 127) / 128;
    case FILL_GRID: return (size_t)cus * 4;
    default: return (nvec + 63) / 64;
    }
}
static int block_of(int shape) {
    return shape == FILL_B256 || shape == DEC_B256 || shape == COPY_B256 || shape == FILL_GRID ||
                   shape == DEC_B256_SC1 || shape == DEC_U2_B256 || shape == FILL_U4_B256 || shape == COPYZ_B256 ||
                   shape == COPYZ_B256_OCC6
               ? 256
               : 64;
}
static_assert(sizeof(kBytes) / sizeof(kBytes[0]) == NSHAPES, "one row per shape");

template <bool STAMP, int POL> __device__ __forceinline__ void copy_body(const Args &a) {
    Clock<STAMP> c;
    c.start();
    const size_t v = (size_t)blockIdx.x * 64 + threadIdx.x;
    if (v < a.nvec) st_pol<POL>(a.out[0] + v, ldn(a.in[0] + v));
    c.stop(a.st);
}
template <bool STAMP> __global__ __launch_bounds__(64) void k_copy(Args a) { copy_body<STAMP, 0>(a); }
template <bool STAMP> __global__ __launch_bounds__(64) void k_copy_sc1(Args a) { copy_body<STAMP, 1>(a); }
template <bool STAMP> __global__ __launch_bounds__(64) void k_copy_sys(Args a) { copy_body<STAMP, 2>(a); }
template <bool STAMP> __global__ __launch_bounds__(64) void k_copyz(Args a) {
    Clock<STAMP> c;
    c.start();
    const size_t v = (size_t)blockIdx.x * 64 + threadIdx.x;
    if (v < a.nvec) {
        const f4 x = ldn(a.in[0] + v);
        st_sc1(a.out[0] + v, x);
        st_sc1(a.out[1] + v, f4{0, 0, 0, 0});
    }
    c.stop(a.st);
}
template <bool STAMP, int POL> __device__ __forceinline__ void fill_body(const Args &a) {
    Clock<STAMP> c;
    c.start();
    const size_t v = (size_t)blockIdx.x * 64 + threadIdx.x;
    if (v < a.nvec) st_pol<POL>(a.out[0] + v, f4{0, 0, 0, 0});
    c.stop(a.st);
}
template <bool STAMP> __global__ __launch_bounds__(64) void k_fill(Args a) { fill_body<STAMP, 0>(a); }
template <bool STAMP> __global__ __launch_bounds__(64) void k_fill_sc1(Args a) { fill_body<STAMP, 1>(a); }
template <bool STAMP> __global__ __launch_bounds__(64) void k_fill_sys(Args a) { fill_body<STAMP, 2>(a); }
template <bool STAMP> __global__ __launch_bounds__(64) void k_fill_plain(Args a) { fill_body<STAMP, 3>(a); }
template <bool STAMP> __global__ __launch_bounds__(64) void k_empty(Args a) {
    Clock<STAMP> c;
    c.start();
    c.stop(a.st);
}
// the product's K = 2 form: both inputs by LDS-DMA, one wait, add from LDS
template <bool STAMP, int POL> __device__ __forceinline__ void sum2_body(const Args &a) {
    Clock<STAMP> c;
    c.start();
    __shared__ f4 lds[2][64];
    const size_t v = (size_t)blockIdx.x * 64 + threadIdx.x;
    if (v < a.nvec) {
#pragma unroll
        for (int j = 0; j < 2; j++)
            __builtin_amdgcn_global_load_lds((const void *)(a.in[j] + v), (__attribute__((address_space(3))) void *)&lds[j][0],
                                             16, 0, 2);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        st_pol<POL>(a.out[0] + v, (lds[0][threadIdx.x] + lds[1][threadIdx.x]) * 0.5f);
    }
    c.stop(a.st);
}
template <bool STAMP> __global__ __launch_bounds__(64) void k_sum2(Args a) { sum2_body<STAMP, 0>(a); }
template <bool STAMP> __global__ __launch_bounds__(64) void k_sum2_sc1(Args a) { sum2_body<STAMP, 1>(a); }
template <bool STAMP> __global__ __launch_bounds__(64) void k_sum2_sys(Args a) { sum2_body<STAMP, 2>(a); }
// the product's K >= 4 form: one load in flight per wave (occupancy capped by the launch);
// HYB = 1: the first CUs x 28 workgroups (they start together at the launch) issue all K loads at
// once instead; HYB = 2: the last CUs x 28 (the tail: each serialized chain of K load latencies ends
// the launch while HBM has little else to serve)
template <int K, bool STAMP, int HYB = 0> __global__ __launch_bounds__(64) void k_sumser(Args a) {
    Clock<STAMP> c;
    c.start();
    const size_t v = (size_t)blockIdx.x * 64 + threadIdx.x;
    if ((HYB == 1 && blockIdx.x < a.first) || (HYB == 2 && blockIdx.x + a.first >= gridDim.x)) {
        if (v < a.nvec) {
            f4 x[K];
#pragma unroll
            for (int j = 0; j < K; j++) x[j] = ldn(a.in[j] + v);
            f4 s = x[0];
#pragma unroll
            for (int j = 1; j < K; j++) s += x[j];
            stn(a.out[0] + v, s * (1.0f / K));
        }
        c.stop(a.st);
        return;
    }
    if (v < a.nvec) {
        f4 s = ldn(a.in[0] + v);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int j = 1; j < K; j++) {
            const f4 x = ldn(a.in[j] + v);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            s += x;
        }
        stn(a.out[0] + v, s * (1.0f / K));
    }
    c.stop(a.st);
}
// gather decode: 8-B f16 load, 16-B f32 store (the f16 input is the first half of in[0])
template <bool STAMP, int POL> __device__ __forceinline__ void dec_body(const Args &a) {
    Clock<STAMP> c;
    c.start();
    const size_t v = (size_t)blockIdx.x * 64 + threadIdx.x;
    if (v < a.nvec) {
        const h4 h = ldn((const h4 *)a.in[0] + v);
        f4 r;
        r.x = (float)__builtin_bit_cast(_Float16, h.x);
        r.y = (float)__builtin_bit_cast(_Float16, h.y);
        r.z = (float)__builtin_bit_cast(_Float16, h.z);
        r.w = (float)__builtin_bit_cast(_Float16, h.w);
        st_pol<POL>(a.out[0] + v, r * 0.5f);
    }
    c.stop(a.st);
}
template <bool STAMP> __global__ __launch_bounds__(64) void k_dec(Args a) { dec_body<STAMP, 0>(a); }
template <bool STAMP> __global__ __launch_bounds__(64) void k_dec_sc1(Args a) { dec_body<STAMP, 1>(a); }
template <bool STAMP> __global__ __launch_bounds__(64) void k_dec_sys(Args a) { dec_body<STAMP, 2>(a); }
template <bool STAMP> __global__ __launch_bounds__(64) void k_dec_plain(Args a) { dec_body<STAMP, 3>(a); }

// U vectors per lane, one wave apart (every store instruction 1 KiB contiguous); fewer workgroups
template <bool STAMP, int U> __global__ __launch_bounds__(64) void k_fill_u(Args a) {
    Clock<STAMP> c;
    c.start();
    const size_t v0 = (size_t)blockIdx.x * 64 * U + threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; u++)
        if (v0 + 64 * u < a.nvec) st_sc1(a.out[0] + v0 + 64 * u, f4{0, 0, 0, 0});
    c.stop(a.st);
}
template <bool STAMP> __global__ __launch_bounds__(256) void k_fill_b256(Args a) {
    Clock<STAMP> c;
    c.start();
    const size_t v = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (v < a.nvec) st_sc1(a.out[0] + v, f4{0, 0, 0, 0});
    c.stop(a.st);
}
// the runtime fill's shape: a few 256-thread workgroups per CU, grid-stride
template <bool STAMP> __global__ __launch_bounds__(256) void k_fill_grid(Args a) {
    Clock<STAMP> c;
    c.start();
    for (size_t v = (size_t)blockIdx.x * 256 + threadIdx.x; v < a.nvec; v += (size_t)gridDim.x * 256)
        st_sc1(a.out[0] + v, f4{0, 0, 0, 0});
    c.stop(a.st);
}
__device__ __forceinline__ f4 dec4h(h4 h) {
    f4 r;
    r.x = (float)__builtin_bit_cast(_Float16, h.x);
    r.y = (float)__builtin_bit_cast(_Float16, h.y);
    r.z = (float)__builtin_bit_cast(_Float16, h.z);
    r.w = (float)__builtin_bit_cast(_Float16, h.w);
    return r;
}
template <bool STAMP, int U> __global__ __launch_bounds__(64) void k_dec_u(Args a) {
    Clock<STAMP> c;
    c.start();
    const size_t v0 = (size_t)blockIdx.x * 64 * U + threadIdx.x;
    h4 h[U];
#pragma unroll
    for (int u = 0; u < U; u++) h[u] = v0 + 64 * u < a.nvec ? ldn((const h4 *)a.in[0] + v0 + 64 * u) : h4{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < U; u++)
        if (v0 + 64 * u < a.nvec) stn(a.out[0] + v0 + 64 * u, dec4h(h[u]) * 0.5f);
    c.stop(a.st);
}
template <bool STAMP> __global__ __launch_bounds__(256) void k_dec_b256(Args a) {
    Clock<STAMP> c;
    c.start();
    const size_t v = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (v < a.nvec) stn(a.out[0] + v, dec4h(ldn((const h4 *)a.in[0] + v)) * 0.5f);
    c.stop(a.st);
}
template <bool STAMP> __global__ __launch_bounds__(256) void k_dec_b256_sc1(Args a) {
    Clock<STAMP> c;
    c.start();
    const size_t v = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (v < a.nvec) st_sc1(a.out[0] + v, dec4h(ldn((const h4 *)a.in[0] + v)) * 0.5f);
    c.stop(a.st);
}
// two vectors per lane one 256-lane block apart, 256-thread workgroups
template <bool STAMP> __global__ __launch_bounds__(256) void k_dec_u2_b256(Args a) {
    Clock<STAMP> c;
    c.start();
    const size_t v0 = (size_t)blockIdx.x * 512 + threadIdx.x;
    h4 h[2];
#pragma unroll
    for (int u = 0; u < 2; u++) h[u] = v0 + 256 * u < a.nvec ? ldn((const h4 *)a.in[0] + v0 + 256 * u) : h4{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < 2; u++)
        if (v0 + 256 * u < a.nvec) stn(a.out[0] + v0 + 256 * u, dec4h(h[u]) * 0.5f);
    c.stop(a.st);
}
template <bool STAMP> __global__ __launch_bounds__(256) void k_fill_u4_b256(Args a) {
    Clock<STAMP> c;
    c.start();
    const size_t v0 = (size_t)blockIdx.x * 1024 + threadIdx.x;
#pragma unroll
    for (int u = 0; u < 4; u++)
        if (v0 + 256 * u < a.nvec) st_sc1(a.out[0] + v0 + 256 * u, f4{0, 0, 0, 0});
    c.stop(a.st);
}
template <bool STAMP, int B> __device__ __forceinline__ void copyz_body(const Args &a) {
    Clock<STAMP> c;
    c.start();
    const size_t v = (size_t)blockIdx.x * B + threadIdx.x;
    if (v < a.nvec) {
        const f4 x = ldn(a.in[0] + v);
        st_sc1(a.out[0] + v, x);
        st_sc1(a.out[1] + v, f4{0, 0, 0, 0});
    }
    c.stop(a.st);
}
template <bool STAMP> __global__ __launch_bounds__(256) void k_copyz_b256(Args a) { copyz_body<STAMP, 256>(a); }
template <bool STAMP> __global__ __launch_bounds__(64) void k_copyz_u2(Args a) {
    Clock<STAMP> c;
    c.start();
    const size_t v0 = (size_t)blockIdx.x * 128 + threadIdx.x;
    f4 x[2];
#pragma unroll
    for (int u = 0; u < 2; u++) x[u] = v0 + 64 * u < a.nvec ? ldn(a.in[0] + v0 + 64 * u) : f4{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < 2; u++)
        if (v0 + 64 * u < a.nvec) {
            st_sc1(a.out[0] + v0 + 64 * u, x[u]);
            st_sc1(a.out[1] + v0 + 64 * u, f4{0, 0, 0, 0});
        }
    c.stop(a.st);
}
template <bool STAMP> __global__ __launch_bounds__(64) void k_copy_u2(Args a) {
    Clock<STAMP> c;
    c.start();
    const size_t v0 = (size_t)blockIdx.x * 128 + threadIdx.x;
    f4 x[2];
#pragma unroll
    for (int u = 0; u < 2; u++) x[u] = v0 + 64 * u < a.nvec ? ldn(a.in[0] + v0 + 64 * u) : f4{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < 2; u++)
        if (v0 + 64 * u < a.nvec) st_sc1(a.out[0] + v0 + 64 * u, x[u]);
    c.stop(a.st);
}
template <bool STAMP> __global__ __launch_bounds__(256) void k_copy_b256(Args a) {
    Clock<STAMP> c;
    c.start();
    const size_t v = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (v < a.nvec) st_sc1(a.out[0] + v, ldn(a.in[0] + v));
    c.stop(a.st);
}

__global__ void k_init(f4 *p, size_t n, unsigned seed) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned h = (unsigned)i * 2654435761u ^ seed;
        p[i] = f4{(float)(h & 1023) * 0.25f, (float)((h >> 10) & 1023), 1.0f, -2.0f};
    }
}

static size_t g_max_elems = 64u << 20;  // per pool buffer (256 MiB)
constexpr int kPool = 27;               // 27 x 256 MiB = 6.75 GiB
static std::vector<f4 *> g_pool;
static int L = 24;

static unsigned lds_for_occ(int occ) { return (unsigned)(160 * 1024 * 2 / (2 * occ + 1)); }

// mode: 0 = un-stamped tool kernel, 1 = stamped tool kernel, 2 = LIB
static int g_cus = 256;
static void launch(int shape, int mode, const Args &a, size_t n, hipStream_t s) {
    const unsigned grid = (unsigned)grid_of(shape, a.nvec, g_cus), blk = (unsigned)block_of(shape);
    const bool st = mode == 1;
#define L2(KER) \
    if (st) hipLaunchKernelGGL(KER<true>, dim3(grid), dim3(blk), 0, s, a); \
    else hipLaunchKernelGGL(KER<false>, dim3(grid), dim3(blk), 0, s, a);
#define L2T(KER, P) \
    if (st) hipLaunchKernelGGL((KER<true, P>), dim3(grid), dim3(blk), 0, s, a); \
    else hipLaunchKernelGGL((KER<false, P>), dim3(grid), dim3(blk), 0, s, a);
    if (mode == 2) {
        switch (shape) {
        case COPY: OK(ono_copy_f32((float *)a.out[0], (const float *)a.in[0], n, s)); return;
        case COPYZ: OK(ono_scale_zero_f32((float *)a.out[0], (const float *)a.in[0], n, 1.0f, (float *)a.out[1], s)); return;
        case FILL: OK(ono_fill_f32((float *)a.out[0], 0.0f, n, s)); return;
        case DEC: OK(ono_f16_decode_scale((float *)a.out[0], (const uint16_t *)a.in[0], n, 2.0f, s)); return;
        case SUM2: case SUM4: case SUM8: {
            const int k = shape == SUM2 ? 2 : shape == SUM4 ? 4 : 8;
            const float *ins[8];
            for (int j = 0; j < k; j++) ins[j] = (const float *)a.in[j];
            OK(ono_sum_scale_f32((float *)a.out[0], ins, k, n, (float)k, s));
            return;
        }
        default: return;
        }
    }
    switch (shape) {
    case COPY: L2(k_copy) break;
    case COPYZ: L2(k_copyz) break;
    case FILL: L2(k_fill) break;
    case SUM2: L2(k_sum2) break;
    case DEC: L2(k_dec) break;
    case EMPTY: L2(k_empty) break;
    case COPY_SC1: L2(k_copy_sc1) break;
    case COPY_SYS: L2(k_copy_sys) break;
    case SUM2_SC1: L2(k_sum2_sc1) break;
    case SUM2_SYS: L2(k_sum2_sys) break;
    case FILL_SC1: L2(k_fill_sc1) break;
    case FILL_SYS: L2(k_fill_sys) break;
    case FILL_PLAIN: L2(k_fill_plain) break;
    case DEC_SC1: L2(k_dec_sc1) break;
    case DEC_SYS: L2(k_dec_sys) break;
    case DEC_PLAIN: L2(k_dec_plain) break;
    case FILL_U4: L2T(k_fill_u, 4) break;
    case FILL_U16: L2T(k_fill_u, 16) break;
    case FILL_B256: L2(k_fill_b256) break;
    case FILL_GRID: L2(k_fill_grid) break;
    case DEC_U2: L2T(k_dec_u, 2) break;
    case DEC_U4: L2T(k_dec_u, 4) break;
    case DEC_B256: L2(k_dec_b256) break;
    case COPY_U2: L2(k_copy_u2) break;
    case COPY_B256: L2(k_copy_b256) break;
    case DEC_B256_SC1: L2(k_dec_b256_sc1) break;
    case DEC_U2_B256: L2(k_dec_u2_b256) break;
    case FILL_U4_B256: L2(k_fill_u4_b256) break;
    case COPYZ_OCC24:
        if (st) hipLaunchKernelGGL(k_copyz<true>, dim3(grid), dim3(blk), lds_for_occ(24), s, a);
        else hipLaunchKernelGGL(k_copyz<false>, dim3(grid), dim3(blk), lds_for_occ(24), s, a);
        break;
    case COPYZ_B256: L2(k_copyz_b256) break;
    case COPYZ_B256_OCC6:  // at most 6 four-wave workgroups per CU (24 waves)
        if (st) hipLaunchKernelGGL(k_copyz_b256<true>, dim3(grid), dim3(blk), lds_for_occ(6), s, a);
        else hipLaunchKernelGGL(k_copyz_b256<false>, dim3(grid), dim3(blk), lds_for_occ(6), s, a);
        break;
    case SUM4_HYB: case SUM8_HYB: case SUM4_HYB2: case SUM8_HYB2: {
        const unsigned l = lds_for_occ(28);
        if (shape == SUM4_HYB) {
            if (st) hipLaunchKernelGGL((k_sumser<4, true, 1>), dim3(grid), dim3(blk), l, s, a);
            else hipLaunchKernelGGL((k_sumser<4, false, 1>), dim3(grid), dim3(blk), l, s, a);
        } else if (shape == SUM8_HYB) {
            if (st) hipLaunchKernelGGL((k_sumser<8, true, 1>), dim3(grid), dim3(blk), l, s, a);
            else hipLaunchKernelGGL((k_sumser<8, false, 1>), dim3(grid), dim3(blk), l, s, a);
        } else if (shape == SUM4_HYB2) {
            if (st) hipLaunchKernelGGL((k_sumser<4, true, 2>), dim3(grid), dim3(blk), l, s, a);
            else hipLaunchKernelGGL((k_sumser<4, false, 2>), dim3(grid), dim3(blk), l, s, a);
        } else {
            if (st) hipLaunchKernelGGL((k_sumser<8, true, 2>), dim3(grid), dim3(blk), l, s, a);
            else hipLaunchKernelGGL((k_sumser<8, false, 2>), dim3(grid), dim3(blk), l, s, a);
        }
        break;
    }
    case COPYZ_U2_OCC12:
        if (st) hipLaunchKernelGGL(k_copyz_u2<true>, dim3(grid), dim3(blk), lds_for_occ(12), s, a);
        else hipLaunchKernelGGL(k_copyz_u2<false>, dim3(grid), dim3(blk), lds_for_occ(12), s, a);
        break;
    case SUM4:
        if (st) hipLaunchKernelGGL((k_sumser<4, true>), dim3(grid), dim3(64), lds_for_occ(28), s, a);
        else hipLaunchKernelGGL((k_sumser<4, false>), dim3(grid), dim3(64), lds_for_occ(28), s, a);
        break;
    case SUM8:
        if (st) hipLaunchKernelGGL((k_sumser<8, true>), dim3(grid), dim3(64), lds_for_occ(28), s, a);
        else hipLaunchKernelGGL((k_sumser<8, false>), dim3(grid), dim3(64), lds_for_occ(28), s, a);
        break;
    }
#undef L2
#undef L2T
    CK(hipGetLastError());
}

struct Phases {
    double span, gap, ramp, ideal, drain, xcd, rate_gbs, first_to_last_start, tail;
};

static double median(std::vector<double> v) {
    if (v.empty()) return 0;
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

// stamps of L launches (nwg each), ticks of 10 ns
static Phases analyse(const std::vector<Stamp> &h, size_t nwg, double bytes) {
    std::vector<double> span, gap, ramp, ideal, drain, xcd, rate, fls, tail;
    std::vector<double> first(L), last(L);
    for (int i = 0; i < L; i++) {
        const Stamp *s = &h[(size_t)i * nwg];
        std::vector<double> st(nwg), en(nwg);
        double xend[16] = {0};
        for (size_t w = 0; w < nwg; w++) {
            const uint64_t t0 = ((uint64_t)s[w].t0_hi << 32) | s[w].t0_lo;
            st[w] = (double)t0 * 10.0;  // ns
            en[w] = st[w] + (double)s[w].dt * 10.0;
            const unsigned x = (s[w].ids >> 16) & 0xF;
            xend[x] = std::max(xend[x], en[w]);
        }
        std::sort(st.begin(), st.end());
        std::sort(en.begin(), en.end());
        first[i] = st.front();
        last[i] = en.back();
        const size_t a = nwg / 5, b = nwg * 4 / 5;
        const double R = (double)(b - a) / std::max(1.0, en[b] - en[a]);  // workgroups per ns
        const double t_lo = en[a] - (double)a / R, t_hi = en[b] + (double)(nwg - 1 - b) / R;
        span.push_back(last[i] - first[i]);
        ramp.push_back(t_lo - first[i]);
        ideal.push_back(t_hi - t_lo);
        drain.push_back(last[i] - t_hi);
        rate.push_back(bytes / ((double)nwg / R));  // bytes per ns = GB/s
        fls.push_back(st.back() - st.front());
        tail.push_back(last[i] - st.back());
        double lo = 1e300, hi = 0;
        for (int x = 0; x < 16; x++)
            if (xend[x] > 0) { lo = std::min(lo, xend[x]); hi = std::max(hi, xend[x]); }
        xcd.push_back(hi - lo);
    }
    for (int i = 0; i + 1 < L; i++) gap.push_back(first[i + 1] - last[i]);
    return {median(span) / 1e3, median(gap) / 1e3, median(ramp) / 1e3, median(ideal) / 1e3, median(drain) / 1e3,
            median(xcd) / 1e3, median(rate), median(fls) / 1e3, median(tail) / 1e3};
}

// Per XCD of one launch (the median launch by span): workgroups, first start and last end relative to
// the launch's first start, median workgroup lifetime; and how many workgroups each XCD finishes in
// the launch's last microsecond.
static void xcd_detail(const std::vector<Stamp> &h, size_t nwg, const char *name) {
    std::vector<std::pair<double, int>> spans;
    for (int i = 0; i < L; i++) {
        const Stamp *s = &h[(size_t)i * nwg];
        double lo = 1e300, hi = 0;
        for (size_t w = 0; w < nwg; w++) {
            const double t0 = (double)(((uint64_t)s[w].t0_hi << 32) | s[w].t0_lo) * 10.0;
            lo = std::min(lo, t0);
            hi = std::max(hi, t0 + s[w].dt * 10.0);
        }
        spans.push_back({hi - lo, i});
    }
    std::sort(spans.begin(), spans.end());
    const int i = spans[spans.size() / 2].second;
    const Stamp *s = &h[(size_t)i * nwg];
    double lo = 1e300, hi = 0;
    for (size_t w = 0; w < nwg; w++) {
        const double t0 = (double)(((uint64_t)s[w].t0_hi << 32) | s[w].t0_lo) * 10.0;
        lo = std::min(lo, t0);
        hi = std::max(hi, t0 + s[w].dt * 10.0);
    }
    printf("#   %s, launch %d (median span %.2f us), per XCD: wgs first_start last_start last_end median_life "
           "ends_in_last_us  (us from the launch's first start)\n", name, i, (hi - lo) / 1e3);
    for (int x = 0; x < 8; x++) {
        std::vector<double> life;
        double fs = 1e300, ls = 0, le = 0;
        int tail = 0;
        for (size_t w = 0; w < nwg; w++) {
            if (((s[w].ids >> 16) & 0xF) != (unsigned)x) continue;
            const double t0 = (double)(((uint64_t)s[w].t0_hi << 32) | s[w].t0_lo) * 10.0 - lo;
            const double t1 = t0 + s[w].dt * 10.0;
            fs = std::min(fs, t0);
            ls = std::max(ls, t0);
            le = std::max(le, t1);
            life.push_back(s[w].dt * 10.0);
            tail += t1 > (hi - lo) - 1000.0;
        }
        if (life.empty()) continue;
        printf("#     xcd %d  %6zu  %7.2f  %7.2f  %7.2f  %6.2f  %5d\n", x, life.size(), fs / 1e3, ls / 1e3, le / 1e3,
               median(life) / 1e3, tail);
    }
}

static void run_size(size_t mib, hipStream_t s) {
    const size_t n = mib << 18, nvec = n / 4, nwg_max = (nvec + 63) / 64;
    Stamp *dst;
    CK(hipMalloc(&dst, sizeof(Stamp) * nwg_max * L));
    printf("\n# %zu MiB per buffer (%zu f32, %zu workgroups), %d back-to-back launches per row, medians\n", mib, n, nwg_max,
           L);
    printf("# %-16s %9s %9s %9s | %8s %7s %7s %7s %7s %7s %7s %7s | %8s %6s\n", "shape", "ev_us", "stamp_us", "lib_us",
           "span", "gap", "ramp", "ideal", "drain", "xcd", "dstart", "tail", "R_GB/s", "frac");
    for (int shape = 0; shape < NSHAPES; shape++) {
        const size_t nwg = grid_of(shape, nvec, g_cus);
        const int per = kReads[shape] + kWrites[shape];
        const int nsets = per ? kPool / per : 1;
        auto args = [&](int it) {
            Args a{};
            const int set = it % nsets;
            for (int j = 0; j < kReads[shape]; j++) a.in[j] = g_pool[set * per + j];
            for (int j = 0; j < kWrites[shape]; j++) a.out[j] = g_pool[set * per + kReads[shape] + j];
            a.nvec = nvec;
            a.first = (uint32_t)g_cus * 28u;
            a.st = dst + (size_t)(it % L) * nwg;
            return a;
        };
        double us[3] = {0, 0, 0};
        std::vector<Stamp> h;
        for (int mode = 0; mode < 3; mode++) {
            if (mode == 2 && (shape == EMPTY || shape >= COPY_SC1)) continue;
            for (int it = 0; it < nsets + 2; it++) launch(shape, mode, args(it), n, s);  // whole rotation touched
            CK(hipStreamSynchronize(s));
            hipEvent_t e0, e1;
            CK(hipEventCreate(&e0));
            CK(hipEventCreate(&e1));
            CK(hipEventRecord(e0, s));
            for (int it = 0; it < L; it++) {
                Args a = args(nsets + 2 + it);
                a.st = dst + (size_t)it * nwg;
                launch(shape, mode, a, n, s);
            }
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            us[mode] = ms * 1e3 / L;
            CK(hipEventDestroy(e0));
            CK(hipEventDestroy(e1));
            if (mode == 1) {
                h.resize(nwg * L);
                CK(hipMemcpy(h.data(), dst, sizeof(Stamp) * nwg * L, hipMemcpyDeviceToHost));
            }
        }
        const double bytes = kBytes[shape] * (double)n;
        const Phases p = analyse(h, nwg, bytes);
        if (shape == SUM2 || shape == COPY || shape == SUM8) xcd_detail(h, nwg, kName[shape]);
        const double best = us[2] > 0 ? std::min(us[0], us[2]) : us[0];
        printf("%-18s %9.2f %9.2f %9.2f | %8.2f %7.2f %7.2f %7.2f %7.2f %7.2f %7.2f %7.2f | %8.0f %6.3f\n", kName[shape],
               us[0], us[1], us[2], p.span, p.gap, p.ramp, p.ideal, p.drain, p.xcd, p.first_to_last_start, p.tail,
               p.rate_gbs, bytes ? bytes / (best * 1e3) / 8000.0 : 0.0);
        fflush(stdout);
    }
    CK(hipFree(dst));
}

int main(int argc, char **argv) {
    std::vector<size_t> sizes = {64, 256};
    if (argc > 1) {
        sizes.clear();
        for (char *t = strtok(argv[1], ","); t; t = strtok(nullptr, ",")) sizes.push_back((size_t)atol(t));
    }
    if (argc > 2) L = atoi(argv[2]);
    const bool synth = argc > 3 && !strcmp(argv[3], "synth");  // the bench's gradient distribution in every buffer
    size_t mx = 0;
    for (size_t m : sizes) mx = std::max(mx, m);
    g_max_elems = mx << 18;
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    g_cus = p.multiProcessorCount;
    printf("# launch_phases: %s, %d CUs; stamps = s_memrealtime (100 MHz) per workgroup, lane 0; data: %s\n",
           p.gcnArchName, p.multiProcessorCount, synth ? "ono_synth_f32 (the bench's)" : "k_init pattern");
    printf("# ev_us: HIP events around L launches (un-stamped tool kernel); stamp_us: the stamped build; lib_us: the\n"
           "# product library on the same buffers; span/gap/ramp/ideal/drain/xcd/dstart/tail in us from the stamps\n"
           "# (dstart = first -> last workgroup start, tail = last start -> last end); R = fitted steady rate of\n"
           "# algorithmic bytes; frac = algorithmic bytes / min(ev_us, lib_us) of 8 TB/s\n");
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (int i = 0; i < kPool; i++) {
        f4 *q;
        CK(hipMalloc(&q, g_max_elems * 4));
        if (synth) OK(ono_synth_f32((float *)q, g_max_elems, 0x0402026 + i, (uint64_t)(i % 9), 0, s));
        else hipLaunchKernelGGL(k_init, dim3(4096), dim3(256), 0, s, q, g_max_elems / 4, 17u + i);
        g_pool.push_back(q);
    }
    CK(hipStreamSynchronize(s));
    for (size_t m : sizes) run_size(m, s);
    for (f4 *q : g_pool) CK(hipFree(q));
    return 0;
}
