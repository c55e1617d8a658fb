// skeleton_variants.hip — measurement tool (not part of the product): the
// stream skeleton of csrc/ono_kernels.hip (ew_kernel) against leaner one-shot
// forms, on the path's HBM shapes, interleaved over several passes (median,
// so clock / box drift hits every variant alike).  Buffers rotate over > 1.5
// GiB so the 256 MiB Infinity Cache cannot serve re-reads; one HIP event pair
// around L back-to-back launches, like bench.py.
//
//   shapes: sum2 / sum4 / sum8 (kR1W, *0.5), dec (f16 -> f32 * 0.125, 2 B in,
//           4 B out), acc (acc += in, nt loads), sz (dst = src; zero = 0, 1R2W)
//   skeletons:
//     loop   the product's: grid-stride loop over a one-shot grid, per-thread
//            head / tail checks (head = 0 here, so only the compares remain)
//     shot   one vector per lane, `if (v < nvec)` guard, no loop
//     shot2  two vectors per lane one wave apart (U = 2), loads first
//     b256   shot with 256-thread workgroups
//
//   skew mode: the `shot` skeleton with operand j placed j * skew bytes past
//   its buffer's start (buffers come from hipMalloc at large power-of-two
//   alignments, so the same element of every operand otherwise maps to the
//   same HBM channel / bank)
//
//   hipcc --offload-arch=gfx950 -O3 -o skeleton_variants skeleton_variants.hip
//   ./skeleton_variants [MiB per f32 buffer = 64] [passes = 5] [skew]
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

static size_t N = 16u << 20;
constexpr int L = 30, W = 3;

template <class T> __device__ __forceinline__ T ldn(const T *p) { return __builtin_nontemporal_load(p); }
template <class T> __device__ __forceinline__ void stn(T *p, T v) { __builtin_nontemporal_store(v, p); }
__device__ __forceinline__ void st_sc1(f4 *p, f4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" : : "v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ float dec1(uint16_t b) { return (float)__builtin_bit_cast(_Float16, b); }

struct Args {
    const void *in[8];
    void *out, *out2;
};

// one vector's work of each shape
template <int S> struct Shape;
template <int K> struct SumShape {
    static constexpr double bytes_per_elem = 4.0 * (K + 1);
    __device__ __forceinline__ static void load(const Args &a, size_t v, f4 &r) {
        r = ldn((const f4 *)a.in[0] + v);
#pragma unroll
        for (int j = 1; j < K; j++) r += ldn((const f4 *)a.in[j] + v);
    }
    __device__ __forceinline__ static void store(const Args &a, size_t v, f4 r) { stn((f4 *)a.out + v, r * 0.5f); }
};
struct DecShape {
    static constexpr double bytes_per_elem = 6.0;
    __device__ __forceinline__ static void load(const Args &a, size_t v, f4 &r) {
        h4 h = ldn((const h4 *)a.in[0] + v);
        r = f4{dec1(h.x), dec1(h.y), dec1(h.z), dec1(h.w)};
    }
    __device__ __forceinline__ static void store(const Args &a, size_t v, f4 r) { stn((f4 *)a.out + v, r * 0.125f); }
};
// the product's decode: half 2.7.1 f16_to_f32 with its NaN rule spelled out
__device__ __forceinline__ float dec1_nan(uint16_t b) {
    float f = (float)__builtin_bit_cast(_Float16, b);
    uint32_t nb = ((uint32_t)(b & 0x8000u) << 16) | 0x7FC00000u | ((uint32_t)(b & 0x3FFu) << 13);
    bool nan = ((b & 0x7C00u) == 0x7C00u) && (b & 0x3FFu);
    return nan ? __builtin_bit_cast(float, nb) : f;
}
struct DecNanShape {
    static constexpr double bytes_per_elem = 6.0;
    __device__ __forceinline__ static void load(const Args &a, size_t v, f4 &r) {
        h4 h = ldn((const h4 *)a.in[0] + v);
        r = f4{dec1_nan(h.x), dec1_nan(h.y), dec1_nan(h.z), dec1_nan(h.w)};
    }
    __device__ __forceinline__ static void store(const Args &a, size_t v, f4 r) { stn((f4 *)a.out + v, r * 0.125f); }
};
struct AccShape {
    static constexpr double bytes_per_elem = 12.0;
    __device__ __forceinline__ static void load(const Args &a, size_t v, f4 &r) {
        r = ldn((const f4 *)a.out + v) + ldn((const f4 *)a.in[0] + v);
    }
    __device__ __forceinline__ static void store(const Args &a, size_t v, f4 r) { stn((f4 *)a.out + v, r); }
};
struct SzShape {
    static constexpr double bytes_per_elem = 12.0;
    __device__ __forceinline__ static void load(const Args &a, size_t v, f4 &r) { r = ldn((const f4 *)a.in[0] + v); }
    __device__ __forceinline__ static void store(const Args &a, size_t v, f4 r) {
        st_sc1((f4 *)a.out + v, r);
        st_sc1((f4 *)a.out2 + v, f4{0, 0, 0, 0});
    }
};

template <class Sh>
__global__ __launch_bounds__(64) void k_loop(Args a, size_t head, size_t nvec, size_t n) {
    const size_t tid = (size_t)blockIdx.x * 64 + threadIdx.x, stride = (size_t)gridDim.x * 64;
    const size_t tail0 = head + 4 * nvec;
    if (tid < head) ((float *)a.out)[tid] = 0.0f;
    if (tid < n - tail0) ((float *)a.out)[tail0 + tid] = 0.0f;
    for (size_t v = tid; v < nvec; v += stride) {
        f4 r;
        Sh::load(a, v, r);
        Sh::store(a, v, r);
    }
}
template <class Sh, int B>
__global__ __launch_bounds__(B) void k_shot(Args a, size_t nvec) {
    const size_t v = (size_t)blockIdx.x * B + threadIdx.x;
    if (v < nvec) {
        f4 r;
        Sh::load(a, v, r);
        Sh::store(a, v, r);
    }
}
template <class Sh>
__global__ __launch_bounds__(64) void k_shot2(Args a, size_t nvec) {
    const size_t v0 = (size_t)blockIdx.x * 128 + threadIdx.x, v1 = v0 + 64;
    f4 r0, r1;
    if (v0 < nvec) Sh::load(a, v0, r0);
    if (v1 < nvec) Sh::load(a, v1, r1);
    if (v0 < nvec) Sh::store(a, v0, r0);
    if (v1 < nvec) Sh::store(a, v1, r1);
}

__global__ void k_fill(f4 *p, size_t nvec, unsigned seed) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (size_t)gridDim.x * 256) {
        unsigned h = (unsigned)i * 2654435761u ^ seed;
        p[i] = f4{(float)(h & 0xFFFF), (float)(h >> 16), (float)(h & 0xFF), 1.0f} * 1e-4f;
    }
}

constexpr size_t kSlack = 1u << 20;  // spare bytes per buffer for the skewed operands
static std::vector<f4 *> g_bufs;
static hipStream_t g_s;
static f4 *buf(int i) {
    while ((int)g_bufs.size() <= i) {
        f4 *p;
        CK(hipMalloc(&p, N * sizeof(float) + kSlack));
        hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, g_s, p, N / 4, 17u + (unsigned)g_bufs.size());
        g_bufs.push_back(p);
    }
    return g_bufs[i];
}

struct Row {
    std::string name;
    double bytes;
    int per_set;  // buffers per set
    void (*launch)(const Args &, size_t nvec);
    std::vector<double> us;
    size_t skew = 0;  // operand j starts j * skew bytes into its buffer
};

template <class Sh> void L_loop(const Args &a, size_t nvec) {
    hipLaunchKernelGGL(k_loop<Sh>, dim3((unsigned)((nvec + 63) / 64)), dim3(64), 0, g_s, a, (size_t)0, nvec, 4 * nvec);
}
template <class Sh> void L_shot(const Args &a, size_t nvec) {
    hipLaunchKernelGGL((k_shot<Sh, 64>), dim3((unsigned)((nvec + 63) / 64)), dim3(64), 0, g_s, a, nvec);
}
template <class Sh> void L_b256(const Args &a, size_t nvec) {
    hipLaunchKernelGGL((k_shot<Sh, 256>), dim3((unsigned)((nvec + 255) / 256)), dim3(256), 0, g_s, a, nvec);
}
template <class Sh> void L_shot2(const Args &a, size_t nvec) {
    hipLaunchKernelGGL(k_shot2<Sh>, dim3((unsigned)((nvec + 127) / 128)), dim3(64), 0, g_s, a, nvec);
}

// f16 decode with 8 values per lane (one 16-B load) and both f32 stores
// wave-contiguous (1 KiB each): lane l stores values 4l..4l+3 and 256+4l..,
// which lanes l/2 and 32 + l/2 loaded (two dwords each, picked by l's parity)
__global__ __launch_bounds__(64) void k_dec8(Args a, size_t nblk) {
    const size_t blk = blockIdx.x;
    if (blk >= nblk) return;
    const int l = threadIdx.x;
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    const u4 h = ldn((const u4 *)a.in[0] + blk * 64 + l);
    const int s0 = l >> 1, s1 = 32 + (l >> 1);
    const bool odd = l & 1;
    const uint32_t x0 = __shfl((int)h.x, s0), x1 = __shfl((int)h.y, s0), x2 = __shfl((int)h.z, s0),
                   x3 = __shfl((int)h.w, s0);
    const uint32_t y0 = __shfl((int)h.x, s1), y1 = __shfl((int)h.y, s1), y2 = __shfl((int)h.z, s1),
                   y3 = __shfl((int)h.w, s1);
    const uint32_t p0 = odd ? x2 : x0, p1 = odd ? x3 : x1, q0 = odd ? y2 : y0, q1 = odd ? y3 : y1;
    const f4 r0 = {dec1((uint16_t)p0), dec1((uint16_t)(p0 >> 16)), dec1((uint16_t)p1), dec1((uint16_t)(p1 >> 16))};
    const f4 r1 = {dec1((uint16_t)q0), dec1((uint16_t)(q0 >> 16)), dec1((uint16_t)q1), dec1((uint16_t)(q1 >> 16))};
    stn((f4 *)a.out + blk * 128 + l, r0 * 0.125f);
    stn((f4 *)a.out + blk * 128 + 64 + l, r1 * 0.125f);
}
void L_dec8(const Args &a, size_t nvec) {
    const size_t nblk = nvec / 128;  // 512 values per wave (N a multiple of 512 here)
    hipLaunchKernelGGL(k_dec8, dim3((unsigned)nblk), dim3(64), 0, g_s, a, nblk);
}

template <class Sh> void add_rows(std::vector<Row> &rows, const char *shape, int per_set) {
    const double b = Sh::bytes_per_elem * (double)N;
    rows.push_back({std::string(shape) + " loop", b, per_set, L_loop<Sh>, {}});
    rows.push_back({std::string(shape) + " shot", b, per_set, L_shot<Sh>, {}});
    rows.push_back({std::string(shape) + " shot2", b, per_set, L_shot2<Sh>, {}});
    rows.push_back({std::string(shape) + " b256", b, per_set, L_b256<Sh>, {}});
}

// Does the hardware conversion already follow the half crate's NaN rules?
//   f16 -> f32: sign | 0x7FC00000 | mant << 13     (every one of the 2^16 patterns)
//   f32 -> f16: sign | 0x7E00 | mant >> 13 for NaN (every NaN f32 pattern, 2^24 of them x sign)
__global__ void k_nan_check(unsigned long long *bad) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t < 65536u) {
        const uint16_t b = (uint16_t)t;
        const uint32_t hw = __builtin_bit_cast(uint32_t, (float)__builtin_bit_cast(_Float16, b));
        const uint32_t sw = __builtin_bit_cast(uint32_t, dec1_nan(b));
        if (hw != sw) atomicAdd(bad, 1ull);
    }
    // f32 NaNs: exponent all ones, mantissa != 0; t enumerates sign and mantissa
    const uint32_t mant = t & 0x7FFFFFu, sign = (t >> 23) & 1u;
    if (mant) {
        const uint32_t u = (sign << 31) | 0x7F800000u | mant;
        const float x = __builtin_bit_cast(float, u);
        const uint16_t hw = __builtin_bit_cast(uint16_t, (_Float16)x);
        const uint16_t sw = (uint16_t)(((u >> 16) & 0x8000u) | 0x7E00u | ((u & 0x7FFFFFu) >> 13));
        if (hw != sw) atomicAdd(bad + 1, 1ull);
    }
}

// ---- optimizer consumer / owner-chain shapes (mode "opt"): load policy L
// (0 plain, 1 nt) and store policy S (0 nt, 1 nt sc1) for the all-reduce
// consumer (GD: params, grad in; params, grad = 0, params copy out) with
// momentum / Adam state, and the 8-input owner chain (8 in; grad, message,
// own slice = 0 out)
template <int L> __device__ __forceinline__ f4 ldp(const void *p, size_t v) {
    if constexpr (L) return ldn((const f4 *)p + v);
    else return ((const f4 *)p)[v];
}
template <int S> __device__ __forceinline__ void stp(void *p, size_t v, f4 x) {
    if constexpr (S) st_sc1((f4 *)p + v, x);
    else stn((f4 *)p + v, x);
}
template <int KIND, int L, int S> struct OptShape {  // KIND 0 GD, 1 momentum, 2 Adam
    static constexpr double bytes_per_elem = KIND == 0 ? 20.0 : KIND == 1 ? 28.0 : 36.0;
    __device__ __forceinline__ static void run(const Args &a, size_t v) {
        f4 w = ldp<L>(a.in[0], v), g = ldp<L>(a.in[1], v) * 0.5f;
        if constexpr (KIND == 0) {
            w -= 0.1f * g;
        } else if constexpr (KIND == 1) {
            f4 m = ldp<L>(a.in[2], v) * 0.9f + g;
            stp<S>((void *)a.in[2], v, m);
            w -= 0.1f * m;
        } else {
            f4 m = ldp<L>(a.in[2], v) * 0.9f + 0.1f * g, q = ldp<L>(a.in[3], v) * 0.999f + 0.001f * g * g;
            stp<S>((void *)a.in[2], v, m);
            stp<S>((void *)a.in[3], v, q);
            w -= 0.001f * m / (f4{__builtin_sqrtf(q.x), __builtin_sqrtf(q.y), __builtin_sqrtf(q.z), __builtin_sqrtf(q.w)} + 1e-8f);
        }
        stp<S>((void *)a.in[0], v, w);
        stp<S>((void *)a.in[1], v, f4{0, 0, 0, 0});
        stp<S>(a.out, v, w);
    }
};
template <int L, int LO, int S> struct ChainShape {  // 7 received (policy L) + own (policy LO) -> grad, msg, own = 0
    static constexpr double bytes_per_elem = 44.0;
    __device__ __forceinline__ static void run(const Args &a, size_t v) {
        f4 p = ldp<L>(a.in[0], v);
#pragma unroll
        for (int k = 1; k < 7; k++) p = ldp<L>(a.in[k], v) + p;
        p = ldp<LO>(a.in[7], v) + p;
        const f4 gv = p * 0.125f;
        stp<S>(a.out, v, gv);
        stp<S>(a.out2, v, gv);
        stp<S>((void *)a.in[7], v, f4{0, 0, 0, 0});
    }
};
template <class Sh>
__global__ __launch_bounds__(64) void k_run(Args a, size_t nvec) {
    const size_t v = (size_t)blockIdx.x * 64 + threadIdx.x;
    if (v < nvec) Sh::run(a, v);
}
template <class Sh> void L_run(const Args &a, size_t nvec) {
    hipLaunchKernelGGL(k_run<Sh>, dim3((unsigned)((nvec + 63) / 64)), dim3(64), 0, g_s, a, nvec);
}

int main(int argc, char **argv) {
    if (argc > 1) N = (size_t)atol(argv[1]) << 18;
    const int passes = argc > 2 ? atoi(argv[2]) : 5;
    CK(hipStreamCreateWithFlags(&g_s, hipStreamNonBlocking));
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    printf("# %s, %d CUs, %zu f32 elements per buffer (%zu MiB), %d passes, median of per-pass means\n",
           p.gcnArchName, p.multiProcessorCount, N, N >> 18, passes);
    std::vector<Row> rows;
    if (argc > 3 && !strcmp(argv[3], "nan")) {
        unsigned long long *bad, hb[2];
        CK(hipMalloc(&bad, 16));
        CK(hipMemset(bad, 0, 16));
        hipLaunchKernelGGL(k_nan_check, dim3((1u << 24) / 256), dim3(256), 0, g_s, bad);
        CK(hipMemcpy(hb, bad, 16, hipMemcpyDeviceToHost));
        printf("hardware vs half-crate NaN rule: f16->f32 mismatches %llu of 65536, f32->f16 NaN mismatches %llu of "
               "%u\n", hb[0], hb[1], (1u << 24) - 2);
        add_rows<DecShape>(rows, "dec", 2);
        add_rows<DecNanShape>(rows, "decnan", 2);
    } else if (argc > 3 && !strcmp(argv[3], "opt")) {
        auto add = [&](const char *nm, double bpe, int per, void (*f)(const Args &, size_t)) {
            rows.push_back(Row{nm, bpe * (double)N, per, f, {}});
        };
        add("gd L0 S0", 20, 3, L_run<OptShape<0, 0, 0>>);
        add("gd L1 S0", 20, 3, L_run<OptShape<0, 1, 0>>);
        add("gd L1 S1", 20, 3, L_run<OptShape<0, 1, 1>>);
        add("mom L0 S0", 28, 4, L_run<OptShape<1, 0, 0>>);
        add("mom L1 S0", 28, 4, L_run<OptShape<1, 1, 0>>);
        add("mom L1 S1", 28, 4, L_run<OptShape<1, 1, 1>>);
        add("adam L0 S0", 36, 5, L_run<OptShape<2, 0, 0>>);
        add("adam L1 S0", 36, 5, L_run<OptShape<2, 1, 0>>);
        add("adam L1 S1", 36, 5, L_run<OptShape<2, 1, 1>>);
        add("chain8 L1 LO0 S0", 44, 10, L_run<ChainShape<1, 0, 0>>);
        add("chain8 L1 LO1 S0", 44, 10, L_run<ChainShape<1, 1, 0>>);
        add("chain8 L1 LO1 S1", 44, 10, L_run<ChainShape<1, 1, 1>>);
        add("chain8 L0 LO0 S0", 44, 10, L_run<ChainShape<0, 0, 0>>);
    } else if (argc > 3 && !strcmp(argv[3], "dec8")) {
        rows.push_back({"dec shot", DecShape::bytes_per_elem * (double)N, 2, L_shot<DecShape>, {}});
        rows.push_back({"dec8 shuffled", DecShape::bytes_per_elem * (double)N, 2, L_dec8, {}});
    } else if (argc > 3 && !strcmp(argv[3], "skew")) {
        for (size_t sk : {(size_t)0, (size_t)256, (size_t)2048, (size_t)4096, (size_t)8192, (size_t)65536 + 512}) {
            char nm[64];
            auto add = [&](const char *shape, double bpe, int per, void (*f)(const Args &, size_t)) {
                snprintf(nm, sizeof nm, "%s skew=%zu", shape, sk);
                Row r{nm, bpe * (double)N, per, f, {}};
                r.skew = sk;
                rows.push_back(r);
            };
            add("sum2", SumShape<2>::bytes_per_elem, 3, L_shot<SumShape<2>>);
            add("sum4", SumShape<4>::bytes_per_elem, 5, L_shot<SumShape<4>>);
            add("sum8", SumShape<8>::bytes_per_elem, 9, L_shot<SumShape<8>>);
            add("dec", DecShape::bytes_per_elem, 2, L_shot<DecShape>);
            add("sz", SzShape::bytes_per_elem, 3, L_shot<SzShape>);
        }
    } else {
        add_rows<SumShape<2>>(rows, "sum2", 3);
        add_rows<SumShape<4>>(rows, "sum4", 5);
        add_rows<SumShape<8>>(rows, "sum8", 9);
        add_rows<DecShape>(rows, "dec", 2);
        add_rows<AccShape>(rows, "acc", 2);
        add_rows<SzShape>(rows, "sz", 3);
    }
    const size_t nvec = N / 4;
    const double rot = 1.6 * (1u << 30);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int pass = 0; pass < passes; pass++) {
        for (Row &r : rows) {
            const int nsets = std::max(2, (int)(rot / (r.per_set * (double)N * 4)) + 1);
            auto go = [&](int i) {
                const int set = i % nsets;
                Args a{};
                auto op = [&](int j) { return (void *)((char *)buf(set * r.per_set + j) + (size_t)j * r.skew); };
                for (int j = 0; j < r.per_set - 1 && j < 8; j++) a.in[j] = op(j);
                a.out = op(r.per_set - 1);
                a.out2 = op(r.per_set > 2 ? 1 : 0);
                if (r.name.rfind("sz", 0) == 0) a.out2 = op(1);
                if (r.per_set == 10) a.out2 = op(8);  // chain8: 8 inputs, grad, message
                r.launch(a, nvec);
            };
            for (int i = 0; i < W; i++) go(i);
            CK(hipStreamSynchronize(g_s));
            CK(hipEventRecord(e0, g_s));
            for (int i = 0; i < L; i++) go(W + i);
            CK(hipEventRecord(e1, g_s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            r.us.push_back(ms * 1e3 / L);
        }
        printf("# pass %d done\n", pass);
        fflush(stdout);
    }
    for (Row &r : rows) {
        std::vector<double> v = r.us;
        std::sort(v.begin(), v.end());
        const double med = v[v.size() / 2], gbs = r.bytes / (med * 1e-6) / 1e9;
        printf("%-12s median %8.2f us  min %8.2f  max %8.2f  %8.1f GB/s  %.3f of 8000\n", r.name.c_str(), med, v.front(),
               v.back(), gbs, gbs / 8000.0);
    }
    for (f4 *q : g_bufs) CK(hipFree(q));
    return 0;
}
