// ono_sparse.hip — the sparse top-(1-r) gradient codec on gfx950
// (comms/src/sparse/protocol.rs:33-144).
//
// Wire format (grad_drop_into, protocol.rs:57-86), all little-endian:
//   [u64 total_len] { [u32 offset from previous run end][u32 run length][f16 x len] }*
// where a run is a maximal stretch of consecutive |g| >= threshold.
//
// Encoding is a stream compaction.  For element i let F(i) = kept values
// before i and S(i) = runs started at or before i; a kept value lands at byte
//   8 + 8 S(i) + 2 F(i)
// and run j (starting at s_j) has its header 8 bytes earlier, with
//   offset_j = U(s_j) - U(s_{j-1}),  U(i) = i - F(i)  (unkept values before i)
//   len_j    = F(s_{j+1}) - F(s_j)   (F_total for the last run).
// Four launches: per-tile counts -> tile scan -> write (block-wide scan with
// wave shuffles + LDS; values written, run starts record U and F) -> headers.
// Decoding walks the run headers on the host (a sequential parse, as in the
// reference, over R records) and expands all values on the device.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <vector>

#include "ono_internal.h"

using namespace ono;

namespace {

constexpr int kSB = 256;             // threads per block (4 waves)
constexpr int kEPT = 8;              // elements per thread
constexpr int kTile = kSB * kEPT;    // 2048 elements per tile

__device__ __forceinline__ uint16_t to_f16_sp(float x) {  // half 2.7.1 f32 -> f16
    uint16_t b = __builtin_bit_cast(uint16_t, (_Float16)x);
    uint32_t u = __builtin_bit_cast(uint32_t, x);
    uint16_t nb = (uint16_t)(((u >> 16) & 0x8000u) | 0x7E00u | ((u & 0x7FFFFFu) >> 13));
    return __builtin_isnan(x) ? nb : b;
}
__device__ __forceinline__ float from_f16_sp(uint16_t b) {
    float f = (float)__builtin_bit_cast(_Float16, b);
    uint32_t nb = ((uint32_t)(b & 0x8000u) << 16) | 0x7FC00000u | ((uint32_t)(b & 0x3FFu) << 13);
    bool nan = ((b & 0x7C00u) == 0x7C00u) && (b & 0x3FFu);
    return nan ? __builtin_bit_cast(float, nb) : f;
}

// g.abs() >= threshold (NaN never kept, as in Rust)
__device__ __forceinline__ bool kept(float x, float t) { return fabsf(x) >= t; }

// Flags of a thread's kEPT elements: bit e = kept, plus whether each starts a run.
struct Bits {
    uint32_t keep = 0, start = 0;
};
__device__ __forceinline__ Bits thread_bits(const float *g, size_t n, float t, size_t base) {
    Bits b;
    bool prev = base > 0 && base - 1 < n ? kept(g[base - 1], t) : false;
#pragma unroll
    for (int e = 0; e < kEPT; e++) {
        size_t i = base + e;
        bool k = i < n && kept(g[i], t);
        if (k) b.keep |= 1u << e;
        if (k && !prev) b.start |= 1u << e;
        prev = k;
    }
    return b;
}

// Exclusive block-wide scan of (a, b) pairs: wave-level shuffles (64 lanes),
// then the 4 wave totals through LDS.  Returns the block totals too.
__device__ __forceinline__ void block_scan2(uint32_t a, uint32_t b, uint32_t &ea, uint32_t &eb, uint32_t &ta,
                                            uint32_t &tb) {
    __shared__ uint32_t wa[kSB / 64], wb[kSB / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t ia = a, ib = b;  // inclusive wave scan
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t ya = __shfl_up(ia, d, 64), yb = __shfl_up(ib, d, 64);
        if (lane >= d) { ia += ya; ib += yb; }
    }
    if (lane == 63) { wa[wave] = ia; wb[wave] = ib; }
    __syncthreads();
    uint32_t pa = 0, pb = 0;
    ta = 0; tb = 0;
#pragma unroll
    for (int w = 0; w < kSB / 64; w++) {
        if (w < wave) { pa += wa[w]; pb += wb[w]; }
        ta += wa[w];
        tb += wb[w];
    }
    ea = pa + ia - a;
    eb = pb + ib - b;
}

__global__ __launch_bounds__(kSB) void sp_count(const float *g, size_t n, float t, uint32_t *tileF, uint32_t *tileS) {
    Bits b = thread_bits(g, n, t, (size_t)blockIdx.x * kTile + (size_t)threadIdx.x * kEPT);
    uint32_t ea, eb, ta, tb;
    block_scan2(__popc(b.keep), __popc(b.start), ea, eb, ta, tb);
    if (threadIdx.x == 0) { tileF[blockIdx.x] = ta; tileS[blockIdx.x] = tb; }
}

// Exclusive scan of the tile counts in place (one block, running carry);
// totals[0] = kept values, totals[1] = runs.
__global__ __launch_bounds__(kSB) void sp_scan_tiles(uint32_t *tileF, uint32_t *tileS, size_t ntiles,
                                                     uint64_t *totals) {
    __shared__ uint32_t carryF, carryS;
    if (threadIdx.x == 0) { carryF = 0; carryS = 0; }
    __syncthreads();
    for (size_t base = 0; base < ntiles; base += kSB) {
        size_t i = base + threadIdx.x;
        uint32_t f = i < ntiles ? tileF[i] : 0, s = i < ntiles ? tileS[i] : 0;
        uint32_t ea, eb, ta, tb;
        block_scan2(f, s, ea, eb, ta, tb);
        uint32_t cf = carryF, cs = carryS;
        if (i < ntiles) { tileF[i] = cf + ea; tileS[i] = cs + eb; }
        __syncthreads();
        if (threadIdx.x == 0) { carryF = cf + ta; carryS = cs + tb; }
        __syncthreads();
    }
    if (threadIdx.x == 0) { totals[0] = carryF; totals[1] = carryS; }
}

__global__ __launch_bounds__(kSB) void sp_write(const float *g, size_t n, float t, const uint32_t *tileF,
                                                const uint32_t *tileS, uint8_t *buf, uint32_t *RU, uint32_t *RF) {
    const size_t base = (size_t)blockIdx.x * kTile + (size_t)threadIdx.x * kEPT;
    Bits b = thread_bits(g, n, t, base);
    uint32_t ea, eb, ta, tb;
    block_scan2(__popc(b.keep), __popc(b.start), ea, eb, ta, tb);
    uint32_t F = tileF[blockIdx.x] + ea;   // kept values before this thread's first element
    uint32_t S = tileS[blockIdx.x] + eb;   // runs started before it
#pragma unroll
    for (int e = 0; e < kEPT; e++) {
        if (!(b.keep >> e & 1u)) continue;
        size_t i = base + e;
        if (b.start >> e & 1u) {
            RU[S] = (uint32_t)(i - F);  // U(s_j): unkept values before the run
            RF[S] = F;                  // F(s_j)
            S++;
        }
        *(uint16_t *)(buf + 8 + 8 * (size_t)S + 2 * (size_t)F) = to_f16_sp(g[i]);
        F++;
    }
}

__global__ __launch_bounds__(kSB) void sp_headers(const uint32_t *RU, const uint32_t *RF, size_t R, uint32_t Ftot,
                                                  uint64_t total_len, uint8_t *buf) {
    size_t j = (size_t)blockIdx.x * kSB + threadIdx.x;
    if (j == 0) {  // u64 LE total length, as four 2-byte stores (buf is 2-B aligned)
        for (int q = 0; q < 4; q++) *(uint16_t *)(buf + 2 * q) = (uint16_t)(total_len >> (16 * q));
    }
    if (j >= R) return;
    uint32_t off = RU[j] - (j ? RU[j - 1] : 0u);
    uint32_t len = (j + 1 < R ? RF[j + 1] : Ftot) - RF[j];
    uint8_t *h = buf + 8 + 8 * j + 2 * (size_t)RF[j];
    *(uint16_t *)(h + 0) = (uint16_t)off;
    *(uint16_t *)(h + 2) = (uint16_t)(off >> 16);
    *(uint16_t *)(h + 4) = (uint16_t)len;
    *(uint16_t *)(h + 6) = (uint16_t)(len >> 16);
}

// Lift: value v belongs to run j with cumF[j] <= v < cumF[j+1] (binary search);
// it sits at byte 16 + 8 j + 2 v and lands at start[j] + (v - cumF[j]).
__global__ __launch_bounds__(kSB) void sp_expand(float *g, const uint8_t *buf, const uint64_t *start,
                                                 const uint64_t *cumF, size_t R, size_t F) {
    size_t v = (size_t)blockIdx.x * kSB + threadIdx.x;
    if (v >= F) return;
    size_t lo = 0, hi = R;  // largest j with cumF[j] <= v
    while (hi - lo > 1) {
        size_t mid = (lo + hi) / 2;
        if (cumF[mid] <= v) lo = mid; else hi = mid;
    }
    const uint8_t *p = buf + 16 + 8 * lo + 2 * v;
    uint16_t h = (uint16_t)(p[0] | (uint16_t)p[1] << 8);
    g[start[lo] + (v - cumF[lo])] = from_f16_sp(h);
}

// worker_ring.rs:128-131 (scatter: zero what was sent, |g| >= t) and
// :183-187 (gather: keep only |g| >= t)
__global__ __launch_bounds__(kSB) void sp_mask(float *g, size_t n, float t, int zero_kept) {
    size_t i = (size_t)blockIdx.x * kSB + threadIdx.x;
    if (i >= n) return;
    float x = g[i];
    if (zero_kept) {
        if (kept(x, t)) g[i] = 0.0f;        // scatter: the sent values leave the residual
    } else {
        if (fabsf(x) < t) g[i] = 0.0f;      // gather: only the sent values stay in grad
    }
}

}  // namespace

extern "C" {

size_t ono_sparse_max_bytes(size_t n) { return 8 + 10 * ((n + 1) / 2) + 2 * n; }

int ono_sparse_drop(uint8_t *buf, size_t cap, size_t *nbytes, const float *g, size_t n, float threshold,
                    void *stream) {
    if (!nbytes || (n && !g) || !buf) return set_error(ONO_E_ARG, "NULL argument");
    if (n >= 0xFFFFFFFFull) return set_error(ONO_E_ARG, "sparse codec offsets are u32 (protocol.rs:13-19)");
    if (cap < 8) return set_error(ONO_E_SIZE, "buffer too small");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const size_t ntiles = n ? (n + kTile - 1) / kTile : 0;
    const size_t maxruns = (n + 1) / 2 + 1;
    uint32_t *tiles = nullptr, *runs = nullptr;
    uint64_t *totals = nullptr;
    ONO_HIP(hipMallocAsync((void **)&tiles, (2 * ntiles + 2) * sizeof(uint32_t), s));
    ONO_HIP(hipMallocAsync((void **)&runs, 2 * maxruns * sizeof(uint32_t), s));
    ONO_HIP(hipMallocAsync((void **)&totals, 2 * sizeof(uint64_t), s));
    ONO_HIP(hipMemsetAsync(totals, 0, 2 * sizeof(uint64_t), s));
    uint32_t *tileF = tiles, *tileS = tiles + ntiles + 1, *RU = runs, *RF = runs + maxruns;
    int rc = ONO_OK;
    uint64_t tot[2] = {0, 0};
    if (ntiles) {
        hipLaunchKernelGGL(sp_count, dim3((unsigned)ntiles), dim3(kSB), 0, s, g, n, threshold, tileF, tileS);
        hipLaunchKernelGGL(sp_scan_tiles, dim3(1), dim3(kSB), 0, s, tileF, tileS, ntiles, totals);
    }
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(tot, totals, sizeof tot, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    const size_t F = tot[0], R = tot[1], bytes = 8 + 8 * R + 2 * F;
    if (e != hipSuccess) {
        rc = hip_error(e, "sparse count", __FILE__, __LINE__);
    } else if (bytes > cap) {
        rc = set_error(ONO_E_SIZE, "sparse encoding needs %zu bytes, buffer holds %zu", bytes, cap);
    } else {
        if (ntiles)
            hipLaunchKernelGGL(sp_write, dim3((unsigned)ntiles), dim3(kSB), 0, s, g, n, threshold, tileF, tileS, buf,
                               RU, RF);
        hipLaunchKernelGGL(sp_headers, dim3((unsigned)((R + kSB) / kSB)), dim3(kSB), 0, s, RU, RF, R, (uint32_t)F,
                           (uint64_t)n, buf);
        e = hipGetLastError();
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = hip_error(e, "sparse write", __FILE__, __LINE__);
        *nbytes = bytes;
    }
    (void)hipFreeAsync(tiles, s);
    (void)hipFreeAsync(runs, s);
    (void)hipFreeAsync(totals, s);
    return rc;
}

int ono_sparse_lift(float *g, size_t cap, size_t *out_len, const uint8_t *buf, size_t nbytes, void *stream) {
    if (!out_len || (!buf && nbytes)) return set_error(ONO_E_ARG, "NULL argument");
    // protocol.rs:96-144, the sequential parse of the record headers (host)
    if (nbytes < 8) return set_error(ONO_E_PROTO, "The given sparse buffer is smaller than TOTAL_LEN_SIZE");
    uint64_t total = 0;
    for (int q = 0; q < 8; q++) total |= (uint64_t)buf[q] << (8 * q);
    if (total > cap) return set_error(ONO_E_SIZE, "sparse gradient of %llu values, buffer of %zu",
                                      (unsigned long long)total, cap);
    std::vector<uint64_t> start, cumF;
    size_t gi = 0, bi = 8, F = 0;
    while (bi < nbytes) {
        if (nbytes - bi < 4) return set_error(ONO_E_PROTO, "Missing index bytes at grad lift");
        uint32_t off = buf[bi] | buf[bi + 1] << 8 | buf[bi + 2] << 16 | (uint32_t)buf[bi + 3] << 24;
        gi += off;
        bi += 4;
        if (nbytes - bi < 4) return set_error(ONO_E_PROTO, "Missing chunk length bytes at grad lift");
        uint32_t len = buf[bi] | buf[bi + 1] << 8 | buf[bi + 2] << 16 | (uint32_t)buf[bi + 3] << 24;
        bi += 4;
        if (gi > total || total - gi < len) return set_error(ONO_E_PROTO, "Gradient chunk exceeds target vector bounds");
        if ((nbytes - bi) / 2 < len) return set_error(ONO_E_PROTO, "Truncated float data");
        start.push_back(gi);  // zero-length records stay in the table: the record
        cumF.push_back(F);    // index must remain the header index (byte math in sp_expand)
        F += len;
        bi += 2 * (size_t)len;
        gi += len;
    }
    *out_len = total;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (total) ONO_HIP(hipMemsetAsync(g, 0, total * sizeof(float), s));  // grad.fill(0); resize(total, 0)
    if (F == 0) return ONO_OK;
    const size_t R = start.size();
    uint8_t *dbuf = nullptr;
    uint64_t *dtab = nullptr;
    ONO_HIP(hipMallocAsync((void **)&dbuf, nbytes, s));
    ONO_HIP(hipMallocAsync((void **)&dtab, 2 * R * sizeof(uint64_t), s));
    ONO_HIP(hipMemcpyAsync(dbuf, buf, nbytes, hipMemcpyHostToDevice, s));
    ONO_HIP(hipMemcpyAsync(dtab, start.data(), R * sizeof(uint64_t), hipMemcpyHostToDevice, s));
    ONO_HIP(hipMemcpyAsync(dtab + R, cumF.data(), R * sizeof(uint64_t), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(sp_expand, dim3((unsigned)((F + kSB - 1) / kSB)), dim3(kSB), 0, s, g, dbuf, dtab, dtab + R, R, F);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(s);  // the host vectors and buffer are released on return
    (void)hipFreeAsync(dbuf, s);
    (void)hipFreeAsync(dtab, s);
    if (e != hipSuccess) return hip_error(e, "sparse lift", __FILE__, __LINE__);
    return ONO_OK;
}

int ono_sparse_mask(float *g, size_t n, float threshold, int zero_kept, void *stream) {
    if (n && !g) return set_error(ONO_E_ARG, "NULL argument");
    if (!n) return ONO_OK;
    hipLaunchKernelGGL(sp_mask, dim3((unsigned)((n + kSB - 1) / kSB)), dim3(kSB), 0,
                       reinterpret_cast<hipStream_t>(stream), g, n, threshold, zero_kept);
    ONO_HIP(hipGetLastError());
    return ONO_OK;
}

}  // extern "C"
