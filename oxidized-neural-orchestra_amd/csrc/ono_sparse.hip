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
// wave shuffles + LDS; values written, run starts record U and F) -> headers,
// back to back on the stream (the totals stay on the device; the host reads
// them once, at the end, for the wire length).
// Decoding is a parallel parse on the device (the record stream is a linked
// list: each header gives the next one's position), see "Lift" below; the
// reference's sequential parse on the host remains as the exact fallback and
// the source of the reference's error messages.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <atomic>
#include <mutex>
#include <vector>

#include "ono_internal.h"

using namespace ono;

namespace {

constexpr int kSB = 256;             // threads per block (4 waves)
constexpr int kEPT = 8;              // elements per thread
constexpr int kTile = kSB * kEPT;    // 2048 elements per tile

// half 2.7.1 conversions = the gfx950 cvt instructions, NaN rules included (ono_kernels.hip to_f16)
__device__ __forceinline__ uint16_t to_f16_sp(float x) { return __builtin_bit_cast(uint16_t, (_Float16)x); }
__device__ __forceinline__ float from_f16_sp(uint16_t b) { return (float)__builtin_bit_cast(_Float16, b); }

// g.abs() >= threshold (NaN never kept, as in Rust)
__device__ __forceinline__ bool kept(float x, float t) { return fabsf(x) >= t; }

// Flags of a thread's kEPT elements: bit e = kept, plus whether each starts a run.
// NTL: the count pass loads g plainly so the 64 MiB bucket stays in the Infinity
// Cache for the write pass, whose nt loads are its last use (70 -> 66 us).
// The kEPT = 8 values come in as two 16-B loads (g is 16-B aligned on the fast
// path; `vec` = false uses scalar loads); whether the element before the
// thread's first one is kept comes from the neighbouring lane (a shuffle), and
// only lane 0 of each wave reads it from memory.
struct Bits {
    uint32_t keep = 0, start = 0;
};
typedef float f4s __attribute__((ext_vector_type(4)));
template <bool NTL>
__device__ __forceinline__ Bits thread_bits(const float *g, size_t n, float t, size_t base, bool vec,
                                            float (&x)[kEPT]) {
    Bits b;
    if (vec && base + kEPT <= n) {
        f4s a, c;
        if constexpr (NTL) {
            a = __builtin_nontemporal_load((const f4s *)(g + base));
            c = __builtin_nontemporal_load((const f4s *)(g + base + 4));
        } else {
            a = *(const f4s *)(g + base);
            c = *(const f4s *)(g + base + 4);
        }
        x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = c.x; x[5] = c.y; x[6] = c.z; x[7] = c.w;
    } else {
#pragma unroll
        for (int e = 0; e < kEPT; e++) x[e] = base + e < n ? g[base + e] : 0.0f;
    }
#pragma unroll
    for (int e = 0; e < kEPT; e++)
        if (base + e < n && kept(x[e], t)) b.keep |= 1u << e;
    // kept(element base-1): the previous lane's last flag; lane 0 loads it
    const int lane = threadIdx.x & 63;
    uint32_t last = (b.keep >> (kEPT - 1)) & 1u;
    uint32_t prev = __shfl_up(last, 1, 64);
    if (lane == 0) prev = base > 0 && base - 1 < n ? (kept(g[base - 1], t) ? 1u : 0u) : 0u;
    b.start = b.keep & ~((b.keep << 1) | prev);
    return b;
}

// Exclusive block-wide scan of (a, b) pairs: wave-level shuffles (64 lanes),
// then the 4 wave totals through LDS.  Returns the block totals too.
template <int NT = kSB>
__device__ __forceinline__ void block_scan2(uint32_t a, uint32_t b, uint32_t &ea, uint32_t &eb, uint32_t &ta,
                                            uint32_t &tb) {
    __shared__ uint32_t wa[NT / 64], wb[NT / 64];
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
    for (int w = 0; w < NT / 64; w++) {
        if (w < wave) { pa += wa[w]; pb += wb[w]; }
        ta += wa[w];
        tb += wb[w];
    }
    ea = pa + ia - a;
    eb = pb + ib - b;
}

// The same scan for the per-thread counts of the count / write passes, which
// are small (kept <= 8, run starts <= 4 of a thread's 8 elements): each bit
// plane of the count is one wave ballot, and mbcnt counts the set bits below
// the lane — an exact exclusive wave scan with no cross-lane data movement
// (7 ballots instead of 12 ds_bpermute round trips of the shuffle ladder).
__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
template <int BITS>
__device__ __forceinline__ void wave_scan_small(uint32_t v, uint32_t &ex, uint32_t &tot) {
    ex = 0;
    tot = 0;
#pragma unroll
    for (int b = 0; b < BITS; b++) {
        const uint64_t m = __ballot((v >> b) & 1u);
        ex += mbcnt64(m) << b;
        tot += (uint32_t)__popcll(m) << b;
    }
}
__device__ __forceinline__ void block_scan_counts(uint32_t a, uint32_t b, uint32_t &ea, uint32_t &eb, uint32_t &ta,
                                                  uint32_t &tb) {
    __shared__ uint32_t wa[kSB / 64], wb[kSB / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t xa, xb, sa, sb;
    wave_scan_small<4>(a, xa, sa);  // a <= kEPT = 8
    wave_scan_small<3>(b, xb, sb);  // b <= kEPT / 2 = 4
    if (lane == 0) { wa[wave] = sa; wb[wave] = sb; }
    __syncthreads();
    uint32_t pa = 0, pb = 0;
    ta = 0;
    tb = 0;
#pragma unroll
    for (int w = 0; w < kSB / 64; w++) {
        if (w < wave) { pa += wa[w]; pb += wb[w]; }
        ta += wa[w];
        tb += wb[w];
    }
    ea = pa + xa;
    eb = pb + xb;
}
static_assert(kEPT == 8, "block_scan_counts sizes its bit planes for 8 elements per thread");

__global__ __launch_bounds__(kSB) void sp_count(const float *g, size_t n, float t, uint32_t *tileF, uint32_t *tileS,
                                                bool vec) {
    float x[kEPT];
    Bits b = thread_bits<false>(g, n, t, (size_t)blockIdx.x * kTile + (size_t)threadIdx.x * kEPT, vec, x);
    uint32_t ea, eb, ta, tb;
    block_scan_counts(__popc(b.keep), __popc(b.start), ea, eb, ta, tb);
    if (threadIdx.x == 0) { tileF[blockIdx.x] = ta; tileS[blockIdx.x] = tb; }
}

// Exclusive scan of the tile counts in place, one block of kScanT threads,
// in chunks of kScanT x kScanPer tiles staged through LDS: coalesced global
// loads into LDS, each thread scans its kScanPer contiguous tiles there, one
// block-wide scan of the per-thread sums, coalesced stores back.
// totals[0] = kept values, totals[1] = runs.
constexpr int kScanT = 1024, kScanPer = 8, kScanChunk = kScanT * kScanPer;
__global__ __launch_bounds__(kScanT) void sp_scan_tiles(uint32_t *tileF, uint32_t *tileS, size_t ntiles,
                                                        uint64_t *totals) {
    __shared__ uint32_t lf[kScanChunk], ls[kScanChunk];
    __shared__ uint32_t carry[2];
    if (threadIdx.x == 0) { carry[0] = 0; carry[1] = 0; }
    for (size_t c0 = 0; c0 < ntiles; c0 += kScanChunk) {
        const size_t m = ntiles - c0 < (size_t)kScanChunk ? ntiles - c0 : (size_t)kScanChunk;
        for (size_t i = threadIdx.x; i < kScanChunk; i += kScanT) {
            lf[i] = i < m ? tileF[c0 + i] : 0u;
            ls[i] = i < m ? tileS[c0 + i] : 0u;
        }
        __syncthreads();
        const int lo = threadIdx.x * kScanPer;
        uint32_t sf = 0, ss = 0;
#pragma unroll
        for (int k = 0; k < kScanPer; k++) { sf += lf[lo + k]; ss += ls[lo + k]; }
        uint32_t ef, es, tf, ts;
        block_scan2<kScanT>(sf, ss, ef, es, tf, ts);
        ef += carry[0];
        es += carry[1];
#pragma unroll
        for (int k = 0; k < kScanPer; k++) {
            const uint32_t a = lf[lo + k], b = ls[lo + k];
            lf[lo + k] = ef;
            ls[lo + k] = es;
            ef += a;
            es += b;
        }
        __syncthreads();
        for (size_t i = threadIdx.x; i < m; i += kScanT) {
            tileF[c0 + i] = lf[i];
            tileS[c0 + i] = ls[i];
        }
        if (threadIdx.x == 0) { carry[0] += tf; carry[1] += ts; }
        __syncthreads();
    }
    if (threadIdx.x == 0) { totals[0] = carry[0]; totals[1] = carry[1]; }
}

// A tile's output is one contiguous byte range of the wire, from
// 8 + 8 S0 + 2 F0 to 8 + 8 (S0 + runs) + 2 (F0 + kept) (S0, F0: the tile's
// prefix).  Values are placed in an LDS image of that range first, then the
// block writes the range out with consecutive 2-byte stores (coalesced,
// instead of one scattered store per kept value).  Header slots in the image
// are left as they are; sp_headers writes them afterwards.
constexpr int kStageU16 = (8 * (kTile / 2 + 1) + 2 * kTile) / 2;  // worst case: alternating kept/unkept
__global__ __launch_bounds__(kSB) void sp_write(const float *g, size_t n, float t, const uint32_t *tileF,
                                                const uint32_t *tileS, uint8_t *buf, uint32_t *RU, uint32_t *RF,
                                                bool vec) {
    __shared__ uint16_t stage[kStageU16];
    __shared__ uint32_t su[kTile / 2 + 1], sf[kTile / 2 + 1];  // the tile's run table rows
    const size_t base = (size_t)blockIdx.x * kTile + (size_t)threadIdx.x * kEPT;
    float x[kEPT];  // the values stay in registers from the flag pass (g is read once here)
    Bits b = thread_bits<true>(g, n, t, base, vec, x);
    uint32_t ea, eb, ta, tb;
    block_scan_counts(__popc(b.keep), __popc(b.start), ea, eb, ta, tb);
    const uint32_t F0 = tileF[blockIdx.x], S0 = tileS[blockIdx.x];
    uint32_t f = ea, sl = eb;  // this thread's kept values / runs before it, within the tile
    if (b.keep) {
#pragma unroll
        for (int e = 0; e < kEPT; e++) {
            if (!(b.keep >> e & 1u)) continue;
            if (b.start >> e & 1u) {
                const size_t i = base + e;
                su[sl] = (uint32_t)(i - (F0 + f));  // U(s_j): unkept values before the run
                sf[sl] = F0 + f;                    // F(s_j)
                sl++;
            }
            stage[4 * sl + f] = to_f16_sp(x[e]);  // byte 8 sl + 2 f of the tile's range
            f++;
        }
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < tb; k += kSB) {  // run table rows, coalesced
        RU[S0 + k] = su[k];
        RF[S0 + k] = sf[k];
    }
    // the range, 4 bytes per store where aligned (it starts 2-B aligned)
    const uint32_t nu16 = 4 * tb + ta;  // the range's length in 2-byte units
    uint16_t *dst = (uint16_t *)(buf + 8 + 8 * (size_t)S0 + 2 * (size_t)F0);
    const uint32_t h = (uint32_t)(((uintptr_t)dst >> 1) & 1u) < nu16 ? (uint32_t)(((uintptr_t)dst >> 1) & 1u) : nu16;
    if (threadIdx.x == 0 && h) dst[0] = stage[0];
    const uint32_t npair = (nu16 - h) / 2;
    uint32_t *d32 = (uint32_t *)(dst + h);
    for (uint32_t k = threadIdx.x; k < npair; k += kSB)
        d32[k] = (uint32_t)stage[h + 2 * k] | (uint32_t)stage[h + 2 * k + 1] << 16;
    if (threadIdx.x == 0 && h + 2 * npair < nu16) dst[nu16 - 1] = stage[nu16 - 1];
}

// R and the kept total come from the device totals (no host round trip); a
// grid-stride loop sized for the worst case idles past R.
__global__ __launch_bounds__(kSB) void sp_headers(const uint32_t *RU, const uint32_t *RF, const uint64_t *totals,
                                                  uint64_t total_len, uint8_t *buf, uint64_t *host_tot) {
    const size_t R = totals[1];
    const uint32_t Ftot = (uint32_t)totals[0];
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // u64 LE total length, as four 2-byte stores (buf is 2-B aligned)
        for (int q = 0; q < 4; q++) *(uint16_t *)(buf + 2 * q) = (uint16_t)(total_len >> (16 * q));
        host_tot[0] = Ftot;  // the wire length's terms, for the caller (host-mapped)
        host_tot[1] = R;
    }
    for (size_t j = (size_t)blockIdx.x * kSB + threadIdx.x; j < R; j += (size_t)gridDim.x * kSB) {
        uint32_t off = RU[j] - (j ? RU[j - 1] : 0u);
        uint32_t len = (j + 1 < R ? RF[j + 1] : Ftot) - RF[j];
        uint8_t *h = buf + 8 + 8 * j + 2 * (size_t)RF[j];
        *(uint16_t *)(h + 0) = (uint16_t)off;
        *(uint16_t *)(h + 2) = (uint16_t)(off >> 16);
        *(uint16_t *)(h + 4) = (uint16_t)len;
        *(uint16_t *)(h + 6) = (uint16_t)(len >> 16);
    }
}

// Fallback lift (after a host parse): value v belongs to run j with
// cumF[j] <= v < cumF[j+1] (binary search);
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

// ---------------------------------------------------------------- lift ----
// The record stream is cut into segments of kSeg bytes.  sl_starts picks, per
// segment, the first 2-byte position whose next kLook records are all
// plausible (a speculative record start; segment 0 starts at the true head,
// byte 8).  sl_walk follows the records from each start until it lands on a
// later segment's start (marking it reached) or the end of the stream.  The
// speculation is checked, not trusted: the walks are exactly the sequential
// parse iff every speculative start was reached and no walk failed (records
// form a successor chain, so a walk that lands on a start has joined the true
// chain there; the earliest start off the chain can only be reached from the
// chain, so it stays unreached).  Otherwise `bad` is raised and the host
// parses sequentially — also how malformed input gets the reference's error
// messages.  Each walk's sum of (offset + length) is scanned (block-wide in
// sl_walk, across blocks by sp_scan_tiles) to give the element index its
// records start at; sl_place walks again and writes the values of short runs
// itself, and queues runs longer than kShort for sl_long (one workgroup per
// run).
constexpr int kSeg = 128, kLook = 4, kShort = 16;
constexpr uint32_t kNone = 0xFFFFFFFFu;

__device__ __forceinline__ uint32_t ld32(const uint8_t *b, size_t p) {  // p even, b 2-B aligned
    const uint16_t *h = (const uint16_t *)(b + p);
    return (uint32_t)h[0] | (uint32_t)h[1] << 16;
}
__device__ __forceinline__ uint16_t ld16(const uint8_t *b, size_t p) { return *(const uint16_t *)(b + p); }

// g[0, total) = 0 (grad.fill(0); resize(total, 0)) with total read from the
// stream's first 8 bytes on the device, so the host need not wait for it.
// tot[0] = total; flags: [0] bad, [1] queued long runs, [2] total > cap (then
// nothing is written and every later kernel stands down through flags[0]).
__global__ __launch_bounds__(kSB) void sl_zero(float *g, const uint8_t *b, size_t cap, int vec, uint64_t *tot,
                                               uint32_t *flags, uint64_t *host_word) {
    uint64_t total = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) total |= (uint64_t)ld16(b, 2 * q) << (16 * q);
    const size_t t = (size_t)blockIdx.x * kSB + threadIdx.x, stride = (size_t)gridDim.x * kSB;
    if (t == 0) {
        tot[0] = total;
        host_word[1] = total;
        flags[0] = total > cap ? 1u : 0u;
        flags[1] = 0;
        flags[2] = total > cap ? 1u : 0u;
    }
    if (total > cap) return;
    if (vec) {
        const f4s z = {0.0f, 0.0f, 0.0f, 0.0f};
        for (size_t i = t; i < total / 4; i += stride) *(f4s *)(g + 4 * i) = z;
        for (size_t i = 4 * (total / 4) + t; i < total; i += stride) g[i] = 0.0f;
    } else {
        for (size_t i = t; i < total; i += stride) g[i] = 0.0f;
    }
}

__global__ __launch_bounds__(kSB) void sl_starts(const uint8_t *b, size_t nbytes, const uint64_t *tot, size_t S,
                                                 uint32_t *p0, uint32_t *reached) {
    const size_t t = (size_t)blockIdx.x * kSB + threadIdx.x;
    if (t >= S) return;
    const uint64_t total = tot[0];
    reached[t] = 0;
    if (t == 0) { p0[0] = 8; return; }
    const size_t lo = 8 + t * kSeg, hi = lo + kSeg < nbytes ? lo + kSeg : nbytes;
    for (size_t p = lo; p < hi; p += 2) {
        size_t q = p;
        uint64_t acc = 0;
        bool ok = true;
        for (int k = 0; k < kLook && q != nbytes; k++) {
            if (nbytes - q < 8) { ok = false; break; }
            const uint32_t off = ld32(b, q), len = ld32(b, q + 4);
            // A start whose records run past the stream is no start; nor is one
            // with a run of >= 2^16 values: a header read 2 B off its true
            // position takes a half of the run length as the high half of its
            // own (so >= 2^16), and such a jump lands on a true header about one
            // time in five, after which every look-ahead record is valid.  Runs
            // are maximal in grad_drop's output, so a record after the first is
            // >= 1 value past the previous run: offset 0 is no start either
            // (zero-filled payload reads as offset 0).  A true start refused
            // here only leaves its segment to the previous walk.
            if (off == 0 || len >= 0x10000u || (nbytes - q - 8) / 2 < len) { ok = false; break; }
            acc += (uint64_t)off + len;
            if (acc > total) { ok = false; break; }
            q += 8 + 2 * (size_t)len;
        }
        if (ok) { p0[t] = (uint32_t)p; return; }
    }
    p0[t] = kNone;
}

// per segment: gsum[t] = sum of (offset + length) over its records;
// per block: bsum[block] = the block's total (scanned afterwards)
__global__ __launch_bounds__(kSB) void sl_walk(const uint8_t *b, size_t nbytes, const uint64_t *tot, size_t S,
                                               const uint32_t *p0, uint32_t *reached, uint32_t *gsum, uint32_t *bsum,
                                               uint32_t *bscratch, uint32_t *flags) {
    const size_t t = (size_t)blockIdx.x * kSB + threadIdx.x;
    const uint64_t total = tot[0];
    uint64_t sum = 0;
    if (t < S && p0[t] != kNone) {
        size_t pos = p0[t];
        const size_t segend = 8 + (t + 1) * kSeg;
        for (;;) {
            if (pos == nbytes) break;  // the end of the stream
            if (pos >= segend) {
                const size_t u = (pos - 8) / kSeg;
                const uint32_t pu = u < S ? p0[u] : kNone;
                if (pu != kNone && pos == pu) { reached[u] = 1; break; }
                if (pu != kNone && pos > pu) { flags[0] = 1; break; }  // stepped over a start: not a record
            }
            if (nbytes - pos < 8) { flags[0] = 1; break; }
            const uint32_t off = ld32(b, pos), len = ld32(b, pos + 4);
            if ((nbytes - pos - 8) / 2 < len) { flags[0] = 1; break; }
            sum += (uint64_t)off + len;
            if (sum > total) { flags[0] = 1; break; }
            pos += 8 + 2 * (size_t)len;
        }
    }
    if (t < S) gsum[t] = (uint32_t)sum;
    uint32_t ea, eb, ta, tb;
    block_scan2((uint32_t)sum, 0u, ea, eb, ta, tb);
    if (threadIdx.x == 0) { bsum[blockIdx.x] = ta; bscratch[blockIdx.x] = 0; }
}

__device__ __forceinline__ void put_run(float *g, const uint8_t *b, uint32_t gi, size_t vpos, uint32_t len,
                                        uint32_t *longq, uint32_t qcap, uint32_t *flags) {
    if (len <= (uint32_t)kShort) {
        for (uint32_t i = 0; i < len; i++) g[gi + i] = from_f16_sp(ld16(b, vpos + 2 * i));
    } else {
        const uint32_t k = atomicAdd(&flags[1], 1u);
        if (k >= qcap) { flags[0] = 1; return; }  // only off-chain walks can overfill it
        longq[3 * k] = gi;
        longq[3 * k + 1] = (uint32_t)vpos;
        longq[3 * k + 2] = len;
    }
}

// bsum: exclusive scan over blocks (sp_scan_tiles)
__global__ __launch_bounds__(kSB) void sl_place(float *g, const uint8_t *b, size_t nbytes, const uint64_t *tot,
                                                size_t S, const uint32_t *p0, const uint32_t *reached,
                                                const uint32_t *gsum, const uint32_t *bsum, uint32_t *longq,
                                                uint32_t qcap, uint32_t *flags) {
    const size_t t = (size_t)blockIdx.x * kSB + threadIdx.x;
    const uint64_t total = tot[0];
    const uint32_t mine = t < S ? gsum[t] : 0u;
    uint32_t ea, eb, ta, tb;
    block_scan2(mine, 0u, ea, eb, ta, tb);
    if (flags[0] || t >= S || p0[t] == kNone) return;  // a failed walk: nothing to place
    if (t > 0 && !reached[t]) { flags[0] = 1; return; }  // a speculative start off the chain
    // the same records sl_walk visited (it checked every one against the
    // stream's bounds), stopping where it stopped
    uint64_t gi = (uint64_t)bsum[blockIdx.x] + ea;
    size_t pos = p0[t];
    const size_t segend = 8 + (t + 1) * kSeg;
    for (;;) {
        if (pos == nbytes) break;
        if (pos >= segend) {
            const size_t u = (pos - 8) / kSeg;
            const uint32_t pu = u < S ? p0[u] : kNone;
            if (pu != kNone && pos >= pu) break;
        }
        const uint32_t off = ld32(b, pos), len = ld32(b, pos + 4);
        gi += off;
        if (gi > total || total - gi < len) { flags[0] = 1; return; }  // protocol.rs:127-129 (host reports it)
        put_run(g, b, (uint32_t)gi, pos + 8, len, longq, qcap, flags);
        gi += len;
        pos += 8 + 2 * (size_t)len;
    }
}

// runs longer than kShort: one workgroup per queued run
__global__ __launch_bounds__(kSB) void sl_long(float *g, const uint8_t *b, const uint32_t *longq,
                                               const uint32_t *flags, uint64_t *host_word) {
    const uint32_t bad = flags[0];
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // every kernel that raises them has run
        host_word[0] = bad;
        host_word[2] = flags[2];
    }
    if (bad) return;
    const uint32_t nq = flags[1];  // <= qcap when bad is clear
    for (uint32_t k = blockIdx.x; k < nq; k += gridDim.x) {
        const uint32_t gi = longq[3 * k], len = longq[3 * k + 2];
        const size_t vpos = longq[3 * k + 1];
        for (uint32_t i = threadIdx.x; i < len; i += kSB) g[gi + i] = from_f16_sp(ld16(b, vpos + 2 * i));
    }
}

// the totals into the host-mapped words (the exact-size path of a small buffer)
__global__ void sp_totals_out(const uint64_t *totals, uint64_t *host_tot) {
    host_tot[0] = totals[0];
    host_tot[1] = totals[1];
}

// Scratch of the encoder (tile counts, run table, device totals, two host-
// mapped words for the result), kept per device and grown on demand: the
// stream-ordered allocations it replaces cost more than the kernels at 64 MiB.
struct Scratch {
    size_t tiles_cap = 0, runs_cap = 0;
    uint32_t *tiles = nullptr, *runs = nullptr;
    uint64_t *totals_dev = nullptr, *host_tot = nullptr, *host_tot_dev = nullptr;
};
std::mutex g_scratch_mu;
Scratch g_scratch[64];

int scratch_for(size_t ntiles, size_t maxruns, Scratch **out) {
    int dev = 0;
    ONO_HIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) return set_error(ONO_E_ARG, "device %d", dev);
    Scratch &sc = g_scratch[dev];
    if (!sc.totals_dev) {
        ONO_HIP(hipMalloc((void **)&sc.totals_dev, 2 * sizeof(uint64_t)));
        ONO_HIP(hipHostMalloc((void **)&sc.host_tot, 2 * sizeof(uint64_t), hipHostMallocMapped | hipHostMallocCoherent));
        ONO_HIP(hipHostGetDevicePointer((void **)&sc.host_tot_dev, sc.host_tot, 0));
    }
    if (2 * ntiles + 2 > sc.tiles_cap) {
        (void)hipFree(sc.tiles);
        sc.tiles = nullptr;
        sc.tiles_cap = 0;
        ONO_HIP(hipMalloc((void **)&sc.tiles, (2 * ntiles + 2) * sizeof(uint32_t)));
        sc.tiles_cap = 2 * ntiles + 2;
    }
    if (2 * maxruns > sc.runs_cap) {
        (void)hipFree(sc.runs);
        sc.runs = nullptr;
        sc.runs_cap = 0;
        ONO_HIP(hipMalloc((void **)&sc.runs, 2 * maxruns * sizeof(uint32_t)));
        sc.runs_cap = 2 * maxruns;
    }
    *out = &sc;
    return ONO_OK;
}

struct LiftScratch {
    size_t seg_cap = 0, rec_cap = 0, buf_cap = 0;
    uint32_t *seg = nullptr, *rec = nullptr, *flags = nullptr;
    uint8_t *buf = nullptr;
    uint64_t *totals = nullptr, *host_word = nullptr, *host_word_dev = nullptr;
};
LiftScratch g_lift[64];
std::atomic<size_t> g_lift_fallbacks{0};

template <class T> int grow(T **p, size_t &cap, size_t want) {
    if (want <= cap) return ONO_OK;
    (void)hipFree(*p);
    *p = nullptr;
    cap = 0;
    ONO_HIP(hipMalloc((void **)p, want * sizeof(T)));
    cap = want;
    return ONO_OK;
}

// The reference's sequential parse (protocol.rs:96-144) of a host copy of the
// stream: the run table, or the reference's error.
int lift_parse_host(const uint8_t *buf, size_t nbytes, uint64_t total, std::vector<uint64_t> &start,
                    std::vector<uint64_t> &cumF) {
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
    return ONO_OK;
}

// Sequential fallback: host parse, tables up, expand (the original lift).
int lift_host_path(float *g, const uint8_t *hbuf, const uint8_t *dbuf, size_t nbytes, uint64_t total,
                   hipStream_t s) {
    std::vector<uint64_t> start, cumF;
    int rc = lift_parse_host(hbuf, nbytes, total, start, cumF);
    if (rc) return rc;
    const size_t R = start.size(), F = (nbytes - 8 - 8 * R) / 2;
    if (F == 0) return ONO_OK;
    uint64_t *dtab = nullptr;
    ONO_HIP(hipMallocAsync((void **)&dtab, 2 * R * sizeof(uint64_t), s));
    hipError_t e = hipMemcpyAsync(dtab, start.data(), R * sizeof(uint64_t), hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(dtab + R, cumF.data(), R * sizeof(uint64_t), hipMemcpyHostToDevice, s);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(sp_expand, dim3((unsigned)((F + kSB - 1) / kSB)), dim3(kSB), 0, s, g, dbuf, dtab, dtab + R,
                           R, F);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipStreamSynchronize(s);  // the host vectors are released on return
    (void)hipFreeAsync(dtab, s);  // on every path
    if (e != hipSuccess) return hip_error(e, "sparse lift", __FILE__, __LINE__);
    return ONO_OK;
}

// Device lift of a device-resident stream, one host wait in all.  hbuf: a
// host copy when the caller has one (the fallback then needs no download).
int lift_device(float *g, size_t cap, size_t *out_len, const uint8_t *dbuf, const uint8_t *hbuf, size_t nbytes,
                hipStream_t s) {
    std::vector<uint8_t> copy;
    auto host_bytes = [&]() -> const uint8_t * {
        if (hbuf) return hbuf;
        copy.resize(nbytes);
        if (hipMemcpyAsync(copy.data(), dbuf, nbytes, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return nullptr;
        return copy.data();
    };
    auto size_error = [&](uint64_t total) {
        return set_error(ONO_E_SIZE, "sparse gradient of %llu values, buffer of %zu", (unsigned long long)total, cap);
    };
    // u32 record positions, element indices and counts: streams under 4 GiB,
    // gradients under 2^32 values; anything larger (or an odd stream address)
    // parses on the host
    if (nbytes >= 0xFFFFFFF0ull || cap >= 0xFFFFFFFFull || ((uintptr_t)dbuf & 1)) {
        const uint8_t *hb = host_bytes();
        if (!hb) return set_error(ONO_E_HIP, "sparse lift: download of the stream failed");
        uint64_t total = 0;
        for (int q = 0; q < 8; q++) total |= (uint64_t)hb[q] << (8 * q);
        if (total > cap) return size_error(total);
        *out_len = total;
        if (total) ONO_HIP(hipMemsetAsync(g, 0, total * sizeof(float), s));
        return lift_host_path(g, hb, dbuf, nbytes, total, s);
    }
    int dev = 0;
    ONO_HIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) return set_error(ONO_E_ARG, "device %d", dev);
    LiftScratch &L = g_lift[dev];
    const size_t S = (nbytes - 8 + kSeg - 1) / kSeg, nblk = S ? (S + kSB - 1) / kSB : 0;
    const size_t qcap = (nbytes - 8) / (8 + 2 * (kShort + 1)) + 1;  // runs longer than kShort fit this many
    if (!L.flags) {
        ONO_HIP(hipMalloc((void **)&L.flags, 4 * sizeof(uint32_t)));
        ONO_HIP(hipHostMalloc((void **)&L.host_word, 4 * sizeof(uint64_t), hipHostMallocMapped | hipHostMallocCoherent));
        ONO_HIP(hipHostGetDevicePointer((void **)&L.host_word_dev, L.host_word, 0));
        ONO_HIP(hipMalloc((void **)&L.totals, 4 * sizeof(uint64_t)));  // [0] total, [1..2] scan totals
    }
    int rc = grow(&L.seg, L.seg_cap, 3 * S + 2 * nblk + 4);
    if (!rc) rc = grow(&L.rec, L.rec_cap, 3 * qcap);
    if (rc) return rc;
    uint32_t *p0 = L.seg, *reached = L.seg + S, *gsum = L.seg + 2 * S, *bsum = L.seg + 3 * S,
             *bscr = L.seg + 3 * S + nblk;
    volatile uint64_t *word = L.host_word;
    word[0] = 1;
    word[1] = word[2] = 0;
    const int vec = ((uintptr_t)g & 15) == 0;
    const unsigned zb = (unsigned)std::max<size_t>(1, std::min<size_t>(8192, (cap / 4 + kSB - 1) / kSB));
    hipLaunchKernelGGL(sl_zero, dim3(zb), dim3(kSB), 0, s, g, dbuf, cap, vec, L.totals, L.flags, L.host_word_dev);
    if (S) {
        hipLaunchKernelGGL(sl_starts, dim3((unsigned)nblk), dim3(kSB), 0, s, dbuf, nbytes, L.totals, S, p0, reached);
        hipLaunchKernelGGL(sl_walk, dim3((unsigned)nblk), dim3(kSB), 0, s, dbuf, nbytes, L.totals, S, p0, reached,
                           gsum, bsum, bscr, L.flags);
        hipLaunchKernelGGL(sp_scan_tiles, dim3(1), dim3(kScanT), 0, s, bsum, bscr, nblk, L.totals + 1);
        hipLaunchKernelGGL(sl_place, dim3((unsigned)nblk), dim3(kSB), 0, s, g, dbuf, nbytes, L.totals, S, p0, reached,
                           gsum, bsum, L.rec, (uint32_t)qcap, L.flags);
    }
    const unsigned lb = (unsigned)std::min<size_t>(1024, qcap);
    hipLaunchKernelGGL(sl_long, dim3(lb), dim3(kSB), 0, s, g, dbuf, L.rec, L.flags, L.host_word_dev);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return hip_error(e, "sparse lift", __FILE__, __LINE__);
    const uint64_t total = word[1];
    if (word[2]) return size_error(total);
    *out_len = total;
    if (word[0] == 0) return ONO_OK;
    // speculation missed or the stream is malformed: the sequential parse decides
    g_lift_fallbacks.fetch_add(1);
    ONO_HIP(hipMemsetAsync(g, 0, total * sizeof(float), s));
    const uint8_t *hb = host_bytes();
    if (!hb) return set_error(ONO_E_HIP, "sparse lift: download of the stream failed");
    return lift_host_path(g, hb, dbuf, nbytes, total, s);
}


// ---------------------------------------------------------- threshold ----
// calculate_threshold (comms/src/sparse/protocol.rs:33-49): the sample's
// |g| values (f32::abs clears the sign bit), the k-th in f32::total_cmp order
// (select_nth_unstable_by), then f32::max with f16::MIN_POSITIVE (NaN-ignoring).
// total_cmp on sign-clear floats is the order of their bit patterns (NaN above
// +inf), so this is an exact radix select over u32 keys: one workgroup, the
// sample (<= 16384 keys) staged in LDS, four 8-bit digit passes, each a
// histogram with LDS atomics and a scan for the digit that holds rank k.
constexpr int kThrT = 1024;
constexpr uint32_t kSampleMax = 16384;  // SAMPLE_SIZE, protocol.rs:13-19
__global__ __launch_bounds__(kThrT) void sp_threshold(const float *g, const uint32_t *idx, uint32_t m, uint32_t k,
                                                      float *t_out) {
    __shared__ uint32_t keys[kSampleMax];
    __shared__ uint32_t hist[256];
    __shared__ uint32_t sel[2];
    for (uint32_t i = threadIdx.x; i < m; i += kThrT) {
        const size_t j = idx ? idx[i] : i;
        keys[i] = __builtin_bit_cast(uint32_t, g[j]) & 0x7FFFFFFFu;
    }
    uint32_t prefix = 0, mask = 0, kk = k;
    for (int shift = 24; shift >= 0; shift -= 8) {
        for (uint32_t b = threadIdx.x; b < 256; b += kThrT) hist[b] = 0;
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < m; i += kThrT) {
            const uint32_t key = keys[i];
            if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t c = 0, d = 0;
            for (; d < 255; d++) {
                if (c + hist[d] > kk) break;
                c += hist[d];
            }
            sel[0] = prefix | (d << shift);
            sel[1] = kk - c;
        }
        __syncthreads();
        prefix = sel[0];
        kk = sel[1];
        mask |= 255u << shift;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const float mp = 6.103515625e-05f;  // f16::MIN_POSITIVE
        const float t = __builtin_bit_cast(float, prefix);
        t_out[0] = prefix > 0x7F800000u ? mp : (t > mp ? t : mp);
    }
}

struct ThrScratch {
    uint32_t *idx = nullptr;
    float *t_host = nullptr, *t_dev = nullptr;
};
ThrScratch g_thr[64];

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
    const bool vec = ((uintptr_t)g & 15u) == 0;
    // A buffer of the worst-case size cannot overflow: count, scan, write and
    // headers run back to back and the host reads the totals once at the end.
    // A smaller buffer needs the exact size first (one extra host round trip).
    const bool worst_case_fits = cap >= ono_sparse_max_bytes(n);
    std::lock_guard<std::mutex> lk(g_scratch_mu);  // one call at a time per process owns the scratch
    Scratch *sc = nullptr;
    int rc = scratch_for(ntiles, maxruns, &sc);
    if (rc) return rc;
    uint32_t *tileF = sc->tiles, *tileS = sc->tiles + ntiles + 1, *RU = sc->runs, *RF = sc->runs + maxruns;
    volatile uint64_t *tot = sc->host_tot;  // pinned, written by the device
    tot[0] = tot[1] = 0;
    uint64_t *totals = sc->totals_dev;
    hipError_t e = hipSuccess;
    if (ntiles) {
        hipLaunchKernelGGL(sp_count, dim3((unsigned)ntiles), dim3(kSB), 0, s, g, n, threshold, tileF, tileS, vec);
        hipLaunchKernelGGL(sp_scan_tiles, dim3(1), dim3(kScanT), 0, s, tileF, tileS, ntiles, totals);
    } else {
        e = hipMemsetAsync(totals, 0, 2 * sizeof(uint64_t), s);
    }
    if (e == hipSuccess) e = hipGetLastError();
    if (e == hipSuccess && !worst_case_fits) {
        hipLaunchKernelGGL(sp_totals_out, dim3(1), dim3(1), 0, s, totals, sc->host_tot_dev);
        e = hipStreamSynchronize(s);
        if (e == hipSuccess && 8 + 8 * tot[1] + 2 * tot[0] > cap)
            return set_error(ONO_E_SIZE, "sparse encoding needs %zu bytes, buffer holds %zu",
                             (size_t)(8 + 8 * tot[1] + 2 * tot[0]), cap);
    }
    if (e != hipSuccess) return hip_error(e, "sparse count", __FILE__, __LINE__);
    if (ntiles)
        hipLaunchKernelGGL(sp_write, dim3((unsigned)ntiles), dim3(kSB), 0, s, g, n, threshold, tileF, tileS, buf, RU,
                           RF, vec);
    const size_t hdr_runs = worst_case_fits ? maxruns : (size_t)tot[1];
    const size_t hblocks = std::min<size_t>(4096, (hdr_runs + kSB) / kSB);
    hipLaunchKernelGGL(sp_headers, dim3((unsigned)hblocks), dim3(kSB), 0, s, RU, RF, totals, (uint64_t)n, buf,
                       sc->host_tot_dev);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return hip_error(e, "sparse write", __FILE__, __LINE__);
    *nbytes = 8 + 8 * (size_t)tot[1] + 2 * (size_t)tot[0];
    return ONO_OK;
}

int ono_sparse_lift(float *g, size_t cap, size_t *out_len, const uint8_t *buf, size_t nbytes, void *stream) {
    if (!out_len || (!buf && nbytes)) return set_error(ONO_E_ARG, "NULL argument");
    // protocol.rs:96-144: the total first, then the records
    if (nbytes < 8) return set_error(ONO_E_PROTO, "The given sparse buffer is smaller than TOTAL_LEN_SIZE");
    uint64_t total = 0;
    for (int q = 0; q < 8; q++) total |= (uint64_t)buf[q] << (8 * q);
    if (total > cap) return set_error(ONO_E_SIZE, "sparse gradient of %llu values, buffer of %zu",
                                      (unsigned long long)total, cap);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    int dev = 0;
    ONO_HIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) return set_error(ONO_E_ARG, "device %d", dev);
    LiftScratch &L = g_lift[dev];
    int rc = grow(&L.buf, L.buf_cap, nbytes);
    if (rc) return rc;
    ONO_HIP(hipMemcpyAsync(L.buf, buf, nbytes, hipMemcpyHostToDevice, s));
    return lift_device(g, cap, out_len, L.buf, buf, nbytes, s);
}


int ono_sparse_threshold(float *t_out, const float *g, size_t n, const uint32_t *idx_host, size_t m, float r,
                         void *stream) {
    if (!t_out || (n && !g)) return set_error(ONO_E_ARG, "NULL argument");
    if (!(r > 0.0f && r <= 1.0f)) return set_error(ONO_E_ARG, "ratio %g outside (0, 1]", (double)r);
    if (idx_host ? (m == 0 || m > kSampleMax) : (n > kSampleMax || m != n))
        return set_error(ONO_E_ARG, "sample of %zu values from %zu: at most %u, and indices above %u values", m, n,
                         kSampleMax, kSampleMax);
    if (n == 0) { *t_out = 0.0f; return ONO_OK; }  // an empty gradient: nothing is kept
    if (idx_host)
        for (size_t i = 0; i < m; i++)
            if (idx_host[i] >= n) return set_error(ONO_E_ARG, "sample index %u out of %zu", idx_host[i], n);
    // (sample.len() as f32 * (1.0 - r)) as usize, clamped to the last index
    const float kf = (float)m * (1.0f - r);
    size_t k = kf <= 0.0f ? 0 : (size_t)kf;
    if (k > m - 1) k = m - 1;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    int dev = 0;
    ONO_HIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) return set_error(ONO_E_ARG, "device %d", dev);
    ThrScratch &T = g_thr[dev];
    if (!T.idx) {
        ONO_HIP(hipMalloc((void **)&T.idx, kSampleMax * sizeof(uint32_t)));
        ONO_HIP(hipHostMalloc((void **)&T.t_host, sizeof(float), hipHostMallocMapped | hipHostMallocCoherent));
        ONO_HIP(hipHostGetDevicePointer((void **)&T.t_dev, T.t_host, 0));
    }
    if (idx_host) ONO_HIP(hipMemcpyAsync(T.idx, idx_host, m * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(sp_threshold, dim3(1), dim3(kThrT), 0, s, g, idx_host ? T.idx : nullptr, (uint32_t)m,
                       (uint32_t)k, T.t_dev);
    ONO_HIP(hipGetLastError());
    ONO_HIP(hipStreamSynchronize(s));
    *t_out = *(volatile float *)T.t_host;
    return ONO_OK;
}

size_t ono_sparse_lift_fallbacks(void) { return g_lift_fallbacks.load(); }

int ono_sparse_lift_dev(float *g, size_t cap, size_t *out_len, const uint8_t *buf_dev, size_t nbytes,
                        void *stream) {
    if (!out_len || (!buf_dev && nbytes)) return set_error(ONO_E_ARG, "NULL argument");
    if (nbytes < 8) return set_error(ONO_E_PROTO, "The given sparse buffer is smaller than TOTAL_LEN_SIZE");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    return lift_device(g, cap, out_len, buf_dev, nullptr, nbytes, s);
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
