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
// Three launches (see "encoder" below): each tile's byte range built in LDS
// and written to a scratch slot -> one scan of the tile records -> each slot
// moved to its place with the two cross-tile header fields completed.  g is
// read once; the totals stay on the device (the blocking form reads them once,
// at the end, for the wire length; the stream-ordered form leaves it in HBM).
// Decoding is a parallel parse on the device (the record stream is a linked
// list: each header gives the next one's position), see "Lift" below; the
// reference's sequential parse on the host remains as the exact fallback and
// the source of the reference's error messages.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <atomic>
#include <map>
#include <mutex>
#include <vector>

#include "ono_internal.h"

using namespace ono;

namespace {

constexpr int kSB = 256;             // threads per block (4 waves)
constexpr int kEPT = 8;              // elements per thread
constexpr int kTile = kSB * kEPT;    // 2048 elements per tile
constexpr int kIT = 128, kIE = kTile / kIT;  // the encoder's tile: 2 waves x 16 values per thread

// half 2.7.1 conversions = the gfx950 cvt instructions, NaN rules included (ono_kernels.hip to_f16)
__device__ __forceinline__ uint16_t to_f16_sp(float x) { return __builtin_bit_cast(uint16_t, (_Float16)x); }
__device__ __forceinline__ float from_f16_sp(uint16_t b) { return (float)__builtin_bit_cast(_Float16, b); }

// g.abs() >= threshold (NaN never kept, as in Rust)
__device__ __forceinline__ bool kept(float x, float t) { return fabsf(x) >= t; }

// Keep flags of a thread's E values and which of them start a run (the
// element before the thread's first one is the previous lane's last, taken by
// a shuffle; lane 0 has it loaded).
struct Bits {
    uint32_t keep = 0, start = 0;
};
typedef float f4s __attribute__((ext_vector_type(4)));

// The value of lane - 1 (DPP wave_shr:1; lane 0 gets 0): no LDS round trip.
__device__ __forceinline__ uint32_t lane_before(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xF, 0xF, false);
}
// Inclusive sum over lanes 0..l, all DPP (row_shr 1 / 2 / 4 / 8 within rows
// of 16, then row_bcast 15 and 31 across rows): six VALU adds.
__device__ __forceinline__ uint32_t wave_incl_sum_dpp(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);
    return v;
}
// The same shape for max (identity 0) and min (identity ~0: lanes without a
// source keep `old`).
__device__ __forceinline__ uint32_t wave_incl_max_dpp(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false));
    return v;
}
__device__ __forceinline__ uint32_t wave_incl_min_dpp(uint32_t v) {
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x111, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x112, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x114, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x118, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x142, 0xA, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x143, 0xC, 0xF, false));
    return v;
}
template <int E>
__device__ __forceinline__ Bits flags_of(const float (&x)[E], float before, size_t n, float t, size_t base) {
    Bits b;
#pragma unroll
    for (int e = 0; e < E; e++)
        if (base + e < n && kept(x[e], t)) b.keep |= 1u << e;
    const uint32_t last = (b.keep >> (E - 1)) & 1u;
    uint32_t prev = lane_before(last);
    if ((threadIdx.x & 63) == 0) prev = base > 0 && base - 1 < n && kept(before, t) ? 1u : 0u;
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

// ------------------------------------------------------------- encoder ----
// Three launches, g read once (64 MiB, 10 % kept, MI355X: about 20 + 7.3 +
// 10.5 us, 38 us per drop back to back with the gradient read from HBM; the
// four-launch count / scan / write / headers design it replaced read g twice
// and took ~50):
//  1. sp_image, one 128-thread workgroup per 2048-value tile (16 values per
//     thread, plain 16-B loads): flags, one LDS exchange of the waves' DPP scans, then the
//     tile's byte range of the wire built in LDS — its values, and its run
//     headers with every field that the tile alone determines, written by the
//     threads that hold the run starts — copied to the tile's slot of a
//     scratch image (5 B per value), plus two 8-B records: recA = {kept | runs
//     << 16, last kept + 1 | first unkept << 16}, recB = {first / last header
//     position, first run's offset | last run's length} (all tile-local).
//  2. sp_scan_rec, one workgroup per 1024 tiles (two levels, the last
//     workgroup to arrive makes the chunk carries): per tile the exclusive prefix sums of kept
//     and runs (its place in the wire), the exclusive prefix max of "last kept
//     + 1" (P: where the run before the tile's first run ended) and the
//     exclusive suffix min of "first unkept" (Q: where a run still open at the
//     tile's end ends).
//  3. sp_move, one wave per tile: the slot to its place in the wire (2-B
//     aligned) in 16-B destination chunks, completing on the way the two
//     header fields that depend on other tiles: the first run's offset (+=
//     tile start - P) and, when the tile's last value is kept, the last run's
//     length (+= Q - tile end).  A run's offset is the gap since the previous
//     run's end, its length the distance to the first unkept value after its
//     start.
constexpr int kSlotU16 = 5128;  // the largest tile image, 3 S + 2049 <= 5121 units (S <= 1024), padded to 16 B
static_assert((kSlotU16 * 2) % 16 == 0, "slots are 16-B aligned");

// Block-wide scans over the threads of a tile (tile-local indices): the
// exclusive prefix of (kept, runs), the last kept index + 1 before the thread
// (0: none) and the first unkept index after it (kTile: none), and the tile's
// totals, last kept + 1 and first unkept — one LDS exchange of wave totals.
struct TileScan {
    uint32_t ef, es;              // this thread's exclusive prefix
    uint32_t tf, ts;              // tile totals
    uint32_t kept1_before, unkept_after;
    uint32_t last_kept1, first_unkept;
};
__device__ __forceinline__ TileScan tile_scan(uint32_t keep, uint32_t start, uint32_t unkept) {
    __shared__ uint32_t wf[kIT / 64], ws[kIT / 64], wl[kIT / 64], wu[kIT / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t lo = threadIdx.x * kIE;
    // kept and run starts packed in one word (a wave holds < 2^16 of each):
    // one DPP scan for both
    const uint32_t own = __popc(keep) | __popc(start) << 16;
    const uint32_t inc = wave_incl_sum_dpp(own), exc = inc - own;
    const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
    const uint32_t xf = exc & 0xFFFFu, xs = exc >> 16, sf = tot & 0xFFFFu, ss = tot >> 16;
    // the nearest lane below with a kept value / above with an unkept one:
    // one ballot and one lane-indexed shuffle each (no scan ladder)
    const uint32_t k1 = keep ? lo + 32u - __clz(keep) : 0u;                  // last kept + 1 in the thread
    const uint32_t u1 = unkept ? lo + (uint32_t)(__ffs(unkept) - 1) : kTile;  // first unkept in the thread
    const uint64_t mk = __ballot(keep != 0), mu = __ballot(unkept != 0);
    const uint64_t below = (1ull << lane) - 1ull, above = ~below & ~(1ull << lane);
    const uint64_t kbm = mk & below, uam = mu & above;
    const int lk = kbm ? 63 - __clzll((long long)kbm) : 0, lu = uam ? __ffsll((unsigned long long)uam) - 1 : 0;
    const uint32_t ykb = __shfl(k1, lk, 64), yua = __shfl(u1, lu, 64);
    const uint32_t kb = kbm ? ykb : 0u, ua = uam ? yua : (uint32_t)kTile;
    const uint32_t wk = __shfl(k1, mk ? 63 - __clzll((long long)mk) : 0, 64);  // all lanes shuffle
    const uint32_t wuu = __shfl(u1, mu ? __ffsll((unsigned long long)mu) - 1 : 0, 64);
    if (lane == 0) {  // wave totals
        wf[wave] = sf;
        ws[wave] = ss;
        wl[wave] = mk ? wk : 0u;
        wu[wave] = mu ? wuu : (uint32_t)kTile;
    }
    __syncthreads();
    TileScan r{xf, xs, 0, 0, kb, ua, 0, kTile};
#pragma unroll
    for (int w = 0; w < kIT / 64; w++) {
        if (w < wave) { r.ef += wf[w]; r.es += ws[w]; r.kept1_before = max(r.kept1_before, wl[w]); }
        if (w > wave) r.unkept_after = min(r.unkept_after, wu[w]);
        r.tf += wf[w];
        r.ts += ws[w];
        r.last_kept1 = max(r.last_kept1, wl[w]);
        r.first_unkept = min(r.first_unkept, wu[w]);
    }
    return r;
}
static_assert(kIE <= 32, "a thread's flags are one 32-bit mask; its counts are packed as 16-bit halves");

// One workgroup per tile: flags, the block scans, then the tile's byte range
// in LDS — each kept value at 8 S + 2 F, each run's header by the thread that
// holds its start (offset = start - end of the previous run, length = first
// unkept after it - start, both tile-local; a run open at either tile edge is
// completed by sp_move) — and out to the tile's slot.  Records: recA = {kept
// | runs << 16, last kept + 1 | first unkept << 16} (what the scan needs),
// recB = {first header | last header << 16, the first run's offset | the
// last run's length << 16} (what the move completes).
__global__ __launch_bounds__(kIT) void sp_image(const float *__restrict__ g, size_t n, float t, bool vec, uint16_t *img,
                                                uint2 *recA, uint2 *recB) {
    __shared__ __attribute__((aligned(16))) uint16_t stage[kSlotU16 + 2 * kIT];  // + a spare dword per thread
    __shared__ uint32_t rb[2];  // header position | offset of the tile's first run; position | length of its last
    const size_t tile = blockIdx.x, tile0 = tile * kTile;
    const uint32_t lo = threadIdx.x * kIE;  // the thread's first element, tile-local
    const size_t base = tile0 + lo;
    float x[kIE];
    // four 16-B loads per thread, 2 KiB per wave in flight; plain loads: nt
    // loads measured slower here even from HBM (64 MiB drop over 6 rotating
    // gradients: 38.2 us with plain loads, 49.9 us with nt)
    if (vec && base + kIE <= n) {
#pragma unroll
        for (int q = 0; q < kIE / 4; q++) {
            const f4s a = *((const f4s *)(g + base) + q);
            x[4 * q] = a.x; x[4 * q + 1] = a.y; x[4 * q + 2] = a.z; x[4 * q + 3] = a.w;
        }
    } else {
#pragma unroll
        for (int e = 0; e < kIE; e++) x[e] = base + e < n ? g[base + e] : 0.0f;
    }
    // the value before the wave's first one (lane 0 uses it): a wave-uniform
    // address, so a scalar load that waits on its own counter — as a vector
    // load under lane 0's branch it was issued, and waited for, only after
    // all of the values had landed (+6 us per drop)
    const uint32_t wbase = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(tile0 + (threadIdx.x & ~63u) * kIE));
    const float before = wbase ? g[min((size_t)wbase - 1, n - 1)] : 0.0f;
    const Bits b = flags_of(x, before, n, t, base);
    const uint32_t full = kIE >= 32 ? 0xFFFFFFFFu : (1u << (kIE & 31)) - 1u;
    const uint32_t valid = base >= n ? 0u : (n - base >= (size_t)kIE ? full : (1u << (n - base)) - 1u);
    const uint32_t unk = valid & ~b.keep;
    const TileScan ts = tile_scan(b.keep, b.start, unk);
    const uint32_t R = ts.ts, F = ts.tf;
    const uint32_t tend_l = (uint32_t)min((size_t)kTile, n - tile0);
    // the values: one store per element, branch-free — to byte 8 S + 2 F of
    // the tile's range when kept, else to this thread's spare unit past the
    // image (no exec-mask branches around 16 conditional stores)
    {
#pragma unroll
        for (int e = 0; e < kIE; e++) {
            const uint32_t f = ts.ef + __popc(b.keep & ((1u << e) - 1u));
            const uint32_t sl = ts.es + __popc(b.start & ((2u << e) - 1u));  // runs started at or before e
            const uint32_t pos = (b.keep >> e & 1u) ? 4 * sl + f : (uint32_t)kSlotU16 + 2 * threadIdx.x;
            stage[pos] = to_f16_sp(x[e]);
        }
    }
    // the headers: a loop over this thread's run starts (offset = start - end
    // of the previous run, length = first unkept after it - start, both
    // tile-local; runs open at a tile edge are completed by sp_move).  The
    // stores are volatile LDS stores so that they stay 2-byte stores: merged
    // into wider ones they would be unaligned LDS accesses.
    typedef __attribute__((address_space(3))) volatile uint16_t lds_u16;
    lds_u16 *vst = (lds_u16 *)stage;
    for (uint32_t m = b.start; m; m &= m - 1u) {
        const int e = __ffs(m) - 1;
        const uint32_t below = (1u << e) - 1u;
        const uint32_t f = ts.ef + __popc(b.keep & below), sl = ts.es + __popc(b.start & below);
        const uint32_t mk = b.keep & below, mu = unk & ~((2u << e) - 1u);
        const uint32_t prev_end = mk ? lo + 32u - __clz(mk) : ts.kept1_before;
        const uint32_t next_unkept =
            mu ? lo + (uint32_t)(__ffs(mu) - 1) : (ts.unkept_after < (uint32_t)kTile ? ts.unkept_after : tend_l);
        const uint32_t off = lo + e - prev_end, len = next_unkept - (lo + e);
        const uint32_t p = 4 * sl + f;  // the header, 8 bytes before the run's first value
        vst[p] = (uint16_t)off;
        vst[p + 1] = 0;
        vst[p + 2] = (uint16_t)len;
        vst[p + 3] = 0;
        if (sl == 0) rb[0] = p | off << 16;
        if (sl == R - 1) rb[1] = p | len << 16;
    }
    __syncthreads();
    const uint32_t nu16 = 4 * R + F;
    uint4 *slot = (uint4 *)(img + tile * kSlotU16);
    const uint4 *st4 = (const uint4 *)stage;
    for (uint32_t k = threadIdx.x; k < (nu16 + 7) / 8; k += kIT) slot[k] = st4[k];
    if (threadIdx.x == 0) {
        recA[tile] = make_uint2(F | R << 16, ts.last_kept1 | ts.first_unkept << 16);
        recB[tile] = R ? make_uint2((rb[0] & 0xFFFFu) | rb[1] << 16, rb[0] >> 16 | (rb[1] & 0xFFFF0000u))
                       : make_uint2(0u, 0u);
    }
}


// recA -> pre = {F0, S0, P, Q} per tile (F0 / S0: kept values / runs before
// the tile; P: last kept index + 1 before it, 0 if none; Q: first unkept
// index after it, n if none), in two levels within one launch: each
// workgroup scans a chunk of kRecChunk tiles (LDS-staged, DPP wave scans;
// the suffix min as a forward scan over the chunk reversed) into chunk-local
// prefixes and publishes the chunk's aggregate; the workgroup that arrives
// last (one agent-scope counter, one arrival per workgroup) turns the
// aggregates into per-chunk carries and the totals.  sp_move adds its
// chunk's carry.
constexpr int kRecT = 256, kRecPer = 4, kRecChunk = kRecT * kRecPer;  // 1024 tiles per workgroup
__global__ __launch_bounds__(kRecT) void sp_scan_rec(const uint2 *recA, uint4 *pre, uint4 *agg, uint4 *carry,
                                                      uint32_t *counter, size_t ntiles, uint32_t n, uint64_t *totals) {
    __shared__ uint32_t la[kRecChunk], lb[kRecChunk];
    __shared__ uint32_t rf[kRecChunk], rs[kRecChunk], rp[kRecChunk], rq[kRecChunk];
    __shared__ uint32_t wa[kRecT / 64], wb[kRecT / 64], wc[kRecT / 64], wd[kRecT / 64];
    __shared__ uint32_t is_last;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const size_t c0 = (size_t)blockIdx.x * kRecChunk;
    const uint32_t m = (uint32_t)min((size_t)kRecChunk, ntiles - c0);
    for (uint32_t i = threadIdx.x; i < kRecChunk; i += kRecT) {
        const uint2 r = i < m ? recA[c0 + i] : make_uint2(0u, (uint32_t)kTile << 16);
        la[i] = r.x;
        lb[i] = r.y;
    }
    __syncthreads();
    const uint32_t lo = threadIdx.x * kRecPer;
    // forward: this thread's tiles lo .. lo + 3
    uint32_t sumf = 0, sums = 0, mx = 0, lk[kRecPer], cnt[kRecPer];
#pragma unroll
    for (int k = 0; k < kRecPer; k++) {
        cnt[k] = la[lo + k];
        const uint32_t l1 = lb[lo + k] & 0xFFFFu;
        sumf += cnt[k] & 0xFFFFu;
        sums += cnt[k] >> 16;
        lk[k] = l1 ? (uint32_t)((c0 + lo + k) * kTile) + l1 : 0u;  // global last kept + 1
        mx = max(mx, lk[k]);
    }
    // backward, as a forward scan over the chunk reversed: tiles m-1-lo .. m-4-lo
    uint32_t fu[kRecPer], mn = n;
#pragma unroll
    for (int k = 0; k < kRecPer; k++) {
        const uint32_t idx = lo + k, i = m - 1 - idx;
        const uint32_t f1 = idx < m ? lb[i] >> 16 : (uint32_t)kTile;
        fu[k] = f1 < (uint32_t)kTile ? (uint32_t)((c0 + i) * kTile) + f1 : n;
        mn = min(mn, fu[k]);
    }
    const uint32_t i_f = wave_incl_sum_dpp(sumf), i_s = wave_incl_sum_dpp(sums);
    const uint32_t i_m = wave_incl_max_dpp(mx), i_u = wave_incl_min_dpp(mn);
    if (lane == 63) { wa[wave] = i_f; wb[wave] = i_s; wc[wave] = i_m; wd[wave] = i_u; }
    __syncthreads();
    uint32_t pf = 0, ps = 0, pm = 0, q = n, tf = 0, tsum = 0, tm = 0, tq = n;
#pragma unroll
    for (int w = 0; w < kRecT / 64; w++) {
        if (w < wave) { pf += wa[w]; ps += wb[w]; pm = max(pm, wc[w]); q = min(q, wd[w]); }
        tf += wa[w];
        tsum += wb[w];
        tm = max(tm, wc[w]);
        tq = min(tq, wd[w]);
    }
    pf += i_f - sumf;  // exclusive, within the wave
    ps += i_s - sums;
    pm = max(pm, lane_before(i_m));  // lane 0 gets 0, the identity
    q = min(q, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)i_u, 0x138, 0xF, 0xF, false));  // lane 0: ~0
#pragma unroll
    for (int k = 0; k < kRecPer; k++) {
        rf[lo + k] = pf;
        rs[lo + k] = ps;
        rp[lo + k] = pm;
        pf += cnt[k] & 0xFFFFu;
        ps += cnt[k] >> 16;
        pm = max(pm, lk[k]);
        const uint32_t idx = lo + k;
        if (idx < m) rq[m - 1 - idx] = q;
        q = min(q, fu[k]);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < m; i += kRecT) pre[c0 + i] = make_uint4(rf[i], rs[i], rp[i], rq[i]);
    // the chunk's aggregate, then one arrival; the last workgroup makes the carries
    if (threadIdx.x == 0) {
        agg[blockIdx.x] = make_uint4(tf, tsum, tm, tq);
        const uint32_t before = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        is_last = before == gridDim.x - 1 ? 1u : 0u;
    }
    __syncthreads();
    if (!is_last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (threadIdx.x == 0) {
        const uint32_t G = gridDim.x;
        uint32_t cf = 0, cs = 0, cm = 0;
        for (uint32_t g = 0; g < G; g++) {  // forward carries (atomic loads: never a stale cached line)
            const uint32_t af = __hip_atomic_load(&agg[g].x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t as = __hip_atomic_load(&agg[g].y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t am = __hip_atomic_load(&agg[g].z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            carry[g] = make_uint4(cf, cs, cm, 0u);
            cf += af;
            cs += as;
            cm = max(cm, am);
        }
        uint32_t cq = n;
        for (uint32_t g = G; g-- > 0;) {  // backward carries
            carry[g].w = cq;
            cq = min(cq, __hip_atomic_load(&agg[g].w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        }
        totals[0] = cf;
        totals[1] = cs;
        __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // for the next drop
    }
}

// One tile's slot -> its place in the wire, in 16-B chunks of the
// destination: the range starts O units (0..7, uniform) into its first
// aligned chunk, so destination chunk c takes slot units 8c - O .. 8c - O + 7
// — the last O units of slot chunk c - 1 (the lane before, by DPP) and the
// first 8 - O of slot chunk c (this lane).  Whole chunks are one 16-B store;
// the range's first and last chunk (shared with the neighbouring tiles) are
// stored unit by unit.  The two completed header fields (slot units c0, c0 + 1
// and hl + 2, hl + 3) are substituted in registers on the way.
constexpr int kMoveBatch = 2;  // 16-B slot chunks per lane loaded up front: 1024 units per wave
typedef uint32_t u4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ldn4(const uint4 *p) {
    const u4v r = __builtin_nontemporal_load((const u4v *)p);
    return make_uint4(r.x, r.y, r.z, r.w);
}
__device__ __forceinline__ uint4 lane_before4(uint4 v) {
    return make_uint4(lane_before(v.x), lane_before(v.y), lane_before(v.z), lane_before(v.w));
}
__device__ __forceinline__ uint4 readlane4(uint4 v, int l) {
    return make_uint4((uint32_t)__builtin_amdgcn_readlane((int)v.x, l), (uint32_t)__builtin_amdgcn_readlane((int)v.y, l),
                      (uint32_t)__builtin_amdgcn_readlane((int)v.z, l), (uint32_t)__builtin_amdgcn_readlane((int)v.w, l));
}
template <int O>
__device__ __forceinline__ void move_chunks(const uint4 *src4, uint4 (&v)[kMoveBatch], uint32_t nu16, uint32_t R,
                                            const uint32_t (&fu)[4], const uint32_t (&fv)[4], uint16_t *base16) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nchunks = nu16 ? (O + nu16 + 7) / 8 : 0;
    // field unit f of the range lands at base16 unit f + O: chunk, word, half
    uint32_t fc[4], fw[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        fc[j] = R ? (fu[j] + O) / 8 : 0xFFFFFFFFu;
        fw[j] = (fu[j] + O) % 8;  // unit within the chunk
    }
    uint4 carry = make_uint4(0, 0, 0, 0);  // slot chunk before this batch's first one
    auto batch = [&](uint32_t c0b) {
#pragma unroll
        for (int k = 0; k < kMoveBatch; k++) {
            const uint4 own = v[k];
            const uint4 up = lane_before4(own);
            const uint4 last = k ? readlane4(v[k - 1], 63) : carry;
            const uint4 prev = lane ? up : last;
            const uint32_t C[8] = {prev.x, prev.y, prev.z, prev.w, own.x, own.y, own.z, own.w};
            uint32_t o[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {  // out word j = concat units 8 - O + 2j, + 1
                const int sft = 8 - O + 2 * j;
                if (sft % 2 == 0) o[j] = C[sft / 2];
                else o[j] = __builtin_amdgcn_alignbit(C[(sft + 1) / 2], C[(sft - 1) / 2], 16);
            }
            const uint32_t c = c0b + lane + 64 * k;
            if (R) {
#pragma unroll
                for (int f = 0; f < 4; f++) {
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        if (c == fc[f] && fw[f] / 2 == (uint32_t)j) {
                            const uint32_t sh = 16 * (fw[f] % 2);
                            o[j] = (o[j] & ~(0xFFFFu << sh)) | fv[f] << sh;
                        }
                    }
                }
            }
            const bool whole = c * 8 >= (uint32_t)O && (size_t)c * 8 + 8 - O <= nu16;
            if (whole) {
                const u4v ov = {o[0], o[1], o[2], o[3]};
                __builtin_nontemporal_store(ov, (u4v *)(base16 + 8 * (size_t)c));
            } else if (c < nchunks) {  // the range's first / last chunk
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    const int64_t u = (int64_t)c * 8 + i - O;  // range unit
                    if (u >= 0 && u < (int64_t)nu16) base16[8 * (size_t)c + i] = (uint16_t)(o[i / 2] >> (16 * (i % 2)));
                }
            }
        }
        carry = readlane4(v[kMoveBatch - 1], 63);
    };
    batch(0);  // unconditionally: no branch for the compiler to sink the early loads behind
    for (uint32_t c0b = 64 * kMoveBatch; c0b < nchunks; c0b += 64 * kMoveBatch) {  // tiles of more than 1023 units
#pragma unroll
        for (int k = 0; k < kMoveBatch; k++) v[k] = ldn4(src4 + c0b + lane + 64 * k);
        batch(c0b);
    }
}

// One wave per tile: its records and prefix by scalar loads, the slot's first
// 1024 units (most tiles' whole image) issued at the same time, then the move.
// Block 0 also writes the u64 total length and publishes the wire length.
__global__ __launch_bounds__(kSB) __attribute__((amdgpu_waves_per_eu(8, 8))) void sp_move(
    const uint16_t *img, const uint2 *recA, const uint2 *recB, const uint4 *pre, const uint4 *carry, size_t ntiles,
    size_t n, const uint64_t *totals, uint8_t *buf, uint64_t *host_tot, uint64_t *nbytes_out) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // u64 LE total length, as four 2-byte stores (buf is 2-B aligned)
        for (int q = 0; q < 4; q++) *(uint16_t *)(buf + 2 * q) = (uint16_t)((uint64_t)n >> (16 * q));
        const uint64_t F = totals[0], R = totals[1];
        host_tot[0] = F;  // the wire length's terms, for the caller (host-mapped)
        host_tot[1] = R;
        if (nbytes_out) *nbytes_out = 8 + 8 * R + 2 * F;  // the stream-ordered form
    }
    const uint32_t lane = threadIdx.x & 63;
    // wave-uniform (readfirstlane): scalar base addresses and branches
    const size_t tile = (size_t)__builtin_amdgcn_readfirstlane((int)(blockIdx.x * (kSB / 64) + (threadIdx.x >> 6)));
    if (tile >= ntiles) return;
    const uint4 *src4 = (const uint4 *)(img + tile * kSlotU16);
    uint4 v[kMoveBatch];
#pragma unroll
    for (int k = 0; k < kMoveBatch; k++) v[k] = ldn4(src4 + lane + 64 * k);
    const uint2 a = recA[tile], hb = recB[tile];
    const uint4 pl = pre[tile], cr = carry[tile / kRecChunk];  // chunk-local prefix + the chunk's carry
    const uint4 p = make_uint4(pl.x + cr.x, pl.y + cr.y, max(pl.z, cr.z), min(pl.w, cr.w));
    const uint32_t F = a.x & 0xFFFFu, R = a.x >> 16, nu16 = 4 * R + F;
    const uint32_t tile0 = (uint32_t)(tile * kTile), tend = (uint32_t)min((size_t)tile0 + kTile, n);
    // the first run's offset and the last run's length (R > 0), completed
    const uint32_t off0 = (hb.y & 0xFFFFu) + (tile0 - p.z);
    const uint32_t lenl = (hb.y >> 16) + (tile0 + (a.y & 0xFFFFu) == tend ? p.w - tend : 0u);
    const uint32_t c0 = hb.x & 0xFFFFu, hl = hb.x >> 16;
    const uint32_t fu[4] = {c0, c0 + 1, hl + 2, hl + 3};
    const uint32_t fv[4] = {off0 & 0xFFFFu, off0 >> 16, lenl & 0xFFFFu, lenl >> 16};
    uint8_t *dst = buf + 8 + 8 * (size_t)p.y + 2 * (size_t)p.x;
    const uint32_t O = (uint32_t)__builtin_amdgcn_readfirstlane((int)(((uintptr_t)dst & 15u) >> 1));
    uint16_t *base16 = (uint16_t *)(dst - 2 * O);
    switch (O) {
    case 0: move_chunks<0>(src4, v, nu16, R, fu, fv, base16); break;
    case 1: move_chunks<1>(src4, v, nu16, R, fu, fv, base16); break;
    case 2: move_chunks<2>(src4, v, nu16, R, fu, fv, base16); break;
    case 3: move_chunks<3>(src4, v, nu16, R, fu, fv, base16); break;
    case 4: move_chunks<4>(src4, v, nu16, R, fu, fv, base16); break;
    case 5: move_chunks<5>(src4, v, nu16, R, fu, fv, base16); break;
    case 6: move_chunks<6>(src4, v, nu16, R, fu, fv, base16); break;
    default: move_chunks<7>(src4, v, nu16, R, fu, fv, base16); break;
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
// mapped words for the result), kept per (device, stream) and grown on
// demand: the stream-ordered allocations it replaces cost more than the
// kernels at 64 MiB.  Per stream, so stream-ordered drops on different
// streams never share it (on one stream they are ordered anyway).
struct Scratch {
    size_t tiles_cap = 0;
    uint2 *rec = nullptr;     // 2 x tiles_cap: recA, then recB
    uint4 *pre = nullptr;     // tiles_cap chunk-local prefixes, then 2 x (tiles_cap / kRecChunk + 1): aggregates, carries
    uint32_t *counter = nullptr;  // the record scan's arrival counter (zero between drops)
    uint16_t *img = nullptr;  // tiles_cap slots of kSlotU16 units (5 B per value)
    uint64_t *totals_dev = nullptr, *host_tot = nullptr, *host_tot_dev = nullptr;
};
std::mutex g_scratch_mu;
std::map<std::pair<int, hipStream_t>, Scratch> g_scratch;

int scratch_for(size_t ntiles, hipStream_t stream, Scratch **out) {
    int dev = 0;
    ONO_HIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) return set_error(ONO_E_ARG, "device %d", dev);
    Scratch &sc = g_scratch[{dev, stream}];
    if (!sc.totals_dev) {
        ONO_HIP(hipMalloc((void **)&sc.counter, sizeof(uint32_t)));
        ONO_HIP(hipMemset(sc.counter, 0, sizeof(uint32_t)));
        ONO_HIP(hipMalloc((void **)&sc.totals_dev, 2 * sizeof(uint64_t)));
        ONO_HIP(hipHostMalloc((void **)&sc.host_tot, 2 * sizeof(uint64_t), hipHostMallocMapped | hipHostMallocCoherent));
        ONO_HIP(hipHostGetDevicePointer((void **)&sc.host_tot_dev, sc.host_tot, 0));
    }
    if (ntiles > sc.tiles_cap) {
        (void)hipFree(sc.rec);
        (void)hipFree(sc.pre);
        (void)hipFree(sc.img);
        sc.rec = nullptr;
        sc.pre = nullptr;
        sc.img = nullptr;
        sc.tiles_cap = 0;
        ONO_HIP(hipMalloc((void **)&sc.rec, 2 * ntiles * sizeof(uint2)));
        ONO_HIP(hipMalloc((void **)&sc.pre, (ntiles + 2 * (ntiles / kRecChunk + 1)) * sizeof(uint4)));
        ONO_HIP(hipMalloc((void **)&sc.img, ntiles * kSlotU16 * sizeof(uint16_t)));
        sc.tiles_cap = ntiles;
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

}  // extern "C"

namespace {

// The four launches of the encoder.  nbytes_dev != NULL: the stream-ordered
// form (the buffer holds the worst case, nothing waits; the headers kernel
// stores the wire length there).  Otherwise blocking: the host reads the
// totals at the end (and, for a buffer below the worst case, once before the
// write pass to check the size).
int drop_launch(uint8_t *buf, size_t cap, size_t *nbytes, uint64_t *nbytes_dev, const float *g, size_t n,
                float threshold, hipStream_t s) {
    const size_t ntiles = n ? (n + kTile - 1) / kTile : 0;
    const bool vec = ((uintptr_t)g & 15u) == 0;
    const bool worst_case_fits = cap >= ono_sparse_max_bytes(n);
    std::lock_guard<std::mutex> lk(g_scratch_mu);  // the host side of one call at a time
    Scratch *sc = nullptr;
    int rc = scratch_for(ntiles, s, &sc);
    if (rc) return rc;
    uint2 *recA = sc->rec, *recB = sc->rec + sc->tiles_cap;
    const size_t nchunks = (ntiles + kRecChunk - 1) / kRecChunk;
    uint4 *pre = sc->pre, *agg = sc->pre + sc->tiles_cap, *carry = agg + (sc->tiles_cap / kRecChunk + 1);
    volatile uint64_t *tot = sc->host_tot;  // pinned, written by the device
    if (!nbytes_dev) tot[0] = tot[1] = 0;
    uint64_t *totals = sc->totals_dev;
    hipError_t e = hipSuccess;
    if (ntiles) {
        hipLaunchKernelGGL(sp_image, dim3((unsigned)ntiles), dim3(kIT), 0, s, g, n, threshold, vec, sc->img, recA,
                           recB);
        hipLaunchKernelGGL(sp_scan_rec, dim3((unsigned)nchunks), dim3(kRecT), 0, s, recA, pre, agg, carry,
                           sc->counter, ntiles, (uint32_t)n, totals);
    } else {
        e = hipMemsetAsync(totals, 0, 2 * sizeof(uint64_t), s);
    }
    if (e == hipSuccess) e = hipGetLastError();
    if (e == hipSuccess && !worst_case_fits) {  // the exact size first (one extra host round trip)
        hipLaunchKernelGGL(sp_totals_out, dim3(1), dim3(1), 0, s, totals, sc->host_tot_dev);
        e = hipStreamSynchronize(s);
        if (e == hipSuccess && 8 + 8 * tot[1] + 2 * tot[0] > cap)
            return set_error(ONO_E_SIZE, "sparse encoding needs %zu bytes, buffer holds %zu",
                             (size_t)(8 + 8 * tot[1] + 2 * tot[0]), cap);
    }
    if (e != hipSuccess) return hip_error(e, "sparse encode", __FILE__, __LINE__);
    const size_t mblocks = std::max<size_t>(1, (ntiles + kSB / 64 - 1) / (kSB / 64));
    hipLaunchKernelGGL(sp_move, dim3((unsigned)mblocks), dim3(kSB), 0, s, sc->img, recA, recB, pre, carry, ntiles, n, totals, buf,
                       sc->host_tot_dev, nbytes_dev);
    e = hipGetLastError();
    if (e != hipSuccess) return hip_error(e, "sparse write", __FILE__, __LINE__);
    if (nbytes_dev) return ONO_OK;
    e = hipStreamSynchronize(s);
    if (e != hipSuccess) return hip_error(e, "sparse write", __FILE__, __LINE__);
    *nbytes = 8 + 8 * (size_t)tot[1] + 2 * (size_t)tot[0];
    return ONO_OK;
}

int drop_args(const float *g, size_t n, const uint8_t *buf, size_t cap) {
    if ((n && !g) || !buf) return set_error(ONO_E_ARG, "NULL argument");
    if (n >= 0xFFFFFFFFull) return set_error(ONO_E_ARG, "sparse codec offsets are u32 (protocol.rs:13-19)");
    if (cap < 8) return set_error(ONO_E_SIZE, "buffer too small");
    return ONO_OK;
}

}  // namespace

extern "C" {

int ono_sparse_drop(uint8_t *buf, size_t cap, size_t *nbytes, const float *g, size_t n, float threshold,
                    void *stream) {
    if (!nbytes) return set_error(ONO_E_ARG, "NULL argument");
    int rc = drop_args(g, n, buf, cap);
    if (rc) return rc;
    return drop_launch(buf, cap, nbytes, nullptr, g, n, threshold, reinterpret_cast<hipStream_t>(stream));
}

int ono_sparse_drop_async(uint8_t *buf, size_t cap, uint64_t *nbytes_dev, const float *g, size_t n,
                          float threshold, void *stream) {
    if (!nbytes_dev) return set_error(ONO_E_ARG, "NULL argument");
    int rc = drop_args(g, n, buf, cap);
    if (rc) return rc;
    if (cap < ono_sparse_max_bytes(n))
        return set_error(ONO_E_SIZE, "the stream-ordered drop needs the worst-case buffer (%zu bytes, have %zu)",
                         ono_sparse_max_bytes(n), cap);
    return drop_launch(buf, cap, nullptr, nbytes_dev, g, n, threshold, reinterpret_cast<hipStream_t>(stream));
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
