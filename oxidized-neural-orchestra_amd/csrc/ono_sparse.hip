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
// Two launches (see "encoder" below): each tile's byte range built in LDS and
// written to a scratch slot, its counts added to its chunk's aggregate -> each
// slot moved to its place (its prefix from its chunk's records and the other
// chunks' aggregates) with the two cross-tile header fields completed.  g is
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
#include <chrono>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "ono_internal.h"

using namespace ono;

namespace {

constexpr int kSB = 256;             // threads per block (4 waves)
constexpr int kEPT = 8;              // elements per thread
constexpr int kTile = kSB * kEPT;    // 2048 elements per tile
constexpr int kIT = 128, kIE = kTile / kIT;  // the encoder's tile: 2 waves x 16 values per thread

#ifdef ONO_SP_STAMP
// Measurement build only (tools/sp_phases.hip compiles this file with ONO_SP_STAMP defined; the
// library never does): {start, mid - start, end - start, XCC id} in 100 MHz ticks per sp_image
// workgroup / sp_move wave, end = after the unit's own memory operations are acknowledged.
__device__ uint4 g_sp_stamp_img[1 << 16], g_sp_stamp_mov[1 << 18], g_sp_stamp_pli[1 << 16], g_sp_stamp_plp[1 << 16];
// pl_fused's look-back per tile: {polls of the slowest chunk lane, of the slowest tile lane, first round's
// loads back - start, publish - start}
__device__ uint4 g_sp_stamp_plf[1 << 16];
// sp_drop1 per tile: {threshold read - start, tile imaged - start, blockIdx.x, own group's look-back done -
// start} beside the sp_stamp record (mid = look-back done)
__device__ uint4 g_sp_stamp_d1[1 << 16], g_sp_stamp_d1b[1 << 16];
// sp_drop1 per tile, lane 0 of the look-back: {polls, their load ticks} of its own group, of earlier groups
__device__ uint4 g_sp_stamp_d1c[1 << 16];
__device__ __forceinline__ void sp_stamp(uint4 *st, size_t i, uint64_t t0, uint64_t tm) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    if ((threadIdx.x & 63) == 0) st[i] = make_uint4((unsigned)t0, (unsigned)(tm - t0), (unsigned)(t1 - t0), x & 0xF);
}
#define SP_CLOCK(v) const uint64_t v = __builtin_amdgcn_s_memrealtime()
#else
#define SP_CLOCK(v) (void)0
#endif

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
// Write-through stores (`nt sc1`): the line leaves the XCD's L2 with the store instead of staying
// dirty there until the kernel's end (a boundary behind B dirty bytes costs about B / 6 TB/s more).
// Used for sp_image's slots (the boundary to sp_move 2.8 -> 1.5 us); the wire (sp_move) and g
// (pl_place) measured slower with them (23 vs 11 us, 25 vs 18.7 us: profiles/r04_s15_*).
typedef uint32_t u4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st4_wt(void *p, uint4 v) {
    const u4v x = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" : : "v"(p), "v"(x) : "memory");
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
// `valid`: the thread's in-range values as a mask (one 32-bit test per thread
// instead of a 64-bit compare per value); keep bits select-and-or, no branches.
template <int E>
__device__ __forceinline__ Bits flags_of(const float (&x)[E], float before, size_t n, float t, size_t base,
                                         uint32_t valid) {
    Bits b;
    uint32_t k[E];
#pragma unroll
    for (int e = 0; e < E; e++) k[e] = kept(x[e], t) ? 1u << e : 0u;
#pragma unroll
    for (int e = 0; e < E; e++) b.keep |= k[e];
    b.keep &= valid;
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
    const uint32_t ia = wave_incl_sum_dpp(a), ib = wave_incl_sum_dpp(b);  // inclusive wave scans (DPP)
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


// ------------------------------------------------------------- encoder ----
// Two launches, g read once:
//  1. sp_image, one 128-thread workgroup per 2048-value tile (16 values per
//     thread, plain 16-B loads): flags, one LDS exchange of the waves' DPP scans, then the
//     tile's byte range of the wire built in LDS — its values, and its run
//     headers with every field that the tile alone determines, written by the
//     threads that hold the run starts — copied to the tile's slot of a
//     scratch image (5 B per value), plus two 8-B records: recA = {kept | runs
//     << 16, last kept + 1 | first unkept << 16}, recB = {first / last header
//     position, first run's offset | last run's length} (all tile-local), and
//     four device-scope atomics into its chunk's aggregate (kRecChunk tiles:
//     kept values, runs, last kept index + 1, first unkept index).
//  2. sp_move, one wave per tile: its place in the wire from the records of
//     its chunk and the aggregates of the others (tile_prefix), then the slot
//     to that place (2-B aligned) in 16-B destination chunks, completing on the
//     way the two header fields that depend on other tiles: the first run's
//     offset (+= tile start - P) and, when the tile's last value is kept, the
//     last run's length (+= Q - tile end).  A run's offset is the gap since the
//     previous run's end, its length the distance to the first unkept value
//     after its start.
// (Round 4 folded a third launch, a scan of the tile records between the two,
// into these: sp_image's atomics and the move's own reduction.)
constexpr int kSlotU16 = 5128;  // the largest tile image, 3 S + 2049 <= 5121 units (S <= 1024), padded to 16 B
static_assert((kSlotU16 * 2) % 16 == 0, "slots are 16-B aligned");
constexpr int kRecChunk = 128;  // tiles per chunk of the aggregates: two records per lane of the move's wave
constexpr int kAggStride = 8;   // one chunk aggregate per 128-B line (uint4 units): atomics of different chunks never share one
// The two aggregate arrays that calls alternate between share each chunk's line: array h at uint4 h * kAggHalf
// of it, so a reader that loads both (sp_emit: the parity comes with the records) asks for no more lines
constexpr int kAggHalf = 4;
static_assert(2 * kAggHalf <= kAggStride, "both arrays in the chunk's line");
// The encoders' error word (host_tot[3], host-mapped): a writer whose range would pass the buffer's end
// stores nothing and leaves kDropErrRange; aggregates that disagree with their records (not zero when
// the call began) kDropErrStale.  The blocking call returns it (ONO_E_IO); a stream-ordered call's
// length reads ~0 when the totals pass the buffer, and ono_sparse_drop_check reports the word.
constexpr uint64_t kDropErrRange = 1, kDropErrStale = 2;
__device__ __forceinline__ void drop_error(uint64_t *host_tot, uint64_t code) {
    __hip_atomic_store(host_tot + 3, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

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

// A tile's values and the value before the wave's first one (lane 0 uses
// it).  That one is a vector load of a wave-uniform address, issued first:
// as a scalar load it shares its counter with the LDS traffic of the tile
// being processed while this one is in flight, and every LDS wait there
// would wait for it.  FULL: all of the tile's values in range, 16-B aligned —
// four 16-B loads per thread (plain loads: nt loads measured slower here even
// from HBM, 38.2 vs 49.9 us per 64 MiB drop), five vector loads in all
// whatever the data, which is what lets the pipelined loop keep them in
// flight (a load count that differs by path makes the compiler wait for all).
template <bool FULL>
__device__ __forceinline__ void load_tile(const float *__restrict__ g, size_t n, size_t tile, float (&x)[kIE],
                                          float &before) {
    const size_t tile0 = tile * kTile, base = tile0 + threadIdx.x * kIE;
    size_t wb = tile0 + (threadIdx.x & ~63u) * kIE;
    wb = wb ? min(wb - 1, n - 1) : 0;
    uint32_t wbv = (uint32_t)wb;
    asm volatile("" : "+v"(wbv));  // a VGPR address: a vector load, not a scalar one
    before = g[wbv];
    if (FULL) {
#pragma unroll
        for (int q = 0; q < kIE / 4; q++) {
            const f4s a = *((const f4s *)(g + base) + q);
            x[4 * q] = a.x; x[4 * q + 1] = a.y; x[4 * q + 2] = a.z; x[4 * q + 3] = a.w;
        }
    } else {
#pragma unroll
        for (int e = 0; e < kIE; e++) x[e] = base + e < n ? g[base + e] : 0.0f;
    }
}

// A workgroup's part of its chunk's aggregate: kept values and runs (one 64-bit add), the last
// kept index + 1 (0: none), the first unkept index complemented (0: none) — identity 0 all.
struct ImgAgg {
    uint64_t fr = 0;
    uint32_t lk = 0, nfu = 0;
};
// One tile, its values in registers: flags, the block scans, then the tile's byte range in LDS —
// each kept value at 8 S + 2 F, each run's header by the thread that holds its start (offset =
// start - end of the previous run, length = first unkept after it - start, both tile-local; a run
// open at either tile edge is completed by sp_move) — and out to the tile's slot.  Records: recA =
// {kept | runs << 16, last kept + 1 | first unkept << 16} (the prefix's terms), recB = {first
// header | last header << 16, the first run's offset | the last run's length << 16} (what the move
// completes); its counts into the workgroup's aggregate (uniform values).
// One loop over the thread's kept values (in order, each position advanced from the last: + 1, + 4
// more at a run start) writes values and headers (the offset at a start, the length when the next
// run starts or after the loop); the values are read back from the thread's own units of an LDS
// copy (an indexable register file).  It replaced a value pass over all 16 elements followed by a
// loop over the run starts with two popcounts each (round 4: 33.9 vs 34.9 us per drop).
// What a tile's image holds beside its units (in LDS until the workgroup's next tile): the tile-local
// counts and edges, the first run's header unit and offset, the last run's header unit, length and start.
struct TileImg {
    uint32_t F, R;                  // kept values, runs
    uint32_t last_kept1, first_unkept;  // tile-local (0: none / kTile: none)
    uint32_t hp0, off0;             // the first run's header unit, its offset since the last kept value in the tile
    uint32_t hpl, lenl, rs_last;    // the last run's header unit, its length within the tile, its start
    const uint16_t *stage;          // the units (LDS)
};
// the tile's f16 values in LDS for the kept-value loop: 1 transposed (word q of thread t at q kIT + t:
// every read conflict-free), 0 the thread's 32 contiguous bytes (two 16-B stores; lanes 4 apart share a
// bank on the reads, up to 8-way)
#ifndef ONO_VALS_T
#define ONO_VALS_T 1
#endif
__device__ __forceinline__ TileImg build_image(size_t tile, const float (&x)[kIE], float before, size_t n, float t) {
    __shared__ __attribute__((aligned(16))) uint16_t stage[kSlotU16 + 2 * kIT];  // + a spare dword per thread
    __shared__ uint32_t rb[3];  // position | offset of the tile's first run; position | length of its last; its start
    const size_t tile0 = tile * kTile;
    const uint32_t lo = threadIdx.x * kIE;  // the thread's first element, tile-local
    const size_t base = tile0 + lo;
    const uint32_t full = kIE >= 32 ? 0xFFFFFFFFu : (1u << (kIE & 31)) - 1u;
    const uint32_t valid = base >= n ? 0u : (n - base >= (size_t)kIE ? full : (1u << (n - base)) - 1u);
    const Bits b = flags_of(x, before, n, t, base, valid);
    const uint32_t unk = valid & ~b.keep;
    const TileScan ts = tile_scan(b.keep, b.start, unk);
    const uint32_t R = ts.ts, F = ts.tf;
    const uint32_t tend_l = (uint32_t)min((size_t)kTile, n - tile0);
    typedef __attribute__((address_space(3))) volatile uint16_t lds_u16;
    lds_u16 *vst = (lds_u16 *)stage;
    {
        __shared__ __attribute__((aligned(16))) uint32_t vals[kTile / 2];
        uint32_t w[kIE / 2];
#pragma unroll
        for (int q = 0; q < kIE / 2; q++) w[q] = to_f16_sp(x[2 * q]) | (uint32_t)to_f16_sp(x[2 * q + 1]) << 16;
        // transposed: the thread's word q at q kIT + thread, so that the lanes' reads below, each of some
        // value of its own, fall in distinct banks whatever the values (a thread's 32 contiguous bytes
        // put lanes 4 apart on one bank: up to 8-way conflicts on every read, and 2-way on the writes)
#if ONO_VALS_T
#pragma unroll
        for (int q = 0; q < kIE / 2; q++) vals[q * kIT + threadIdx.x] = w[q];
        typedef __attribute__((address_space(3))) const uint16_t lds_cu16;
        lds_cu16 *v16 = (lds_cu16 *)vals + 2 * threadIdx.x;  // (an LDS read: a generic pointer would be a flat load)
#else
        uint4 *v4 = (uint4 *)(vals + lo / 2);
#pragma unroll
        for (int q = 0; q < kIE / 8; q++) v4[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
        typedef __attribute__((address_space(3))) const uint16_t lds_cu16;
        lds_cu16 *v16 = (lds_cu16 *)vals;  // (an LDS read: a generic pointer would be a flat load)
#endif
        uint32_t pos = 4 * ts.es + ts.ef;  // the next value's unit, before a header of its own
        uint32_t sl = ts.es, last = ts.kept1_before, hp = 0, rs = 0, hsl = 0;
        bool open = false;  // a run started in this thread, its length not written yet
        for (uint32_t m = b.keep; m; m &= m - 1u) {
            const uint32_t e = (uint32_t)__ffs(m) - 1u, i = lo + e;
            if (b.start >> e & 1u) {
                if (open) {  // the previous run ended at last (an unkept value before i)
                    const uint32_t len = last - rs;
                    vst[hp + 2] = (uint16_t)len;
                    vst[hp + 3] = 0;
                    if (hsl == R - 1) rb[1] = hp | len << 16;
                }
                hp = pos;
                pos += 4;
                rs = i;
                hsl = sl++;
                const uint32_t off = i - last;  // since the previous run's end (tile-local)
                vst[hp] = (uint16_t)off;
                vst[hp + 1] = 0;
                if (hsl == 0) rb[0] = hp | off << 16;
                if (hsl == R - 1) rb[2] = i;
                open = true;
            }
#if ONO_VALS_T
            vst[pos++] = v16[2 * kIT * (e >> 1) + (e & 1)];
#else
            vst[pos++] = v16[i];
#endif
            last = i + 1;
        }
        if (open) {  // the first unkept after the run: in the thread, else after it (tile-local)
            const uint32_t eo = last - lo;
            const uint32_t end = eo < (uint32_t)kIE && (valid >> eo & 1u)
                                     ? last : (ts.unkept_after < (uint32_t)kTile ? ts.unkept_after : tend_l);
            const uint32_t len = end - rs;
            vst[hp + 2] = (uint16_t)len;
            vst[hp + 3] = 0;
            if (hsl == R - 1) rb[1] = hp | len << 16;
        }
    }
    __syncthreads();
    TileImg ti{F, R, ts.last_kept1, ts.first_unkept, 0, 0, 0, 0, 0, stage};
    if (R) {
        ti.hp0 = rb[0] & 0xFFFFu;
        ti.off0 = rb[0] >> 16;
        ti.hpl = rb[1] & 0xFFFFu;
        ti.lenl = rb[1] >> 16;
        ti.rs_last = rb[2];
    }
    return ti;
}

__device__ __forceinline__ void image_tile(size_t tile, const float (&x)[kIE], float before, size_t n, float t,
                                           uint16_t *img, uint2 *recA, uint2 *recB, ImgAgg &acc) {
    const size_t tile0 = tile * kTile;
    const TileImg ti = build_image(tile, x, before, n, t);
    const uint32_t nu16 = 4 * ti.R + ti.F;
    uint4 *slot = (uint4 *)(img + tile * kSlotU16);
    const uint4 *st4 = (const uint4 *)ti.stage;
    for (uint32_t k = threadIdx.x; k < (nu16 + 7) / 8; k += kIT) st4_wt(slot + k, st4[k]);
    if (threadIdx.x == 0) {
        recA[tile] = make_uint2(ti.F | ti.R << 16, ti.last_kept1 | ti.first_unkept << 16);
        recB[tile] = ti.R ? make_uint2(ti.hp0 | ti.hpl << 16, ti.off0 | ti.lenl << 16) : make_uint2(0u, 0u);
    }
    acc.fr += (uint64_t)ti.F | (uint64_t)ti.R << 32;
    if (ti.F) acc.lk = (uint32_t)tile0 + ti.last_kept1;  // tiles in order: the latest one's is the max
    if (ti.first_unkept < (uint32_t)kTile && !acc.nfu) acc.nfu = ~((uint32_t)tile0 + ti.first_unkept);  // the first
}

// The encoder's first launch: workgroup w images tiles w tpw .. w tpw + tpw - 1 (tpw a power of two
// <= kRecChunk, so all in one chunk).  Over the full tiles of an aligned gradient the next tile's
// values are loaded while the current one is imaged, into two register sets in turn (no copy
// between them to wait for the loads); the last one's "next" is the current tile again (L2 hits),
// so that every pass has the same loads in flight.  A ragged last tile, or every tile of an
// unaligned gradient, goes one at a time after that.  Then three device-scope atomics add the
// workgroup's counts to its chunk's aggregate (one 128-B line per chunk: kRecChunk / tpw
// workgroups per line).  It also zeroes the next call's aggregates (the previous call's sp_move,
// which read them, is done).
__global__ __launch_bounds__(kIT) void sp_image(const float *__restrict__ g, size_t n, size_t ntiles, uint32_t tpw,
                                                float t, const float *t_dev, bool vec, uint16_t *img, uint2 *recA,
                                                uint2 *recB, uint4 *agg, uint4 *agg_next, uint32_t gcap) {
    SP_CLOCK(sp_t0);
    if (t_dev) t = *t_dev;  // the threshold a stream-ordered sp_threshold left (the TCP ring's push)
    for (size_t i = (size_t)blockIdx.x * kIT + threadIdx.x; i < gcap; i += (size_t)gridDim.x * kIT)
        agg_next[i * kAggStride] = make_uint4(0u, 0u, 0u, 0u);
    const size_t nfull = vec ? n / kTile : 0;
    const size_t t0 = (size_t)blockIdx.x * tpw, t1 = min(t0 + tpw, ntiles), f1 = min(t1, nfull);
    size_t tile = t0;
    ImgAgg acc;
    float xa[kIE], xb[kIE], ba = 0.0f, bb = 0.0f;
    if (tile < f1) {
        load_tile<true>(g, n, tile, xa, ba);
        for (;;) {
            size_t next = tile + 1;
            load_tile<true>(g, n, next < f1 ? next : tile, xb, bb);
            __builtin_amdgcn_sched_barrier(0);  // the loads issued before any use of the current values
            image_tile(tile, xa, ba, n, t, img, recA, recB, acc);
            tile = next;
            __syncthreads();  // the LDS image is reused
            if (tile >= f1) break;
            next = tile + 1;
            load_tile<true>(g, n, next < f1 ? next : tile, xa, ba);
            __builtin_amdgcn_sched_barrier(0);
            image_tile(tile, xb, bb, n, t, img, recA, recB, acc);
            tile = next;
            __syncthreads();
            if (tile >= f1) break;
        }
    }
    for (; tile < t1; tile++) {
        load_tile<false>(g, n, tile, xa, ba);
        image_tile(tile, xa, ba, n, t, img, recA, recB, acc);
        __syncthreads();
    }
    if (threadIdx.x == 0 && t0 < t1) {
        uint32_t *a = (uint32_t *)(agg + (t0 / kRecChunk) * kAggStride);
        if (acc.fr) {
            atomicAdd((unsigned long long *)a, (unsigned long long)acc.fr);
            atomicMax(a + 2, acc.lk);
        }
        if (acc.nfu) atomicMax(a + 3, acc.nfu);
    }
#ifdef ONO_SP_STAMP
    SP_CLOCK(sp_tm);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x < 64) sp_stamp(g_sp_stamp_img, blockIdx.x, sp_t0, sp_tm);
#endif
}

// Tiles are grouped in chunks of kRecChunk; sp_image leaves per chunk {kept values, runs, last kept
// index + 1 (0: none), ~first unkept index (0: none)} in agg.  A tile's place in the wire — kept
// values and runs before it, the last kept index + 1 before it (P, 0 if none) and the first unkept
// index after it (Q, n if none) — then takes one wave: the records of its own chunk (two per lane)
// and the aggregates of the others, every load issued before the first is waited for, one DPP
// reduction per field.  *own = the tile's own recA.
__device__ __forceinline__ uint4 tile_prefix(const uint2 *recA, const uint4 *agg, size_t ntiles, uint32_t G,
                                             size_t tile, uint32_t n, uint2 *own) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t c = (uint32_t)(tile / kRecChunk), cs = c * (uint32_t)kRecChunk;
    const uint32_t i = (uint32_t)tile - cs, m = (uint32_t)min((size_t)kRecChunk, ntiles - cs);
    // every load unconditional (clamped indices, out-of-range lanes masked afterwards): no
    // exec-masked branches between them for the compiler to put waits in
    uint2 r[kRecChunk / 64];
#pragma unroll
    for (int k = 0; k < kRecChunk / 64; k++) r[k] = recA[cs + min(lane + 64 * k, m - 1)];
    uint32_t f = 0, s = 0, mx = 0, q = n;
    // the aggregates of the chunks before (kept values, runs, last kept) and of the next one (first
    // unkept; a later one only when neither the tile's own chunk after it nor the next chunk has one):
    // the other lanes issue no load.  Every wave of the grid reads these few lines at once, so each
    // line request counts (a load per lane of all G lines, clamped duplicates included, held the move's
    // loads at 4 us); four per lane in flight, blocks of 64 past the first only when G needs them
    auto fold = [&](uint32_t j0) {
        uint4 a[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t j = j0 + 64 * k + lane;
            a[k] = make_uint4(0u, 0u, 0u, 0u);
            if (j0 + 64 * k < G && (j < c || j == c + 1) && j < G) a[k] = agg[(size_t)j * kAggStride];
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t j = j0 + 64 * k + lane;
            const bool before = j < c;
            f += before ? a[k].x : 0u;
            s += before ? a[k].y : 0u;
            mx = max(mx, before ? a[k].z : 0u);
            q = min(q, j == c + 1 && a[k].w ? ~a[k].w : q);
        }
    };
    for (uint32_t j0 = 0; j0 <= c + 1 && j0 < G; j0 += 256) fold(j0);
#pragma unroll
    for (int k = 0; k < kRecChunk / 64; k++) {
        const uint32_t j = lane + 64 * k, t0 = (cs + j) * (uint32_t)kTile;
        if (j < i) {
            f += r[k].x & 0xFFFFu;
            s += r[k].x >> 16;
            const uint32_t l1 = r[k].y & 0xFFFFu;
            if (l1) mx = max(mx, t0 + l1);
        } else if (j > i && j < m) {
            const uint32_t f1 = r[k].y >> 16;
            if (f1 < (uint32_t)kTile) q = min(q, t0 + f1);
        }
    }
    // no unkept value after the tile in its chunk nor in the next: the first later chunk with one
    // (wave-uniform, rare: a chunk of 128 tiles all kept)
    if (c + 2 < G && !__ballot(q < n)) {
        for (uint32_t j0 = c + 2; j0 < G; j0 += 64) {
            const uint32_t j = j0 + lane;
            const uint32_t w = j < G ? agg[(size_t)j * kAggStride].w : 0u;
            q = min(q, w ? ~w : q);
            if (__ballot(q < n)) break;
        }
    }
    const uint2 o0 = make_uint2((uint32_t)__builtin_amdgcn_readlane((int)r[0].x, i & 63),
                                (uint32_t)__builtin_amdgcn_readlane((int)r[0].y, i & 63));
    const uint2 o1 = make_uint2((uint32_t)__builtin_amdgcn_readlane((int)r[1].x, i & 63),
                                (uint32_t)__builtin_amdgcn_readlane((int)r[1].y, i & 63));
    *own = i < 64 ? o0 : o1;
    return make_uint4((uint32_t)__builtin_amdgcn_readlane((int)wave_incl_sum_dpp(f), 63),
                      (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_sum_dpp(s), 63),
                      (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_max_dpp(mx), 63),
                      (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_min_dpp(q), 63));
}
static_assert(kRecChunk == 128, "tile_prefix holds two records per lane");

// The totals (kept values, runs) over all chunks, by one wave.
__device__ __forceinline__ uint2 chunk_totals(const uint4 *agg, uint32_t G) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t f = 0, r = 0;
    for (uint32_t j = lane; j < G; j += 64) {
        const uint4 a = agg[(size_t)j * kAggStride];
        f += a.x;
        r += a.y;
    }
    return make_uint2((uint32_t)__builtin_amdgcn_readlane((int)wave_incl_sum_dpp(f), 63),
                      (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_sum_dpp(r), 63));
}

// tile_prefix for kGP consecutive tiles tb.. (one chunk: tb % kGP == 0), by one wave:
// the records and aggregates are loaded once, reduced once for the first tile (kept values, runs and
// last kept before it; first unkept after the last), and the other tiles' prefixes follow from the
// group's own records.  pre[k] / own[k] for tile tb + k (tiles past ntiles: left alone).  sp_emit's
// four waves then share one set of loads: every wave of the grid reads the same few aggregate lines
// at the same moment, and a quarter of the requests shortens that phase.
constexpr int kGP = kSB / 64;  // tiles per group_prefix (sp_emit's workgroup, sp_count's kCountTpw)
// sp_count's records carry the call's aggregate parity in bit 31 of .x (kept | runs << 16 | parity << 31:
// runs <= 1024 fit 15 bits), so sp_emit learns which of the two aggregate arrays holds this call's sums
// from records it loads anyway — no hot parity word read by every workgroup at once
constexpr uint32_t kRecRunsMask = 0x7FFFu;
__device__ __forceinline__ uint32_t rec_runs(uint32_t x) { return (x >> 16) & kRecRunsMask; }
__device__ __forceinline__ uint32_t wsum_dpp(uint32_t v) { return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_sum_dpp(v), 63); }
__device__ __forceinline__ uint32_t wmax_dpp(uint32_t v) { return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_max_dpp(v), 63); }
__device__ __forceinline__ uint32_t wmin_dpp(uint32_t v) { return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_min_dpp(v), 63); }
__device__ __forceinline__ uint4 readlane4(uint4 v, int l) {
    return make_uint4((uint32_t)__builtin_amdgcn_readlane((int)v.x, l), (uint32_t)__builtin_amdgcn_readlane((int)v.y, l),
                      (uint32_t)__builtin_amdgcn_readlane((int)v.z, l), (uint32_t)__builtin_amdgcn_readlane((int)v.w, l));
}
// The chunk's aggregate against its tiles' records (every record of the chunk is in r[], two per lane):
// sp_count adds exactly the records' kept values and runs and takes the maxima of their edges, so any
// difference means an aggregate that was not zero when sp_count began (or was written since) — the
// stale-aggregate case in which every later place in the wire would be wrong.
__device__ __forceinline__ bool chunk_agrees(const uint2 (&r)[kRecChunk / 64], uint32_t cs, uint32_t m, uint4 oc) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t f = 0, s = 0, lk = 0, fu = 0xFFFFFFFFu;
#pragma unroll
    for (int k = 0; k < kRecChunk / 64; k++) {
        const uint32_t j = lane + 64 * k, t0 = (cs + j) * (uint32_t)kTile;
        if (j < m) {
            const uint32_t F = r[k].x & 0xFFFFu, L1 = r[k].y & 0xFFFFu, FU = r[k].y >> 16;
            f += F;
            s += rec_runs(r[k].x);
            if (F) lk = max(lk, t0 + L1);
            if (FU < (uint32_t)kTile) fu = min(fu, t0 + FU);
        }
    }
    const uint32_t F = wsum_dpp(f), S = wsum_dpp(s), LK = wmax_dpp(lk), FUm = wmin_dpp(fu);
    return oc.x == F && oc.y == S && oc.z == LK && oc.w == (FUm != 0xFFFFFFFFu ? ~FUm : 0u);
}
// agg2: the two aggregate arrays (kAggHalf apart in each chunk's line); *par: which one this call's sp_count
// filled (from the records);
// *ok: the chunk's aggregate agrees with its records (chunk_agrees)
// DEVPAR false: the host knows the parity (hpar; every call on the stream so far was uncaptured) and one array's
// lines are loaded, four 64-chunk instructions as in round 5; true (a graph may have replayed calls on this
// stream, so only the device knows it): both arrays, paired lanes, the parity taken from the records.  The
// paired form holds twice the load registers (66 VGPRs: 7 waves per SIMD, and 8192 waves of a 64 MiB drop
// no longer fit at once: +2.8 us per drop, profiles/r06_s4_*), so it is kept to the streams that need it.
template <bool DEVPAR>
__device__ __forceinline__ void group_prefix(const uint2 *recA, const uint4 *agg2, uint32_t hpar, size_t ntiles,
                                             uint32_t G, size_t tb, uint32_t n, uint4 (&pre)[kGP], uint2 (&own)[kGP],
                                             uint32_t &par, bool &ok) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t c = (uint32_t)(tb / kRecChunk), cs = c * (uint32_t)kRecChunk;
    const uint32_t i0 = (uint32_t)tb - cs, m = (uint32_t)min((size_t)kRecChunk, ntiles - cs);
    uint2 r[kRecChunk / 64];
#pragma unroll
    for (int k = 0; k < kRecChunk / 64; k++) r[k] = recA[cs + min(lane + 64 * k, m - 1)];
#if defined(ONO_EXP_EMIT) && ONO_EXP_EMIT == 6  // measurement only (tools/sp_phases_e6): no records, wrong wire
    r[0] = r[1] = make_uint2(0u, 0u);
#endif
    // both arrays (DEVPAR), issued with the records (the parity comes with them: no load waits for another):
    // lanes 2 i and 2 i + 1 take chunk j0 + i's two aggregates, one line; or this call's array alone, a chunk
    // per lane.  The own chunk's line too, for the check.
    constexpr int kAL = DEVPAR ? 8 : 4;     // instructions over the first 256 chunks
    constexpr int kCPI = DEVPAR ? 32 : 64;  // chunks per instruction
    uint4 a[kAL];
#pragma unroll
    for (int k = 0; k < kAL; k++) {
        const uint32_t j = kCPI * k + (DEVPAR ? lane >> 1 : lane);
        a[k] = make_uint4(0u, 0u, 0u, 0u);
#if !defined(ONO_EXP_EMIT) || ONO_EXP_EMIT != 5  // (measurement only, tools/sp_phases_e5: no aggregates, wrong wire)
        if (kCPI * k < G && kCPI * k <= c + 1 && j <= c + 1 && j < G)
            a[k] = agg2[(size_t)j * kAggStride + (DEVPAR ? (lane & 1) : hpar) * kAggHalf];
#endif
    }
    par = DEVPAR ? (uint32_t)__builtin_amdgcn_readfirstlane((int)r[0].x) >> 31 : hpar;
    const uint4 *agg = agg2 + par * kAggHalf;
    const bool mine = !DEVPAR || (lane & 1u) == par;  // the lane holds this call's array
    uint4 oc;  // the own chunk's aggregate
    if (c < (uint32_t)(kCPI * kAL)) {
        uint4 o4 = a[0];
#pragma unroll
        for (int k = 1; k < kAL; k++)
            if (c / kCPI == (uint32_t)k) o4 = a[k];
        oc = readlane4(o4, (int)(DEVPAR ? 2 * (c & 31) + par : c & 63));
    } else {
        uint32_t ca = c;
        asm volatile("" : "+v"(ca));  // (a vector load)
        oc = agg[(size_t)ca * kAggStride];
    }
    ok = chunk_agrees(r, cs, m, oc);
    uint32_t f = 0, s = 0, mx = 0, q = n;
    for (uint32_t j0 = 256; j0 < c; j0 += 64) {  // chunks before past the first 256 (G > 256: n > 2^26)
        const uint32_t j = j0 + lane;
        const uint4 b = j < c ? agg[(size_t)j * kAggStride] : make_uint4(0u, 0u, 0u, 0u);
        f += b.x;
        s += b.y;
        mx = max(mx, b.z);
    }
    if (c + 1 >= 256 && c + 1 < G && lane == 0) {
        const uint32_t w = agg[(size_t)(c + 1) * kAggStride].w;
        q = w ? ~w : q;
    }
#pragma unroll
    for (int k = 0; k < kAL; k++) {
        const uint32_t j = kCPI * k + (DEVPAR ? lane >> 1 : lane);
        const bool before = mine && j < c;
        f += before ? a[k].x : 0u;
        s += before ? a[k].y : 0u;
        mx = max(mx, before ? a[k].z : 0u);
        q = min(q, mine && j == c + 1 && a[k].w ? ~a[k].w : q);
    }
    const uint32_t ilast = i0 + kGP - 1;
#pragma unroll
    for (int k = 0; k < kRecChunk / 64; k++) {
        const uint32_t j = lane + 64 * k, t0 = (cs + j) * (uint32_t)kTile;
        if (j < i0) {
            f += r[k].x & 0xFFFFu;
            s += rec_runs(r[k].x);
            const uint32_t l1 = r[k].y & 0xFFFFu;
            if (l1) mx = max(mx, t0 + l1);
        } else if (j > ilast && j < m) {
            const uint32_t f1 = r[k].y >> 16;
            if (f1 < (uint32_t)kTile) q = min(q, t0 + f1);
        }
    }
    if (c + 2 < G && !__ballot(q < n)) {  // as tile_prefix: the first later chunk with an unkept value
        for (uint32_t j0 = c + 2; j0 < G; j0 += 64) {
            const uint32_t j = j0 + lane;
            const uint32_t w = j < G ? agg[(size_t)j * kAggStride].w : 0u;
            q = min(q, w ? ~w : q);
            if (__ballot(q < n)) break;
        }
    }
    uint32_t F = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_sum_dpp(f), 63);
    uint32_t S = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_sum_dpp(s), 63);
    uint32_t MX = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_max_dpp(mx), 63);
    uint32_t Q = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_min_dpp(q), 63);
    uint2 rg[kGP];
#pragma unroll
    for (int k = 0; k < kGP; k++) {  // the group's own records (i0 + k < 128: one of the two per lane)
        const uint32_t i = i0 + k;
        const uint2 lo2 = make_uint2((uint32_t)__builtin_amdgcn_readlane((int)r[0].x, i & 63),
                                     (uint32_t)__builtin_amdgcn_readlane((int)r[0].y, i & 63));
        const uint2 hi2 = make_uint2((uint32_t)__builtin_amdgcn_readlane((int)r[1].x, i & 63),
                                     (uint32_t)__builtin_amdgcn_readlane((int)r[1].y, i & 63));
        rg[k] = i < 64 ? lo2 : hi2;
        own[k] = rg[k];
    }
    uint32_t Qk[kGP];
    Qk[kGP - 1] = Q;
#pragma unroll
    for (int k = kGP - 2; k >= 0; k--) {  // first unkept after tile i0 + k: tile i0 + k + 1's, or later
        const uint32_t i = i0 + k + 1, f1 = rg[k + 1].y >> 16;
        Qk[k] = i < m && f1 < (uint32_t)kTile ? min(Qk[k + 1], (cs + i) * (uint32_t)kTile + f1) : Qk[k + 1];
    }
#pragma unroll
    for (int k = 0; k < kGP; k++) {
        pre[k] = make_uint4(F, S, MX, Qk[k]);
        const uint32_t l1 = rg[k].y & 0xFFFFu;
        F += rg[k].x & 0xFFFFu;
        S += rec_runs(rg[k].x);
        if (l1) MX = max(MX, (cs + i0 + k) * (uint32_t)kTile + l1);
    }
}

// One tile's slot -> its place in the wire, in 16-B chunks of the
// destination: the range starts O units (0..7, uniform) into its first
// aligned chunk, so destination chunk c takes slot units 8c - O .. 8c - O + 7
// — the last O units of slot chunk c - 1 (the lane before, by DPP) and the
// first 8 - O of slot chunk c (this lane).  Whole chunks are one 16-B store;
// the range's first and last chunk (shared with the neighbouring tiles) are
// stored unit by unit.  The two header fields completed from other tiles are
// stored after these by one lane (same wave, same addresses, later in program
// order).
constexpr int kMoveBatch = 2;  // 16-B slot chunks per lane loaded up front: 1024 units per wave
__device__ __forceinline__ uint4 ldn4(const uint4 *p) {
    const u4v r = __builtin_nontemporal_load((const u4v *)p);
    return make_uint4(r.x, r.y, r.z, r.w);
}
__device__ __forceinline__ uint4 lane_before4(uint4 v) {
    return make_uint4(lane_before(v.x), lane_before(v.y), lane_before(v.z), lane_before(v.w));
}
template <int O>
__device__ __forceinline__ void move_chunks(const uint4 *src4, uint4 (&v)[kMoveBatch], uint32_t nu16, uint16_t *base16) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nchunks = nu16 ? (O + nu16 + 7) / 8 : 0;
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
            const bool whole = c * 8 >= (uint32_t)O && (size_t)c * 8 + 8 - O <= nu16;
            if (whole) {  // (write-through stores measured slower here: 23 vs 11 us)
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

// One tile's slot to its place (sp_move).
__device__ __forceinline__ void move_tile(const uint16_t *__restrict__ img, const uint2 *__restrict__ recA,
                                          const uint2 *__restrict__ recB, const uint4 *__restrict__ agg, size_t ntiles,
                                          uint32_t G, size_t n, uint8_t *__restrict__ buf, size_t cap,
                                          uint64_t *__restrict__ host_tot, size_t tile) {
    const uint32_t lane = threadIdx.x & 63;
    SP_CLOCK(sp_t0);
    const uint4 *src4 = (const uint4 *)(img + tile * kSlotU16);
    uint4 v[kMoveBatch];
#pragma unroll
    for (int k = 0; k < kMoveBatch; k++) v[k] = ldn4(src4 + lane + 64 * k);
    const uint2 hb = recB[tile];
    uint2 a;
    const uint4 p = tile_prefix(recA, agg, ntiles, G, tile, (uint32_t)n, &a);
#ifdef ONO_SP_STAMP
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the slot's first loads landed too)
    SP_CLOCK(sp_tm);
#endif
    const uint32_t F = a.x & 0xFFFFu, R = a.x >> 16, nu16 = 4 * R + F;
    const uint32_t tile0 = (uint32_t)(tile * kTile), tend = (uint32_t)min((size_t)tile0 + kTile, n);
    // the first run's offset and the last run's length (R > 0), completed
    const uint32_t off0 = (hb.y & 0xFFFFu) + (tile0 - p.z);
    const uint32_t lenl = (hb.y >> 16) + (tile0 + (a.y & 0xFFFFu) == tend ? p.w - tend : 0u);
    const uint32_t c0 = hb.x & 0xFFFFu, hl = hb.x >> 16;
    uint8_t *dst = buf + 8 + 8 * (size_t)p.y + 2 * (size_t)p.x;
    if (8 + 8 * (size_t)p.y + 2 * ((size_t)p.x + nu16) > cap) {  // never past the buffer (uniform)
        if (lane == 0) drop_error(host_tot, kDropErrRange);
        return;
    }
    const uint32_t O = (uint32_t)__builtin_amdgcn_readfirstlane((int)(((uintptr_t)dst & 15u) >> 1));
    uint16_t *base16 = (uint16_t *)(dst - 2 * O);
    switch (O) {
    case 0: move_chunks<0>(src4, v, nu16, base16); break;
    case 1: move_chunks<1>(src4, v, nu16, base16); break;
    case 2: move_chunks<2>(src4, v, nu16, base16); break;
    case 3: move_chunks<3>(src4, v, nu16, base16); break;
    case 4: move_chunks<4>(src4, v, nu16, base16); break;
    case 5: move_chunks<5>(src4, v, nu16, base16); break;
    case 6: move_chunks<6>(src4, v, nu16, base16); break;
    default: move_chunks<7>(src4, v, nu16, base16); break;
    }
    if (R && lane == 0) {  // the first run's offset (units c0, c0 + 1) and the last run's length (hl + 2, + 3)
        uint16_t *r16 = base16 + O;
        r16[c0] = (uint16_t)off0;
        r16[c0 + 1] = (uint16_t)(off0 >> 16);
        r16[hl + 2] = (uint16_t)lenl;
        r16[hl + 3] = (uint16_t)(lenl >> 16);
    }
#ifdef ONO_SP_STAMP
    sp_stamp(g_sp_stamp_mov, tile, sp_t0, sp_tm);
#endif
}

// sp_emit's staged range (LDS, 16-B aligned, at least one spare block past nu16 units) to its place in
// the wire in 16-B destination chunks, as move_chunks does from a slot
typedef __attribute__((address_space(3))) uint4 lds_u4;
template <int O>
__device__ __forceinline__ void stage_out(const lds_u4 *src4, uint32_t nu16, uint16_t *base16) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nchunks = nu16 ? (O + nu16 + 7) / 8 : 0;
    uint4 carry = make_uint4(0, 0, 0, 0);
    for (uint32_t c0b = 0; c0b < nchunks; c0b += 64) {
        const uint32_t c = c0b + lane;
        uint4 own = make_uint4(0, 0, 0, 0);
        if (c < nchunks) {
            const lds_u4 &q = src4[c];
            own = make_uint4(q.x, q.y, q.z, q.w);
        }
        const uint4 up = lane_before4(own);
        const uint4 prev = lane ? up : carry;
        const uint32_t C[8] = {prev.x, prev.y, prev.z, prev.w, own.x, own.y, own.z, own.w};
        uint32_t o[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {  // out word j = concat units 8 - O + 2j, + 1
            const int sft = 8 - O + 2 * j;
            if (sft % 2 == 0) o[j] = C[sft / 2];
            else o[j] = __builtin_amdgcn_alignbit(C[(sft + 1) / 2], C[(sft - 1) / 2], 16);
        }
        const bool whole = c * 8 >= (uint32_t)O && (size_t)c * 8 + 8 - O <= nu16;
        if (whole) {
            const u4v ov = {o[0], o[1], o[2], o[3]};
#if defined(ONO_EXP_EMIT) && ONO_EXP_EMIT == 3  // measurement only (tools/sp_phases_e3): plain stores
            *(u4v *)(base16 + 8 * (size_t)c) = ov;
#else
            __builtin_nontemporal_store(ov, (u4v *)(base16 + 8 * (size_t)c));
#endif
#if defined(ONO_EXP_EMIT) && ONO_EXP_EMIT == 4  // measurement only (tools/sp_phases_e4): no boundary stores
        } else if (false) {
#else
        } else if (c < nchunks) {  // the range's first / last chunk (shared with the neighbouring tiles)
#endif
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const int64_t u = (int64_t)c * 8 + i - O;
                if (u >= 0 && u < (int64_t)nu16) base16[8 * (size_t)c + i] = (uint16_t)(o[i / 2] >> (16 * (i % 2)));
            }
        }
        carry = readlane4(own, 63);
    }
}

// One wave per tile: its records and prefix, the slot's first 1024 units (most tiles' whole image)
// issued at the same time, then the move.  (Two or four tiles per wave in turn measured slower in
// round 4: 35.7 / 39.2 vs 33.9 us per drop.)
// Block 0 also writes the u64 total length and publishes the wire length.
__global__ __launch_bounds__(kSB) void sp_move(
    const uint16_t *__restrict__ img, const uint2 *__restrict__ recA, const uint2 *__restrict__ recB,
    const uint4 *__restrict__ agg, size_t ntiles, size_t n, uint8_t *__restrict__ buf, size_t cap,
    uint64_t *__restrict__ host_tot, uint64_t *__restrict__ nbytes_out) {
    const uint32_t G = (uint32_t)((ntiles + kRecChunk - 1) / kRecChunk);
    if (blockIdx.x == 0 && threadIdx.x < 64) {  // u64 LE total length, as four 2-byte stores (buf is 2-B aligned)
        const uint2 t = chunk_totals(agg, G);
        if (threadIdx.x == 0) {
            for (int q = 0; q < 4; q++) *(uint16_t *)(buf + 2 * q) = (uint16_t)((uint64_t)n >> (16 * q));
            const uint64_t F = t.x, R = t.y, nb = 8 + 8 * R + 2 * F;
            if (nb > cap) drop_error(host_tot, kDropErrRange);
            if (nbytes_out) {
                *nbytes_out = nb <= cap ? nb : ~0ull;  // the stream-ordered form: nothing crosses PCIe
            } else {
                host_tot[0] = F;  // the blocking form: the wire length's terms for the host (host-mapped)
                host_tot[1] = R;
            }
        }
    }
    // wave-uniform (readfirstlane): scalar base addresses and branches
    const size_t tile = (size_t)__builtin_amdgcn_readfirstlane((int)(blockIdx.x * (kSB / 64) + (threadIdx.x >> 6)));
    if (tile < ntiles) move_tile(img, recA, recB, agg, ntiles, G, n, buf, cap, host_tot, tile);
}


// -------------------------------------------------- count + emit encoder ----
// Round 5 (the 64 MiB drop): two launches without the slot image, the default above
// kDropOneLaunchTiles (ONO_DROP_FORM=image keeps sp_image + sp_move).  sp_count reads g once, one wave
// per tile with 32 values per lane: the keep flags as one 32-bit word per lane (256 B per tile, the
// "mask"), the tile's kept values as compact f16 in its slot of cv, the tile's record (recA, as sp_image
// writes it) and the chunk aggregates (four tiles per workgroup round, one set of atomics).  sp_emit,
// one wave per tile: the workgroup's four prefixes from one wave (group_prefix, through LDS), the run
// starts and the thread's place from the mask and one DPP scan, the compact values into LDS, and the
// tile's range built in an LDS stage — each header with its global offset and length (the previous
// kept index and the next unkept one from the thread, the wave, or the prefix P / Q), so no field is
// completed later — then stored in 16-B chunks.  Traffic: 4 N + the wire + the mask (N / 8, written
// and read) + the kept values' f16 (written and read).  29.4-29.9 vs 33.3-34.1 us per 64 MiB drop for
// the image form (profiles/r05_final_e_ab.txt; DESIGN.md §3 "count + emit").
constexpr int kCW = 32;                // values per lane: one wave per 2048-value tile
static_assert(64 * kCW == kTile, "a wave holds a tile");
constexpr int kCountTpw = kGP;        // tiles per sp_count workgroup (a wave each): one set of atomics
static_assert(kRecChunk % kCountTpw == 0, "a workgroup's tiles share one chunk aggregate");

template <bool FULL>
__device__ __forceinline__ void load_w32(const float *__restrict__ g, size_t n, size_t tile, float (&x)[kCW]) {
    const size_t base = tile * kTile + (size_t)(threadIdx.x & 63) * kCW;
    if (FULL) {
#pragma unroll
        for (int q = 0; q < kCW / 4; q++) {
            const f4s a = *((const f4s *)(g + base) + q);
            x[4 * q] = a.x; x[4 * q + 1] = a.y; x[4 * q + 2] = a.z; x[4 * q + 3] = a.w;
        }
    } else {
#pragma unroll
        for (int e = 0; e < kCW; e++) x[e] = base + e < n ? g[base + e] : 0.0f;
    }
}
// the lane's valid values as a mask (the last tile may end inside the lane)
__device__ __forceinline__ uint32_t valid_w32(size_t n, size_t tile) {
    const size_t base = tile * kTile + (size_t)(threadIdx.x & 63) * kCW;
    return base >= n ? 0u : (n - base >= (size_t)kCW ? 0xFFFFFFFFu : (1u << (n - base)) - 1u);
}
// A workgroup takes kCountTpw tiles at a time (a wave each) and strides over the tiles by the grid
// (count_grid: a few workgroups per CU), the wave's next tile loaded while the current one is
// counted and stored.  One tile per wave in a single pass (every workgroup resident at once, 8 KiB
// requested per wave at the start) read g at about 4.5 TB/s: the one-shot shape of DESIGN §2.
//
// The compaction walks only the lanes' kept values — the lane's 32 values as f16 in its LDS row
// (80 B apart: the 16-B writes conflict-free), then max-over-lanes-of-kept steps of one LDS read and one
// write each (a lane out of values writes its dummy slot) — 1 us per drop less than 32 predicated
// LDS writes per lane (profiles/r05_s67_*).
constexpr int kCRow = 40;  // u16 per padded lane row (64 B of values + 16 B)
typedef _Float16 h2s __attribute__((ext_vector_type(2)));
typedef float f2s __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_f16(float a, float b) {  // v_cvt_pk_f16_f32: the to_f16_sp rounding
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f2s){a, b}, h2s));
}
__global__ __launch_bounds__(kSB) void sp_count(const float *__restrict__ g, size_t n, size_t ntiles, float t,
                                                const float *t_dev, bool vec, uint32_t *__restrict__ mask,
                                                uint16_t *__restrict__ cv, uint2 *__restrict__ recA, uint4 *agg2,
                                                uint32_t gcap, uint32_t *state) {
    // per round's parity (thread 0 reads one round's while a faster wave writes the next one's)
    __shared__ uint32_t s_fr[2][kCountTpw][2], s_lk[2][kCountTpw], s_fu[2][kCountTpw];
    // a wave's compact values (+ a dummy slot per lane)
    __shared__ __attribute__((aligned(16))) uint16_t s_cv[kCountTpw][kTile + 64];
    __shared__ __attribute__((aligned(16))) uint16_t s_row[kCountTpw][64 * kCRow];  // the lanes' values as f16
    SP_CLOCK(sp_t0);
    if (t_dev) t = *t_dev;
    // The two aggregate arrays alternate by a parity kept on the device (state[0], flipped by sp_emit's
    // workgroup 0 once every wave has read this call's sums): this call adds into agg2[par] — zeroed by
    // the previous call — and zeroes the other one for the next call.  A replayed graph follows it as
    // an uncaptured call does (a host-side parity would be frozen into the graph).
    // (read after the first tile's loads are issued: the word is one line every workgroup reads at once)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const size_t step = (size_t)gridDim.x * kCountTpw;
#ifdef ONO_SP_STAMP
    uint64_t sp_tm = sp_t0;
#endif
    // the wave's tile's values and the value before the tile (lane 0's previous bit), loaded ahead
    float x[kCW];
    float xb = 0.0f;
    auto load = [&](size_t tl) {
        if (tl >= ntiles) return;
        if (vec && (tl + 1) * kTile <= n) load_w32<true>(g, n, tl, x);
        else load_w32<false>(g, n, tl, x);
        uint32_t a = (uint32_t)(tl ? tl * kTile - 1 : 0);
        asm volatile("" : "+v"(a));  // (a vector load)
        xb = g[a];
    };
    size_t tile = (size_t)blockIdx.x * kCountTpw + wave;
    load(tile);
    const uint32_t apar = state[0] & 1u;
    uint4 *agg = agg2 + apar * kAggHalf, *agg_next = agg2 + (apar ^ 1u) * kAggHalf;
    if (blockIdx.x == 0 && threadIdx.x == 0) state[1] = apar;  // (sp_totals_out's)
    for (size_t i = (size_t)blockIdx.x * kSB + threadIdx.x; i < gcap; i += (size_t)gridDim.x * kSB)
        agg_next[i * kAggStride] = make_uint4(0u, 0u, 0u, 0u);
    int par = 0;
    for (size_t b0 = (size_t)blockIdx.x * kCountTpw; b0 < ntiles; b0 += step, tile += step) {
        uint32_t F = 0, R = 0, LK = 0, FU = kTile;
        if (tile < ntiles) {
            const uint32_t valid = valid_w32(n, tile);
#ifdef ONO_SP_STAMP
            if (b0 == (size_t)blockIdx.x * kCountTpw) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                sp_tm = __builtin_amdgcn_s_memrealtime();
            }
#endif
            uint32_t keep = 0;
#pragma unroll
            for (int e = 0; e < kCW; e++) keep |= kept(x[e], t) ? 1u << e : 0u;
            keep &= valid;
            uint32_t prev = lane_before(keep >> 31);
            if (lane == 0) prev = tile && kept(xb, t) ? 1u : 0u;
            const uint32_t start = keep & ~((keep << 1) | prev), unk = valid & ~keep;
#if defined(ONO_EXP_COUNT) && ONO_EXP_COUNT >= 2  // measurement only (tools/sp_phases_c2): the loads and the flags
            if (lane == 0) recA[tile] = make_uint2(keep, start);
            load(tile + step);
            continue;
#endif
            mask[tile * 64 + lane] = keep;
            const uint32_t lo = (uint32_t)lane * kCW;
            // the tile's kept values as f16, compact, in its slot of cv (in order: the lanes' exclusive
            // prefix), through LDS so that the stores are 16-B pieces (2-byte stores from every lane: +5 us
            // per drop); the wave's next tile requested once its values are in LDS
            const uint32_t kc = (uint32_t)__popc(keep), incl = wave_incl_sum_dpp(kc);
            F = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
            typedef __attribute__((address_space(3))) uint16_t lds_u16;
            lds_u16 *sc = (lds_u16 *)s_cv[wave];
            uint32_t cp = incl - kc;
#ifndef ONO_EXP_COUNT  // (measurement builds: no compaction)
            typedef __attribute__((address_space(3))) u4v lds_w4;
            lds_u16 *rw = (lds_u16 *)s_row[wave] + lane * kCRow;
#pragma unroll
            for (int q = 0; q < kCW / 8; q++) {
                u4v w;
                w.x = pk_f16(x[8 * q], x[8 * q + 1]);
                w.y = pk_f16(x[8 * q + 2], x[8 * q + 3]);
                w.z = pk_f16(x[8 * q + 4], x[8 * q + 5]);
                w.w = pk_f16(x[8 * q + 6], x[8 * q + 7]);
                ((lds_w4 *)rw)[q] = w;
            }
            const uint32_t steps = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_max_dpp(kc), 63);
            uint32_t m = keep;
            for (uint32_t k = 0; k < steps; k++) {
                const bool has = m != 0u;
                const uint32_t e = has ? (uint32_t)__ffs(m) - 1u : 0u;
                const uint16_t v = rw[e];
                sc[has ? cp : (uint32_t)kTile + lane] = v;
                cp += has ? 1u : 0u;
                m &= m - 1u;
            }
#endif
            load(tile + step);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            typedef __attribute__((address_space(3))) const u4v lds_cw4;
            const lds_cw4 *s4 = (const lds_cw4 *)s_cv[wave];
            u4v *d4 = (u4v *)(cv + tile * kTile);
            for (uint32_t c = (uint32_t)lane; c < (F + 7) / 8; c += 64) d4[c] = s4[c];
            R = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_sum_dpp((uint32_t)__popc(start)), 63);
            LK = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_max_dpp(keep ? lo + 32u - (uint32_t)__clz(keep) : 0u), 63);
            FU = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_min_dpp(unk ? lo + (uint32_t)(__ffs(unk) - 1) : (uint32_t)kTile), 63);
            if (lane == 0) recA[tile] = make_uint2(F | R << 16 | apar << 31, LK | FU << 16);  // (group_prefix)
        }
        if (lane == 0) {
            s_fr[par][wave][0] = F;
            s_fr[par][wave][1] = R;
            s_lk[par][wave] = F ? (uint32_t)(tile * kTile) + LK : 0u;  // global last kept + 1 (0: none)
            s_fu[par][wave] = FU < (uint32_t)kTile ? ~((uint32_t)(tile * kTile) + FU) : 0u;  // complemented (0: none)
        }
        __syncthreads();
#ifdef ONO_EXP_NOATOM  // measurement only (tools/sp_phases_na): sp_count without its chunk atomics, wrong wire
        if (false) {
#else
        if (threadIdx.x == 0) {
#endif
            uint64_t fr = 0;
            uint32_t lk = 0, nfu = 0;
#pragma unroll
            for (int w = 0; w < kCountTpw; w++) {
                fr += (uint64_t)s_fr[par][w][0] | (uint64_t)s_fr[par][w][1] << 32;
                lk = max(lk, s_lk[par][w]);
                if (!nfu) nfu = s_fu[par][w];  // the first tile's first unkept
            }
            uint32_t *a = (uint32_t *)(agg + (b0 / kRecChunk) * kAggStride);
            if (fr) {
                atomicAdd((unsigned long long *)a, (unsigned long long)fr);
                atomicMax(a + 2, lk);
            }
            if (nfu) atomicMax(a + 3, nfu);
        }
        par ^= 1;  // (a round's words are written again two rounds on, after the next round's barrier)
    }
#ifdef ONO_SP_STAMP
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x < 64) sp_stamp(g_sp_stamp_img, blockIdx.x, sp_t0, sp_tm);  // mid: the wave's first values loaded
#endif
}

// STAGE: a tile's range of at most kEmitStage units is built in LDS and stored in 16-B chunks (a longer
// one, and every range without STAGE, unit by unit straight to the wire)
constexpr int kEmitStage = 1504;  // units (+16 spare); with kEmitVals values and the shared prefixes 20 KB: 8 workgroups per CU
constexpr int kEmitVals = 1024;
#ifndef ONO_EMIT_SPEC
#define ONO_EMIT_SPEC 256
#endif
constexpr int kEmitSpec = ONO_EMIT_SPEC;  // values loaded speculatively (10 % kept: 205 +- 14 per tile)
template <bool STAGE, bool DEVPAR>
__global__ __launch_bounds__(kSB) __attribute__((amdgpu_waves_per_eu(8))) void sp_emit(const uint16_t *__restrict__ cv, size_t n, size_t ntiles,
                                               const uint32_t *__restrict__ mask, const uint2 *__restrict__ recA,
                                               const uint4 *__restrict__ agg2, uint32_t *__restrict__ state,
                                               uint32_t hpar, uint8_t *__restrict__ buf, size_t cap,
                                               uint64_t *__restrict__ host_tot, uint64_t *__restrict__ nbytes_out) {
    __shared__ __attribute__((aligned(16))) uint16_t vals[kSB / 64][kEmitVals];  // per wave: the tile's compact values
    __shared__ __attribute__((aligned(16))) uint16_t stage[STAGE ? kSB / 64 : 1][STAGE ? kEmitStage + 16 : 8];
    SP_CLOCK(sp_t0);
    const uint32_t G = (uint32_t)((ntiles + kRecChunk - 1) / kRecChunk);
    const int wave = threadIdx.x >> 6;
    // block 0's first wave, first: the totals, the header and the parity flip (the array: the host's parity,
    // or the one sp_count's workgroup 0 named in state[1])
    if (blockIdx.x == 0 && wave == 0) {
        const uint32_t par = DEVPAR ? state[1] & 1u : hpar;
        const uint2 t = chunk_totals(agg2 + par * kAggHalf, G);
        if ((threadIdx.x & 63) == 0) {  // u64 LE total length, as four 2-byte stores (buf 2-B aligned, cap >= 8)
            for (int q = 0; q < 4; q++) *(uint16_t *)(buf + 2 * q) = (uint16_t)((uint64_t)n >> (16 * q));
            const uint64_t F = t.x, R = t.y, nb = 8 + 8 * R + 2 * F;
            const bool good = nb <= cap;  // (a wire past the buffer: no length, an error)
            if (nbytes_out) *nbytes_out = good ? nb : ~0ull;
            else { host_tot[0] = F; host_tot[1] = R; }
            if (!good) drop_error(host_tot, kDropErrRange);
            state[0] = par ^ 1u;  // the next call's sp_count adds into the other array (sp_emit reads none)
        }
    }
    const size_t tb = (size_t)blockIdx.x * kCountTpw;  // the workgroup's first tile (< ntiles)
    const size_t tile = (size_t)__builtin_amdgcn_readfirstlane((int)(tb + wave));
    const bool live = tile < ntiles;  // (wave-uniform; every wave reaches the barrier below)
    const size_t tl = live ? tile : tb;  // (a dead wave's loads: the group's first tile, unused)
    const uint32_t lane = threadIdx.x & 63, lo = lane * kCW;
    const uint32_t tile0 = (uint32_t)(tile * kTile);
    // every load first: the lane's mask word, the bit before the tile, the values, the prefix's records
    const uint32_t keep = mask[tl * 64 + lane];
    uint32_t pa = (uint32_t)(tl ? tl * 64 - 1 : 0);
    asm volatile("" : "+v"(pa));  // (a vector load)
    const uint32_t pw = mask[pa];
    // the first kEmitSpec of the tile's compact values, before the count is known (sp_count's slot;
    // the rest, rarely there, after it)
    const u4v *src = (const u4v *)(cv + tl * kTile);
    u4v v0 = {0u, 0u, 0u, 0u};
    if (lane < kEmitSpec / 8) v0 = src[lane];
    // the prefixes of the workgroup's tiles (F0, R0, P, Q) and their records, by wave 0, through LDS
    __shared__ uint4 s_pre[kCountTpw];
    __shared__ uint2 s_own[kCountTpw];
    __shared__ uint32_t s_ok;
    if (wave == 0) {
        uint4 pre[kCountTpw];
        uint2 ow[kCountTpw];
        uint32_t par;
        bool ok;
        group_prefix<DEVPAR>(recA, agg2, hpar, ntiles, G, tb, (uint32_t)n, pre, ow, par, ok);
        if (lane == 0) {
#pragma unroll
            for (int k = 0; k < kCountTpw; k++) {
                s_pre[k] = pre[k];
                s_own[k] = ow[k];
            }
            s_ok = ok;
        }
        (void)par;
    }
    const uint32_t valid = valid_w32(n, tile), unk = valid & ~keep;
    uint32_t prev = lane_before(keep >> 31);
    if (lane == 0) prev = tile ? pw >> 31 : 0u;
    const uint32_t start = keep & ~((keep << 1) | prev);
    // the thread's place: kept values and runs of the lanes before it (one DPP scan of both)
    const uint32_t ownc = (uint32_t)__popc(keep) | (uint32_t)__popc(start) << 16;
    const uint32_t exc = wave_incl_sum_dpp(ownc) - ownc;
    const uint32_t ef = exc & 0xFFFFu, es = exc >> 16;
    // the nearest kept value before the lane and unkept one after it, within the tile (tile-local + 1 /
    // index; 0 / kTile: none)
    const uint32_t k1 = keep ? lo + 32u - (uint32_t)__clz(keep) : 0u;
    const uint32_t u1 = unk ? lo + (uint32_t)(__ffs(unk) - 1) : (uint32_t)kTile;
    const uint64_t mk = __ballot(keep != 0), mu = __ballot(unk != 0);
    const uint64_t below = (1ull << lane) - 1ull, above = ~below & ~(1ull << lane);
    const uint64_t kbm = mk & below, uam = mu & above;
    const int lk = kbm ? 63 - __clzll((long long)kbm) : 0, lu = uam ? __ffsll((unsigned long long)uam) - 1 : 0;
    const uint32_t ykb = (uint32_t)__shfl((int)k1, lk, 64), yua = (uint32_t)__shfl((int)u1, lu, 64);
    const uint32_t kept1_before = kbm ? ykb : 0u, unkept_after = uam ? yua : (uint32_t)kTile;
    __syncthreads();
    if (!live) return;  // (no barrier below)
    const uint4 p = s_pre[wave];
    const uint2 own = s_own[wave];
    // the tile's range inside the buffer, from aggregates that agree with their records — else no store
    // at all (a wrong prefix never becomes an address), and the call reports the error (uniform)
    {
        const size_t end = 8 + 2 * (4 * (size_t)p.y + (size_t)p.x + 4 * (size_t)rec_runs(own.x) + (own.x & 0xFFFFu));
        if (!s_ok || end > cap) {
            if (lane == 0) drop_error(host_tot, s_ok ? kDropErrRange : kDropErrStale);
            return;
        }
    }
    // the tile's compact values (sp_count's slot) into LDS in 16-B pieces, read below by position: the
    // lane's k-th kept value is the tile's (ef + k)-th
    const uint32_t Ft = own.x & 0xFFFFu;
    const bool fits = Ft <= (uint32_t)kEmitVals;  // (uniform) else the values are read from cv one by one
    if (fits) {
        typedef __attribute__((address_space(3))) u4v lds_w4;
        lds_w4 *vw = (lds_w4 *)vals[wave];
        if (lane < (Ft + 7) / 8 && lane < kEmitSpec / 8) vw[lane] = v0;
        for (uint32_t c = lane + (lane < kEmitSpec / 8 ? 64 : 0); c < (Ft + 7) / 8; c += 64) vw[c] = src[c];
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
    }
#ifdef ONO_SP_STAMP
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    SP_CLOCK(sp_tm);  // the mask, the prefix and the values in
#endif
    typedef __attribute__((address_space(3))) const uint16_t lds_cu16;
    lds_cu16 *v16 = (lds_cu16 *)vals[wave] + ef;
    const uint16_t *g16 = cv + tile * kTile + ef;
    uint16_t *w16 = (uint16_t *)(buf + 8);
    const size_t U0 = 4 * (size_t)p.y + (size_t)p.x;  // the tile's first unit
    const uint32_t nu16 = 4 * rec_runs(own.x) + (own.x & 0xFFFFu);
    if (STAGE && fits && nu16 <= (uint32_t)kEmitStage) {  // (uniform)
        typedef __attribute__((address_space(3))) uint16_t lds_u16;
        lds_u16 *st = (lds_u16 *)stage[STAGE ? wave : 0];
        uint32_t lp = 4 * es + ef, kv = 0;  // the lane's first unit within the tile's range; its kept values
        for (uint32_t m = keep; m; m &= m - 1u) {
            const uint32_t e = (uint32_t)__ffs(m) - 1u, gi = tile0 + lo + e;
            if (start >> e & 1u) {
                const uint32_t kb = keep & ((1u << e) - 1u);
                const uint32_t prev_end = kb ? tile0 + lo + 32u - (uint32_t)__clz(kb)
                                             : (kept1_before ? tile0 + kept1_before : p.z);
                const uint32_t ua = e == 31u ? 0u : unk >> (e + 1u);
                const uint32_t end = ua ? gi + 1u + (uint32_t)__ffs(ua) - 1u
                                        : (unkept_after < (uint32_t)kTile ? tile0 + unkept_after : p.w);
                const uint32_t off = gi - prev_end, len = end - gi;
                st[lp] = (uint16_t)off;
                st[lp + 1] = (uint16_t)(off >> 16);
                st[lp + 2] = (uint16_t)len;
                st[lp + 3] = (uint16_t)(len >> 16);
                lp += 4;
            }
            st[lp++] = v16[kv++];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's stage writes, before its reads
        __builtin_amdgcn_wave_barrier();
        uint8_t *dst = buf + 8 + 2 * U0;
        const uint32_t O = (uint32_t)__builtin_amdgcn_readfirstlane((int)(((uintptr_t)dst & 15u) >> 1));
        uint16_t *base16 = (uint16_t *)(dst - 2 * O);
        const lds_u4 *s4 = (const lds_u4 *)stage[STAGE ? wave : 0];
#if defined(ONO_EXP_EMIT) && ONO_EXP_EMIT == 1  // measurement only (tools/sp_phases_e1): no wire stores
        if (nu16 != 0xFFFFFFFFu) return;
#endif
        switch (O) {
        case 0: stage_out<0>(s4, nu16, base16); break;
        case 1: stage_out<1>(s4, nu16, base16); break;
        case 2: stage_out<2>(s4, nu16, base16); break;
        case 3: stage_out<3>(s4, nu16, base16); break;
        case 4: stage_out<4>(s4, nu16, base16); break;
        case 5: stage_out<5>(s4, nu16, base16); break;
        case 6: stage_out<6>(s4, nu16, base16); break;
        default: stage_out<7>(s4, nu16, base16); break;
        }
#ifdef ONO_SP_STAMP
        sp_stamp(g_sp_stamp_mov, tile, sp_t0, sp_tm);
#endif
        return;
    }
    size_t pos = U0 + 4 * (size_t)es + ef;  // the lane's first unit
    uint32_t kv = 0;
    for (uint32_t m = keep; m; m &= m - 1u) {
        const uint32_t e = (uint32_t)__ffs(m) - 1u, gi = tile0 + lo + e;
        if (start >> e & 1u) {
            const uint32_t kb = keep & ((1u << e) - 1u);
            const uint32_t prev_end = kb ? tile0 + lo + 32u - (uint32_t)__clz(kb)
                                         : (kept1_before ? tile0 + kept1_before : p.z);
            const uint32_t ua = e == 31u ? 0u : unk >> (e + 1u);
            const uint32_t end = ua ? gi + 1u + (uint32_t)__ffs(ua) - 1u
                                    : (unkept_after < (uint32_t)kTile ? tile0 + unkept_after : p.w);
            const uint32_t off = gi - prev_end, len = end - gi;
            w16[pos] = (uint16_t)off;
            w16[pos + 1] = (uint16_t)(off >> 16);
            w16[pos + 2] = (uint16_t)len;
            w16[pos + 3] = (uint16_t)(len >> 16);
            pos += 4;
        }
        w16[pos++] = fits ? v16[kv] : g16[kv];
        kv++;
    }
#ifdef ONO_SP_STAMP
    sp_stamp(g_sp_stamp_mov, tile, sp_t0, sp_tm);
#endif
}

// ------------------------------------------------- one-launch encoder ----
// sp_drop1 (round 5): the drop in one launch, no slot image and no sp_move.
// Workgroup b takes tile b, builds the tile's byte range in LDS exactly as sp_image does, publishes
// its aggregate, looks back over the earlier tiles (decoupled look-back: per tile four 64-bit granules
// {tag, value} for kept values, runs, last kept index + 1 and last run start + 1, tagged "aggregate"
// or "inclusive prefix" with the call's epoch), publishes its inclusive prefix, and writes the range
// straight to its place in the wire.  The look-back has two levels: the earlier tiles of the tile's
// group of 64, then one descriptor per earlier group, which the group's last tile publishes as an
// aggregate once it has seen its group and as an inclusive prefix with its own (a walk back over k
// tiles is k / 4096 + 2 window reads, not k / 64).
// No dispatch order is assumed (HIP promises none): a descriptor that has not come after fb_polls
// polls (~80 us by default) — its workgroup may not have started — is computed by the waiting wave
// from g itself (tile_agg_wave; a group's from its tiles' descriptors and those), the decoupled
// fallback of Smith, Levien & Owens (2024), so every wait ends whatever the placement.  The first
// version took tiles by an atomic ticket instead (in start order, so every wait was on a running
// workgroup): one word takes ~88 returning atomics per us, and 8192 tickets per 64 MiB drop made it
// 0.13 ms (tools/sp_phases: ticket p50 5 us, max 30 us per workgroup).
// The two fields that depend on other tiles: the first run's offset (from the last kept index before
// the tile, known after the look-back) and the length of a run still open at the tile's end, which
// only a later tile knows — that tile (the first one with an unkept value after the run's start, or
// the last tile) writes it, and the tile where the run starts leaves those two units alone.  The last
// tile writes the stream's total and the wire length.
// Traffic: g read once, the wire written once (4 N + wire bytes), plus 64 B of granules per tile.
constexpr size_t kDropGroup = 64;            // tiles per group descriptor (the look-back's second level)
#ifndef DR_SLEEP
#define DR_SLEEP 4
#endif
#ifndef DR_BACK
#define DR_BACK 8
#endif
constexpr uint32_t kDropFallbackPolls = 96;
// the one launch up to 256 tiles (512 Ki values), the two launches above: stream-ordered drops at ~10 %
// kept, one launch / two (tools/drop_sizes.py, profiles/r05_s28_drop_sizes.json): 54,693 values 9.6 /
// 14.8 us, 256 Ki 12.7 / 15.5, 1 Mi 16.8 / 15.6, 16 Mi 95.9 / 33.4.  Past one residency wave of tiles a
// tile's life (its loads under a saturated HBM queue, then the wait for the slowest earlier tile's
// aggregate plus ~3 cross-XCD round trips: ~20 us) times the tiles LDS lets run at once (~2560, 20 MB
// of input) bounds the one launch at ~1 TB/s
constexpr size_t kDropOneLaunchTiles = 256;  // polls (backing off to ~0.85 us each) before the fallback
__device__ __forceinline__ uint64_t dr_ld(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void dr_st(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the three data granules first, acknowledged, then the flag granule (0): a reader polls the flag alone
// and reads the rest once it shows the tag (each still tagged, so a mixed read is seen and retried).
// (Unordered stores with all four granules polled: 88 vs 77 us per 64 MiB drop.)
__device__ __forceinline__ void dr_publish(uint64_t *d, uint32_t tag, uint32_t f, uint32_t r, uint32_t lk, uint32_t lrs) {
    const uint64_t tg = (uint64_t)tag << 32;
    dr_st(d + 1, tg | r);
    dr_st(d + 2, tg | lk);
    dr_st(d + 3, tg | lrs);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    dr_st(d, tg | f);
}
struct DAgg {
    uint32_t f = 0, r = 0, k = 0, s = 0;  // kept values, runs, last kept index + 1, last run start + 1
};
struct PollAcc {  // measurement build: polls and their load time (100 MHz ticks)
    uint32_t polls = 0, ticks = 0;
};
// a descriptor, polled at most `polls` times (at least once), backing off ~0.1 -> ~0.85 us (thousands of
// waiting waves polling every ~50 ns load the fabric): 0 not there, 1 an aggregate, 2 an inclusive prefix
__device__ __forceinline__ int dr_poll(const uint64_t *e, uint32_t tagA, uint32_t tagP, uint32_t polls, DAgg &a,
                                       PollAcc &pa) {
    for (uint32_t it = 0, back = 1;; it++) {
#ifdef ONO_SP_STAMP
        const uint64_t q0 = __builtin_amdgcn_s_memrealtime();
#endif
        const uint64_t a0 = dr_ld(e);
        const uint32_t g0 = (uint32_t)(a0 >> 32);
#ifdef ONO_SP_STAMP
        if (g0 != 0xFFFFFFFFu) {  // (uses it: waits)
            pa.polls++;
            pa.ticks += (uint32_t)(__builtin_amdgcn_s_memrealtime() - q0);
        }
#endif
        if (g0 == tagA || g0 == tagP) {
            const uint64_t a1 = dr_ld(e + 1), a2 = dr_ld(e + 2), a3 = dr_ld(e + 3);
            if ((uint32_t)(a1 >> 32) == g0 && (uint32_t)(a2 >> 32) == g0 && (uint32_t)(a3 >> 32) == g0) {
                a.f = (uint32_t)a0;
                a.r = (uint32_t)a1;
                a.k = (uint32_t)a2;
                a.s = (uint32_t)a3;
                return g0 == tagP ? 2 : 1;
            }
        }
        if (it + 1 >= polls) return 0;
        for (uint32_t q = 0; q < back; q++) __builtin_amdgcn_s_sleep(DR_SLEEP);
        back = min(2 * back, (uint32_t)DR_BACK);
    }
}
// the wave's sums / maxima of one lane value each (all 64 lanes active)
__device__ __forceinline__ uint32_t wsum(uint32_t v) { return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_sum_dpp(v), 63); }
__device__ __forceinline__ uint32_t wmax(uint32_t v) { return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_max_dpp(v), 63); }
// tile j's aggregate straight from g, by one whole wave (j wave-uniform): lane l holds values
// 32 l .. 32 l + 31 of the tile as a keep mask; a run starts at a kept value whose predecessor (the
// value before the tile for the first) is not kept — flags_of's rule
__device__ DAgg tile_agg_wave(const float *g, size_t n, uint32_t j, float t) {
    static_assert(kTile == 64 * 32, "one 32-bit mask per lane");
    const int lane = threadIdx.x & 63;
    const size_t tile0 = (size_t)j * kTile, b = tile0 + 32 * (size_t)lane;
    uint32_t k = 0;
    for (int e = 0; e < 32; e++)
        if (b + e < n && kept(g[b + e], t)) k |= 1u << e;
    uint32_t prev = (uint32_t)__shfl_up((int)(k >> 31), 1, 64);
    if (lane == 0) prev = tile0 > 0 && tile0 - 1 < n && kept(g[tile0 - 1], t) ? 1u : 0u;
    const uint32_t st = k & ~((k << 1) | prev);
    DAgg a;
    a.f = wsum((uint32_t)__popc(k));
    a.r = wsum((uint32_t)__popc(st));
    a.k = wmax(k ? (uint32_t)b + 32u - (uint32_t)__clz(k) : 0u);
    a.s = wmax(st ? (uint32_t)b + 32u - (uint32_t)__clz(st) : 0u);
    return a;
}
// the lanes' results of a window: the nearest inclusive prefix (lane `near` first: lowest, or highest
// when !low) ends the walk and everything from the window's start up to it is added in
__device__ __forceinline__ bool dr_combine(DAgg a, bool isP, bool has, bool low, DAgg &acc) {
    const int lane = threadIdx.x & 63;
    const uint64_t pm = __ballot(has && isP);
    const bool take = has && (!pm || (low ? lane <= __ffsll((unsigned long long)pm) - 1 : lane >= 63 - __clzll(pm)));
    acc.f += wsum(take ? a.f : 0u);
    acc.r += wsum(take ? a.r : 0u);
    acc.k = max(acc.k, wmax(take ? a.k : 0u));
    acc.s = max(acc.s, wmax(take ? a.s : 0u));
    return pm != 0;
}
__device__ __forceinline__ void st_u16(uint8_t *p, uint16_t v) { *(uint16_t *)p = v; }
__device__ __forceinline__ void st_u32_2b(uint8_t *p, uint32_t v) {  // a 2-B aligned u32, as two halves
    st_u16(p, (uint16_t)v);
    st_u16(p + 2, (uint16_t)(v >> 16));
}

// The blocking one-launch drop's completion, in the kernel (no signal launch behind it, no stream wait): every
// wave waits for its stores to be acknowledged, the workgroup meets, and thread 0 releases at system scope (the
// wire in pinned coherent memory can sit dirty in its XCD's L2 until written back: without this fence the TCP
// ring sent frames the host read before their last bytes landed — tools/ono_tcp_bench, profiles/r06_s4_*) and
// counts the workgroup in; the one whose returned count is the call's `target` (the last of the grid to
// arrive: every other workgroup's stores are then out) stores the call's tag into host_tot[2], which the host
// spins on.  The count only grows (the host adds each call's grid to its target), so it is never reset.
// (pl_fused's completion for the TCP ring's lift is the same, into the ring's word)
__device__ __forceinline__ void grid_complete(uint64_t *word, uint64_t *arrive, uint64_t target, uint32_t sig) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __atomic_thread_fence(__ATOMIC_RELEASE);  // (system scope: this XCD's L2 written back)
        const uint64_t old = __hip_atomic_fetch_add(arrive, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == target) __hip_atomic_store(word, (uint64_t)sig, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}
__device__ __forceinline__ void drop1_complete(uint64_t *host_tot, uint64_t *arrive, uint64_t target, uint32_t sig) {
    grid_complete(host_tot + 2, arrive, target, sig);
}
// measurement A/B (round 6): ONO_DROP1_SIGNAL=0 waits for the blocking one launch by a signal kernel behind it
bool drop1_signal_in_kernel() {
    static const bool v = [] {
        const char *e = getenv("ONO_DROP1_SIGNAL");
        return !(e && !strcmp(e, "0"));
    }();
    return v;
}

__global__ __launch_bounds__(kIT) void sp_drop1(const float *__restrict__ g, size_t n, size_t ntiles, float t,
                                                const float *t_dev, bool vec, uint64_t *desc, uint32_t epoch,
                                                uint32_t fb_polls, uint8_t *buf, size_t cap, uint64_t *host_tot,
                                                uint64_t *nbytes_out, uint64_t *arrive, uint64_t target,
                                                uint32_t sig) {
    __shared__ uint32_t s_pre[4];
    SP_CLOCK(sp_t0);
    if (t_dev) t = *t_dev;
    const size_t tile = blockIdx.x;
    SP_CLOCK(sp_tk);
    const uint32_t tagA = 2 * epoch, tagP = 2 * epoch + 1;
    if (ntiles == 0) {  // an empty gradient: the total alone
        if (threadIdx.x == 0) {
            for (int q = 0; q < 4; q++) st_u16(buf + 2 * q, 0);
            if (nbytes_out) *nbytes_out = 8;
            else { host_tot[0] = 0; host_tot[1] = 0; }
        }
        if (sig) drop1_complete(host_tot, arrive, target, sig);
        return;
    }
    const size_t tile0 = tile * kTile;
    float x[kIE], before = 0.0f;
    if (vec && tile0 + kTile <= n) load_tile<true>(g, n, tile, x, before);
    else load_tile<false>(g, n, tile, x, before);
    const TileImg ti = build_image(tile, x, before, n, t);
    SP_CLOCK(sp_ti);
    const uint32_t tend = (uint32_t)min(tile0 + kTile, n);
    const uint32_t lk = ti.F ? (uint32_t)tile0 + ti.last_kept1 : 0u;
    const uint32_t lrs = ti.R ? (uint32_t)tile0 + ti.rs_last + 1u : 0u;
    uint64_t *d = desc + 4 * tile;
    uint64_t *gdesc = desc + 4 * ntiles;  // one descriptor per group of kDropGroup tiles, after the tiles'
    const int lane = threadIdx.x & 63;
    if (threadIdx.x < 64) {
        DAgg pre;
        const uint32_t gi = (uint32_t)(tile / kDropGroup), pos = (uint32_t)(tile % kDropGroup);
        const bool glast = pos == kDropGroup - 1;
        // one look-back window: lane l reads descriptor j_l (if it has one); those that did not come are
        // computed by the wave, one at a time (tile_agg_wave; a group from its tiles)
        PollAcc pa0, pa1;  // (measurement build: lane 0's polls per level)
        auto window = [&](uint32_t j, bool has, bool group) -> bool {
            DAgg a;
            const int st = has ? dr_poll((group ? gdesc : desc) + 4 * (size_t)j, tagA, tagP, fb_polls, a,
                                         group ? pa1 : pa0) : 0;
            bool isP = st == 2;
            for (uint64_t m = __ballot(has && st == 0); m; m &= m - 1) {
                const int l = __ffsll((unsigned long long)m) - 1;
                const uint32_t jl = (uint32_t)__builtin_amdgcn_readlane((int)j, l);
                DAgg b;
                bool bp = false;
                if (!group) {
                    b = tile_agg_wave(g, n, jl, t);
                } else {  // the group's tiles, nearest inclusive prefix first (their descriptors, polled once)
                    const uint32_t tj = jl * (uint32_t)kDropGroup + (uint32_t)lane;
                    DAgg c;
                    const int ct = dr_poll(desc + 4 * (size_t)tj, tagA, tagP, 1, c, pa1);
                    for (uint64_t mm = __ballot(ct == 0); mm; mm &= mm - 1) {
                        const int q = __ffsll((unsigned long long)mm) - 1;
                        const DAgg e = tile_agg_wave(g, n, jl * (uint32_t)kDropGroup + (uint32_t)q, t);
                        if (lane == q) c = e;
                    }
                    bp = dr_combine(c, ct == 2, true, false, b);
                }
                if (lane == l) { a = b; isP = bp; }
            }
            return dr_combine(a, isP, has, true, pre);
        };
        if (tile == 0) {
            if (lane == 0) dr_publish(d, tagP, ti.F, ti.R, lk, lrs);
        } else {
            if (lane == 0) dr_publish(d, tagA, ti.F, ti.R, lk, lrs);
            // level 0: the earlier tiles of the tile's own group, lane 0 the nearest
            bool done = pos && window((uint32_t)tile - 1u - (uint32_t)lane, (uint32_t)lane < pos, false);
#ifdef ONO_SP_STAMP
            if (lane == 0 && tile < (1u << 16)) g_sp_stamp_d1b[tile].w = (unsigned)(__builtin_amdgcn_s_memrealtime() - sp_t0);
#endif
            // the group's aggregate, by its last tile, when no inclusive prefix came with it
            if (!done && glast && lane == 0)
                dr_publish(gdesc + 4 * (size_t)gi, tagA, pre.f + ti.F, pre.r + ti.R, max(pre.k, lk), max(pre.s, lrs));
            // level 1: the earlier groups, 64 a window, lane 0 the nearest
            for (int64_t hi = (int64_t)gi; !done && hi > 0; hi -= 64) {
                const int64_t j = hi - 1 - lane;
                done = window((uint32_t)(j >= 0 ? j : 0), j >= 0, true);
            }
#ifdef ONO_SP_STAMP
            if (lane == 0 && tile < (1u << 16)) g_sp_stamp_d1c[tile] = make_uint4(pa0.polls, pa0.ticks, pa1.polls, pa1.ticks);
#endif
            if (lane == 0) {
                dr_publish(d, tagP, pre.f + ti.F, pre.r + ti.R, max(pre.k, lk), max(pre.s, lrs));
                if (glast) dr_publish(gdesc + 4 * (size_t)gi, tagP, pre.f + ti.F, pre.r + ti.R, max(pre.k, lk), max(pre.s, lrs));
            }
        }
        if (lane == 0) {
            s_pre[0] = pre.f;
            s_pre[1] = pre.r;
            s_pre[2] = pre.k;
            s_pre[3] = pre.s;
        }
    }
    __syncthreads();
    SP_CLOCK(sp_tm);
    const uint32_t F0 = s_pre[0], R0 = s_pre[1], LK0 = s_pre[2], LRS0 = s_pre[3];
    const uint32_t nu16 = 4 * ti.R + ti.F;
    uint8_t *dst = buf + 8 + 8 * (size_t)R0 + 2 * (size_t)F0;  // the tile's first unit
    // the range's units with the cross-tile fields: the first run's offset (units hp0, + 1) completed
    // from the last kept index before the tile; a last run still open at the tile's end (not the last
    // tile) leaves its length units (hpl + 2, + 3) to the tile that ends it
    const bool open_end = ti.R && ti.last_kept1 == tend - (uint32_t)tile0 && tile + 1 < ntiles;
    const uint32_t off0 = ti.off0 + ((uint32_t)tile0 - LK0);
    typedef __attribute__((address_space(3))) const uint16_t lds_cu16;
    lds_cu16 *u16 = (lds_cu16 *)ti.stage;
    auto unit = [&](uint32_t u, uint16_t &v) -> bool {
        if (u >= nu16) return false;
        if (ti.R && u == ti.hp0) { v = (uint16_t)off0; return true; }
        if (ti.R && u == ti.hp0 + 1) { v = (uint16_t)(off0 >> 16); return true; }
        if (open_end && (u == ti.hpl + 2 || u == ti.hpl + 3)) return false;
        v = u16[u];
        return true;
    };
    const uint32_t O = (uint32_t)(((uintptr_t)dst & 15u) >> 1);  // the range starts O units into a 16-B chunk
    uint16_t *base16 = (uint16_t *)(dst - 2 * O);
    // the range inside the buffer, else no store (uniform; the prefix is a look-back over tagged
    // granules, so this is the bound that keeps any wrong prefix from becoming an address)
    const bool in_buf = 8 + 8 * (size_t)R0 + 2 * ((size_t)F0 + nu16) <= cap;
    if (!in_buf && threadIdx.x == 0) drop_error(host_tot, kDropErrRange);
    const uint32_t nch = nu16 && in_buf ? (O + nu16 + 7) / 8 : 0;
    for (uint32_t c = threadIdx.x; c < nch; c += kIT) {
        uint16_t v[8];
        bool all = true, any = false;
        bool ok[8];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int64_t u = (int64_t)c * 8 + i - O;
            ok[i] = u >= 0 && unit((uint32_t)u, v[i]);
            all &= ok[i];
            any |= ok[i];
        }
        if (all) {
            const u4v ov = {v[0] | (uint32_t)v[1] << 16, v[2] | (uint32_t)v[3] << 16, v[4] | (uint32_t)v[5] << 16,
                            v[6] | (uint32_t)v[7] << 16};
            __builtin_nontemporal_store(ov, (u4v *)(base16 + 8 * (size_t)c));
        } else if (any) {
#pragma unroll
            for (int i = 0; i < 8; i++)
                if (ok[i]) base16[8 * (size_t)c + i] = v[i];
        }
    }
    if (threadIdx.x == 0) {
        // a run open at the tile's start (the value before it kept) ends here, at the first unkept value,
        // or at n in the last tile: its length goes into its header, R0 - 1, whose values from its start s
        // to this tile are all kept
        if (tile0 > 0 && LK0 == (uint32_t)tile0 && LRS0 && (ti.first_unkept < (uint32_t)kTile || tile + 1 == ntiles)) {
            const uint32_t s0 = LRS0 - 1u;
            const uint32_t end = ti.first_unkept < (uint32_t)kTile && (uint32_t)tile0 + ti.first_unkept < tend
                                     ? (uint32_t)tile0 + ti.first_unkept : (uint32_t)n;
            const size_t hpos = 8 + 8 * (size_t)(R0 - 1) + 2 * (size_t)(F0 - ((uint32_t)tile0 - s0));
            if (hpos + 8 <= cap) st_u32_2b(buf + hpos + 4, end - s0);
            else drop_error(host_tot, kDropErrRange);
        }
        if (tile + 1 == ntiles) {  // the total (u64 LE, 2-B aligned buf, cap >= 8) and the wire length
            for (int q = 0; q < 4; q++) st_u16(buf + 2 * q, (uint16_t)((uint64_t)n >> (16 * q)));
            const uint64_t F = F0 + ti.F, R = R0 + ti.R, nb = 8 + 8 * R + 2 * F;
            if (nbytes_out) *nbytes_out = nb <= cap ? nb : ~0ull;
            else { host_tot[0] = F; host_tot[1] = R; }
            if (nb > cap) drop_error(host_tot, kDropErrRange);
        }
    }
    if (sig) drop1_complete(host_tot, arrive, target, sig);
#ifdef ONO_SP_STAMP
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x < 64 && tile < (1u << 16)) {
        sp_stamp(g_sp_stamp_d1, tile, sp_t0, sp_tm);
        if (threadIdx.x == 0) {
            g_sp_stamp_d1b[tile].x = (unsigned)(sp_tk - sp_t0);
            g_sp_stamp_d1b[tile].y = (unsigned)(sp_ti - sp_t0);
            g_sp_stamp_d1b[tile].z = blockIdx.x;
            if (tile == 0) g_sp_stamp_d1b[tile].w = (unsigned)(sp_ti - sp_t0);
        }
    }
#endif
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
__global__ __launch_bounds__(kSB) void sp_mask(float *g, size_t n, float t, const float *t_dev, int zero_kept) {
    size_t i = (size_t)blockIdx.x * kSB + threadIdx.x;
    if (i >= n) return;
    if (t_dev) t = *t_dev;
    float x = g[i];
    if (zero_kept) {
        if (kept(x, t)) g[i] = 0.0f;        // scatter: the sent values leave the residual
    } else {
        if (fabsf(x) < t) g[i] = 0.0f;      // gather: only the sent values stay in grad
    }
}

// The TCP ring's SparseCapable hop after its exchange, in one launch (ono_tcp.cpp): the received values into
// their chunk (dst += src, AccOp's add, for the scatter; dst = src, a copy, for the gather) and the sparse
// push's mask of the chunk it sent (sp_mask's two forms, the threshold where the push left it) — two
// different chunks, so the two parts are independent workgroups: one launch instead of two on the hop's path.
// keys != NULL: the next push's sample keys too, whose chunk is dst — its indices bucketed by workgroup (the
// sampler's helper thread sorted them by idx / kSB: offs[b] .. offs[b + 1] fall in workgroup b's values), so
// each workgroup reads back the values it has just written (no order between workgroups needed) and the
// push's own gather launch goes (the select needs the sample's values, not their order).  The first part
// then covers the whole chunk [0, L) (an add over the shorter length leaves [k, L) as they are).
__global__ __launch_bounds__(kSB) void sp_hop_post(float *dst, const float *src, size_t k, int add, float *mg,
                                                   size_t mn, const float *t_dev, int zero_kept, uint32_t b1,
                                                   const uint32_t *idx, const uint32_t *offs, uint32_t *keys) {
    if (blockIdx.x < b1) {
        const size_t i = (size_t)blockIdx.x * kSB + threadIdx.x;
        if (i < k) dst[i] = add ? dst[i] + src[i] : src[i];
        if (keys) {  // (uniform)
            __syncthreads();
            const uint32_t a = offs[blockIdx.x], e = offs[blockIdx.x + 1];
            for (uint32_t j = a + threadIdx.x; j < e; j += kSB)  // (|x| as its bits: abs_key)
                keys[j] = __builtin_bit_cast(uint32_t, dst[idx[j]]) & 0x7FFFFFFFu;
        }
        return;
    }
    const size_t i = (size_t)(blockIdx.x - b1) * kSB + threadIdx.x;
    if (i >= mn) return;
    const float t = *t_dev;
    const float x = mg[i];
    if (zero_kept) {
        if (kept(x, t)) mg[i] = 0.0f;
    } else {
        if (fabsf(x) < t) mg[i] = 0.0f;
    }
}

// ---------------------------------------------------------------- lift ----
// The record stream is a linked list (each header's run length gives the next
// header's position), cut into segments of kSeg bytes.  Three launches:
//  1. sl_index, one workgroup per window of kLW segments (32 KiB of stream
//     staged in LDS with one coalesced pass): each thread picks its segment's
//     first 2-byte position whose next kLook records are all plausible (a
//     speculative record start; segment 0 starts at the true head, byte 8),
//     then walks the records from there in LDS until it lands on a later
//     segment's start (stamping that segment reached with this call's epoch)
//     or the end, noting each record (position, element offset within the
//     walk, length, and a run of at most two values whole).  A block scan of
//     the walks' sums of (offset + length) gives each segment's element index
//     within the window.
//  2. sl_place, a workgroup per 16 segments: the window's prefix, the checks,
//     and the group's whole range of g written with its values and zeros
//     (built in LDS and stored once when it is at most kImg values).
//  3. sl_long: queued chunks (long runs outside an image, wide gaps).
// (64 MiB gradient at 10 % kept on MI355X: 26 + 29.5 + 4 us against 81 us of
// kernels for the six-launch design it replaced; the walks are chains of
// dependent LDS reads per thread, so sl_index is latency-bound.  Tried and
// dropped: the zero-fill on a side stream (event cost > overlap), a
// tile-image fill that re-walks the records per 4096-value tile (58 us: ~10
// walking lanes per workgroup), gap-zeroing by the records' lanes (50 us:
// per-lane scalar stores), a first-record mask of every position (+12 us).)
// The speculation is checked, not trusted: the walks are exactly the
// sequential parse iff every speculative start was reached and no walk failed
// (records form a successor chain, so a walk that lands on a start has joined
// the true chain there; the earliest start off the chain can only be reached
// from the chain, so it stays unreached).  Otherwise `bad` (a host-mapped
// word, this call's epoch) is raised and the host parses sequentially — also
// how malformed input gets the reference's error messages.
constexpr int kSeg = 128, kLook = 4;
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr int kLW = 256;                      // sl_index: threads = segments per window
constexpr size_t kWin = (size_t)kLW * kSeg;   // 32 KiB of stream per window
constexpr int kMarg = 1024;                   // staged past the window (the last segments' look-ahead)
constexpr int kRecK = 32;                     // records kept per segment walk (the rest walked again)
constexpr int kShortP = 32;                   // runs up to this long are placed by one lane
constexpr int kLongChunk = 4096;              // longer runs: queued chunks, one workgroup each

// The stream's u16 units: [lo, lo + 2 n16) from LDS, every other one from
// global memory (p even, b 2-B aligned).  The two pointers carry their address
// spaces, so the two loads cannot be merged into one flat load through a
// selected pointer (which the compiler otherwise does: a flat access to LDS has
// the vector-memory latency).
typedef __attribute__((address_space(3))) const uint16_t lds_u16;
typedef __attribute__((address_space(1))) const uint16_t glb_u16;
struct Bytes {
    const uint8_t *b;
    lds_u16 *lds;
    size_t lo, n16;
    // [p, p + nb) lies in the staged range (p even; p - lo wraps below lo)
    __device__ __forceinline__ bool staged(size_t p, size_t nb) const {
        const size_t d = p - lo;
        return d < 2 * n16 && nb <= 2 * n16 - d;
    }
    // A record header (offset, length): one range check, then four loads
    // issued together from one memory or the other.
    __device__ __forceinline__ void hdr(size_t p, uint32_t &off, uint32_t &len) const {
        uint32_t h0, h1, h2, h3;
        if (staged(p, 8)) {
            lds_u16 *q = lds + ((p - lo) >> 1);
            h0 = q[0]; h1 = q[1]; h2 = q[2]; h3 = q[3];
        } else {
            glb_u16 *q = (glb_u16 *)(b + p);
            h0 = q[0]; h1 = q[1]; h2 = q[2]; h3 = q[3];
        }
        off = h0 | h1 << 16;
        len = h2 | h3 << 16;
    }
    __device__ __forceinline__ uint16_t u16s(size_t p) const { return lds[(p - lo) >> 1]; }  // staged(p, 2)
    __device__ __forceinline__ uint32_t hdr32(size_t p) const {                             // staged(p, 4)
        lds_u16 *q = lds + ((p - lo) >> 1);
        return (uint32_t)q[0] | (uint32_t)q[1] << 16;
    }
};
__device__ __forceinline__ lds_u16 *as_lds(const uint16_t *p) { return (lds_u16 *)p; }

// u16 units [lo, lo + 2 n16) of b (at most MAXB bytes) into lds (8-B
// aligned): 8-B loads when b + lo is 8-B aligned, 4-B loads when 4-B aligned,
// else 2-B loads.  Every load of a thread is issued before the first LDS
// store (one memory latency, not one per load).
template <int NT, int MAXB>
__device__ __forceinline__ void stage_bytes(uint16_t *lds, const uint8_t *b, size_t lo, size_t n16) {
    const uint8_t *src = b + lo;
    const uintptr_t a = (uintptr_t)src;
    size_t done = 0;
    if ((a & 7) == 0) {
        constexpr int K = (MAXB / 8 + NT - 1) / NT;
        const size_t n8 = n16 / 4;
        uint2 v[K];
#pragma unroll
        for (int k = 0; k < K; k++) {
            const size_t i = threadIdx.x + (size_t)k * NT;
            if (i < n8) v[k] = ((const uint2 *)src)[i];
        }
#pragma unroll
        for (int k = 0; k < K; k++) {
            const size_t i = threadIdx.x + (size_t)k * NT;
            if (i < n8) ((uint2 *)lds)[i] = v[k];
        }
        done = 4 * n8;
    } else if ((a & 3) == 0) {
        constexpr int K = (MAXB / 4 + NT - 1) / NT;
        const size_t n4 = n16 / 2;
        uint32_t v[K];
#pragma unroll
        for (int k = 0; k < K; k++) {
            const size_t i = threadIdx.x + (size_t)k * NT;
            if (i < n4) v[k] = ((const uint32_t *)src)[i];
        }
#pragma unroll
        for (int k = 0; k < K; k++) {
            const size_t i = threadIdx.x + (size_t)k * NT;
            if (i < n4) ((uint32_t *)lds)[i] = v[k];
        }
        done = 2 * n4;
    }
    for (size_t i = done + threadIdx.x; i < n16; i += NT) lds[i] = ((const uint16_t *)src)[i];
}

__device__ __forceinline__ uint64_t stream_total(const uint8_t *b) {
    uint64_t total = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) total |= (uint64_t)*(const uint16_t *)(b + 2 * q) << (16 * q);
    return total;
}

// A speculation refuted or a malformed stream: the host parses sequentially.  (A system-scope store: the
// word reaches host memory without waiting for an L2 write-back.)
__device__ __forceinline__ void raise_bad(uint64_t *host_word, uint32_t epoch) {
    __hip_atomic_store(host_word, (uint64_t)epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Segment s's speculative record start: the first 2-byte position whose next
// kLook records are plausible (kNone: none).  A start whose records run past
// the stream is no start; nor is one with a run of >= 2^16 values: a header
// read 2 B off its true position takes a half of the run length as the high
// half of its own (so >= 2^16), and such a jump lands on a true header about
// one time in five, after which every look-ahead record is valid.  Runs are
// maximal in grad_drop's output, so a record after the first is >= 1 value
// past the previous run: offset 0 is no start either (zero-filled payload
// reads as offset 0).  A true start refused here only leaves its segment to
// the previous walk.
__device__ uint32_t seg_start(const Bytes &src, size_t s, size_t nbytes, uint64_t total) {
    if (s == 0) return 8;
    const size_t lo = 8 + s * kSeg, hi = lo + kSeg < nbytes ? lo + kSeg : nbytes;
    for (size_t p = lo; p < hi; p += 2) {
        size_t q = p;
        uint64_t acc = 0;
        bool ok = true;
        for (int k = 0; k < kLook && q != nbytes; k++) {
            if (nbytes - q < 8) { ok = false; break; }
            uint32_t off, len;
            src.hdr(q, off, len);
            if (off == 0 || len >= 0x10000u || (nbytes - q - 8) / 2 < len) { ok = false; break; }
            acc += (uint64_t)off + len;
            if (acc > total) { ok = false; break; }
            q += 8 + 2 * (size_t)len;
        }
        if (ok) return (uint32_t)p;
    }
    return kNone;
}

// seg_start over the staged bytes alone, 32-bit positions: kUnknown when a
// candidate's look-ahead leaves them (then seg_start decides).
constexpr uint32_t kUnknown = 0xFFFFFFFEu;
__device__ uint32_t seg_start_lds(lds_u16 *L, uint32_t lo, uint32_t lim, uint32_t s, uint32_t nbytes, uint64_t total) {
    if (s == 0) return 8;
    const uint32_t a = 8 + s * kSeg, hi = a + kSeg < nbytes ? a + kSeg : nbytes;
    // Candidates four at a time: their first-record tests share one read of 14 bytes (independent
    // of each other, so one LDS latency), and only the survivors, in order, walk their look-ahead.
    for (uint32_t p0 = a; p0 < hi; p0 += 8) {
        if (p0 < lo || p0 + 14 > lim) return kUnknown;  // (not all staged: seg_start decides)
        lds_u16 *h = L + ((p0 - lo) >> 1);
        uint32_t u[7];
#pragma unroll
        for (int i = 0; i < 7; i++) u[i] = h[i];
        uint32_t cand = 0;
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const uint32_t p = p0 + 2 * c, off = u[c] | u[c + 1] << 16, len = u[c + 2] | u[c + 3] << 16;
            const bool ok = p < hi && nbytes - p >= 8 && off != 0 && len < 0x10000u && (nbytes - p - 8) / 2 >= len;
            cand |= (ok ? 1u : 0u) << c;
        }
        while (cand) {
            const uint32_t c = (uint32_t)__builtin_ctz(cand);
            cand &= cand - 1;
            const uint32_t p = p0 + 2 * c;
            uint32_t q = p;
            uint64_t acc = 0;
            bool ok = true;
            for (int k = 0; k < kLook && q != nbytes; k++) {
                if (nbytes - q < 8) { ok = false; break; }
                if (q < lo || q + 8 > lim) return kUnknown;
                lds_u16 *hq = L + ((q - lo) >> 1);
                const uint32_t off = (uint32_t)hq[0] | (uint32_t)hq[1] << 16, len = (uint32_t)hq[2] | (uint32_t)hq[3] << 16;
                if (off == 0 || len >= 0x10000u || (nbytes - q - 8) / 2 < len) { ok = false; break; }
                acc += (uint64_t)off + len;
                if (acc > total) { ok = false; break; }
                q += 8 + 2 * len;
            }
            if (ok) return p;
        }
    }
    return kNone;
}

// Block-wide sum of a u64 (the same value in every thread).
template <int NT>
__device__ __forceinline__ uint64_t block_sum64(uint64_t v) {
    __shared__ uint64_t ws[NT / 64];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += (uint64_t)__shfl_xor((unsigned long long)v, d, 64);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = v;
    __syncthreads();
    uint64_t t = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; w++) t += ws[w];
    __syncthreads();
    return t;
}

// Block-wide max of a u64 (the same value in every thread).
template <int NT>
__device__ __forceinline__ uint64_t block_max64(uint64_t v) {
    __shared__ uint64_t wm[NT / 64];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = max(v, (uint64_t)__shfl_xor((unsigned long long)v, d, 64));
    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = v;
    __syncthreads();
    uint64_t m = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; w++) m = max(m, wm[w]);
    __syncthreads();
    return m;
}

// Per segment s (sl_index): p0 (its speculative start or kNone), gpre (the
// element index its records start from, within its window), the stamps of the
// starts its walk landed on (reached = this call's epoch), and its records:
// rcnt = how many, ent[s K + j] = {byte position, the run's element offset
// within the walk, length, its first two values} for the first K; per window:
// wsum.
__global__ __launch_bounds__(kLW) void sl_index(const uint8_t *b, size_t nbytes, size_t S, uint32_t epoch,
                                                uint32_t *p0g, uint32_t *gpre,
                                                uint32_t *rcnt, uint4 *ent, uint32_t *reached, uint32_t *wsum,
                                                uint32_t *qcount, uint64_t *host_word) {
    __shared__ uint2 lw8[(kWin + kMarg) / 8];
    __shared__ uint32_t lp0[kLW];
    uint16_t *lw = (uint16_t *)lw8;
    const size_t w = blockIdx.x, s0 = w * kLW, s = s0 + threadIdx.x;
    const size_t lo = 8 + w * kWin, hi = lo + kWin + kMarg < nbytes ? lo + kWin + kMarg : nbytes;
    const uint64_t total = stream_total(b);
    if (w == 0 && threadIdx.x == 0) *qcount = 0;  // sl_place's long-run queue
    stage_bytes<kLW, kWin + kMarg>(lw, b, lo, (hi - lo) / 2);
    __syncthreads();
    const Bytes src{b, as_lds(lw), lo, (hi - lo) / 2};
    // (device-path streams are below 4 GiB: 32-bit positions in the LDS loops)
    const uint32_t lo32 = (uint32_t)lo, lim = (uint32_t)(lo + 2 * src.n16), nb32 = (uint32_t)nbytes;
    lds_u16 *L = as_lds(lw);
    uint32_t mine = s < S ? seg_start_lds(L, lo32, lim, (uint32_t)s, nb32, total) : kNone;
    if (mine == kUnknown) mine = seg_start(src, s, nbytes, total);  // look-ahead past the staged bytes
    lp0[threadIdx.x] = mine;
    __syncthreads();
    uint64_t sum = 0;
    uint32_t cnt = 0;
    if (mine != kNone) {
        size_t pos = mine;
        const size_t segend = 8 + (s + 1) * kSeg;
        uint4 *my = ent + s * kRecK;
        bool done = false;
        {  // the walk while every record is staged and every start it meets is in this window:
           // LDS reads only (no memory wait in the loop), 32-bit positions
            // Every exit condition is computed first and tested once (the reads are clamped into the
            // staged bytes), so a step is one divergent branch, not six.
            uint32_t p = mine;
            const uint32_t seg32 = (uint32_t)segend, s032 = (uint32_t)s0, S32 = (uint32_t)S;
            for (;;) {
                const bool end = p == nb32, cross = p >= seg32;
                const uint32_t u = (p - 8) / kSeg, ui = u - s032;
                const bool inwin = ui < (uint32_t)kLW, live = cross && u < S32;
                const uint32_t pu = lp0[inwin ? ui : 0u];
                const bool has = live && inwin && pu != kNone;
                const bool land = has && p == pu, over = has && p > pu, leave = live && !inwin;
                const bool hdr_ok = nb32 - p >= 8 && p + 8 <= lim;
                const uint32_t pc = hdr_ok ? p : lo32;
                lds_u16 *q = L + ((pc - lo32) >> 1);
                const uint32_t off = (uint32_t)q[0] | (uint32_t)q[1] << 16, len = (uint32_t)q[2] | (uint32_t)q[3] << 16;
                const bool len_ok = (nb32 - pc - 8) / 2 >= len;
                if (end || land || over || leave || !hdr_ok || !len_ok) {
                    // the end, a start (joined), a stepped-over start: done; a header not staged or
                    // truncated, another window's start: the general walk takes over
                    if (land) reached[u] = epoch;
                    if (over) raise_bad(host_word, epoch);
                    done = end || land || over;
                    break;
                }
                if (cnt < (uint32_t)kRecK) {
                    const bool whole = len <= 2 && p + 8 + 2 * len <= lim;
                    const uint32_t v01 = len == 2 ? (uint32_t)q[4] | (uint32_t)q[5] << 16 : len == 1 ? (uint32_t)q[4] : 0u;
                    my[cnt] = make_uint4(p | (whole ? 1u : 0u), (uint32_t)(sum + off), len, whole ? v01 : 0u);
                }
                cnt++;
                sum += (uint64_t)off + len;
                if (sum > total) { raise_bad(host_word, epoch); done = true; break; }
                p += 8 + 2 * len;
            }
            pos = p;
        }
        for (; !done;) {
            if (pos == nbytes) break;  // the end of the stream
            if (pos >= segend) {
                const size_t u = (pos - 8) / kSeg;
                const uint32_t pu =
                    u >= S ? kNone : (u - s0 < (size_t)kLW ? lp0[u - s0] : seg_start(src, u, nbytes, total));
                if (pu != kNone && pos == pu) { reached[u] = epoch; break; }
                if (pu != kNone && pos > pu) { raise_bad(host_word, epoch); break; }  // stepped over a start
            }
            if (nbytes - pos < 8) { raise_bad(host_word, epoch); break; }
            uint32_t off, len;
            src.hdr(pos, off, len);
            if ((nbytes - pos - 8) / 2 < len) { raise_bad(host_word, epoch); break; }
            if (cnt < (uint32_t)kRecK) {
                // a run of at most two values rides along whole (most runs are
                // that short): bit 0 of the (even) position says so
                uint32_t v01 = 0, whole = 0;
                if (len <= 2 && src.staged(pos + 8, 2 * (size_t)len)) {
                    whole = 1;
                    v01 = len == 2 ? src.hdr32(pos + 8) : len == 1 ? (uint32_t)src.u16s(pos + 8) : 0u;
                }
                my[cnt] = make_uint4((uint32_t)pos | whole, (uint32_t)(sum + off), len, v01);
            }
            cnt++;
            sum += (uint64_t)off + len;
            if (sum > total) { raise_bad(host_word, epoch); break; }
            pos += 8 + 2 * (size_t)len;
        }
    }
    uint32_t ea, eb, ta, tb;
    block_scan2<kLW>((uint32_t)sum, 0u, ea, eb, ta, tb);
    if (s < S) {
        p0g[s] = mine;
        gpre[s] = ea;
        rcnt[s] = cnt;
    }
    if (threadIdx.x == 0) wsum[w] = ta;
}

// A span of g for sl_long as chunks of kLongChunk: zeros (kind 1) or the f16
// values from stream byte vp on (kind 0).  Reserved with one atomic (rare:
// long runs, and the gaps of groups spanning more than kZeroMax values).
// qflag (pattern path): a host-mapped word set to the epoch, so the host
// launches sl_long only when something was queued.
__device__ __forceinline__ void queue_span(size_t dst, size_t vp, size_t n, uint32_t kind, uint4 *queue,
                                           uint32_t *qcount, uint32_t qcap, uint64_t *host_word, uint32_t epoch,
                                           uint64_t *qflag = nullptr) {
    if (n == 0) return;
    if (qflag) *(volatile uint64_t *)qflag = epoch;
    const uint32_t nc = (uint32_t)((n + kLongChunk - 1) / kLongChunk);
    const uint32_t k = atomicAdd(qcount, nc);
    if (k + nc > qcap || k + nc < k) { raise_bad(host_word, epoch); return; }  // only a refuted stream overfills it
    for (uint32_t c = 0; c < nc; c++) {
        const size_t o = (size_t)c * kLongChunk;
        queue[k + c] = make_uint4((uint32_t)(dst + o), (uint32_t)(vp + 2 * o), (uint32_t)min((size_t)kLongChunk, n - o),
                                  kind);
    }
}

// sl_place: workgroup shape, the largest range built in LDS, its long-run queue, the widest range it zeroes
constexpr int kPT = 256, kPG = 16, kPSeg = kPT / kPG;  // 16 segments per workgroup
constexpr int kImg = 4096, kLQ = 32;
constexpr size_t kZeroMax = 1u << 20;
static_assert(kLW % kPSeg == 0, "a workgroup's segments share a window");

// Where a record's values go: the LDS image of the group's range (dense
// groups), or g itself (wide groups).  Runs longer than kShortP: the LDS
// queue of the workgroup (image) or sl_long's queue (g).
struct Place {
    float *g;
    const uint8_t *b;
    uint64_t ea;     // the group's first element (image index 0)
    float *img;      // nullptr: write g
    uint32_t *lq, *lqn;  // LDS queue of long runs: {image index, stream byte, count} x kLQ
    uint4 *queue;
    uint32_t *qcount, qcap;
    uint64_t *host_word;
    uint32_t epoch;
    __device__ void run(uint64_t gi, size_t vp, uint32_t n, bool carried, uint32_t v01) const {
        if (carried) {
            float *d = img ? img + (gi - ea) : g + gi;
            if (n >= 1) d[0] = from_f16_sp((uint16_t)v01);
            if (n == 2) d[1] = from_f16_sp((uint16_t)(v01 >> 16));
            return;
        }
        glb_u16 *q = (glb_u16 *)(b + vp);
        if (n <= (uint32_t)kShortP) {
            float *d = img ? img + (gi - ea) : g + gi;
            for (uint32_t i = 0; i < n; i++) d[i] = from_f16_sp(q[i]);
            return;
        }
        if (img) {
            const uint32_t k = atomicAdd(lqn, 1u);
            if (k < (uint32_t)kLQ) {
                lq[3 * k] = (uint32_t)(gi - ea);
                lq[3 * k + 1] = (uint32_t)vp;
                lq[3 * k + 2] = n;
                return;
            }
            for (uint32_t i = 0; i < n; i++) img[gi - ea + i] = from_f16_sp(q[i]);  // (queue full: rare)
            return;
        }
        queue_span(gi, vp, n, 0u, queue, qcount, qcap, host_word, epoch);
    }
};

// kPG lanes per segment, kPSeg segments per workgroup (a "group"): the
// window's prefix (a sum over the earlier windows' totals), the speculation
// check (every start reached), the total check (the records' offsets and
// lengths sum to at most the stream's total length: every record lies in
// [0, total), protocol.rs:127-129), then the group's range of g, [E of its
// first segment, E of the next group's) — the tail up to total for the last —
// written with every value and zero in it (grad.fill(0); resize(total, 0);
// the runs: protocol.rs:96-144):
//  * up to kImg values (nearly every group at 10 % kept): built in LDS (zeros,
//    then each noted record placed by one lane) and stored once, coalesced;
//  * up to kZeroMax: zeroed in g by the workgroup, then the values scattered;
//  * wider (a long gap in a sparse stream): the gaps before the records and
//    the tail queued as zero chunks for sl_long, the values scattered.
__global__ __launch_bounds__(kPT) void sl_place(float *g, const uint8_t *b, size_t nbytes, size_t S, size_t cap,
                                                int vec, uint32_t epoch, const uint32_t *p0g, const uint32_t *gpre,
                                                const uint32_t *rcnt, const uint4 *ent, const uint32_t *reached,
                                                const uint32_t *wsum, uint4 *queue, uint32_t *qcount, uint32_t qcap,
                                                uint64_t *host_word) {
    __shared__ f4s img4[kImg / 4];
    float *img = (float *)img4;
    __shared__ uint32_t lq[3 * kLQ], lqn;
    const uint64_t total = stream_total(b);
    if (blockIdx.x == 0 && threadIdx.x == 0) host_word[1] = total;
    if (total > cap) return;  // ONO_E_SIZE: nothing is written
    const size_t sb = (size_t)blockIdx.x * kPSeg, w = sb / kLW, s = sb + threadIdx.x / kPG;
    const uint32_t lane = threadIdx.x % kPG;
    const uint32_t p = s < S ? p0g[s] : kNone;
    const uint32_t gp = s < S ? gpre[s] : 0u, cnt = s < S ? rcnt[s] : 0u;
    const uint32_t rc = s < S && lane == 0 ? reached[s] : 0u;
    const size_t sn = sb + kPSeg;  // the next group's first segment
    const bool last = sn >= S, wend = !last && sn % kLW == 0;
    const uint32_t gpn = !last && !wend ? gpre[sn] : 0u, wsw = S > 0 ? wsum[w] : 0u, gpa = S > 0 ? gpre[sb] : 0u;
    // the lane's two records, loaded with the rest (no dependence on the prefix)
    const uint4 *my = ent + s * kRecK;
    uint4 r[2] = {make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
    if (s < S) {
        r[0] = my[lane];
        r[1] = my[lane + kPG];
    }
    constexpr int U = 4;  // wsum loads in flight per thread per step
    uint64_t part = 0;
    for (size_t j0 = 0; j0 < w; j0 += U * kPT) {
        uint32_t v[U];
#pragma unroll
        for (int k = 0; k < U; k++) {
            const size_t j = j0 + k * kPT + threadIdx.x;
            v[k] = j < w ? wsum[j] : 0u;
        }
#pragma unroll
        for (int k = 0; k < U; k++) part += v[k];
    }
    const uint64_t wp = block_sum64<kPT>(part);
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0 && wp + wsw > total) raise_bad(host_word, epoch);
    if (p != kNone && lane == 0 && s > 0 && rc != epoch) raise_bad(host_word, epoch);  // a start off the chain
    // the group's range (uniform); a refuted stream may give nonsense: clamp into [0, total]
    const uint64_t ea = min(S > 0 ? wp + gpa : 0, total);
    uint64_t eb = last ? total : wend ? wp + wsw : wp + gpn;
    eb = max(min(eb, total), ea);
    const uint64_t R = eb - ea;
    // the image starts at the 16-B boundary at or below ea (g 16-B aligned: whole-vector LDS reads and stores)
    const uint64_t ia = vec ? ea & ~3ull : ea;
    const int mode = eb - ia <= (uint64_t)kImg ? 0 : R <= (uint64_t)kZeroMax ? 1 : 2;  // image / zero + scatter / queue
    if (threadIdx.x == 0) lqn = 0;
    if (mode == 0) {
        const f4s z = {0.0f, 0.0f, 0.0f, 0.0f};
        for (uint32_t i = threadIdx.x; i < (uint32_t)(eb - ia + 3) / 4; i += kPT) img4[i] = z;
    } else if (mode == 1) {
        if (vec) {
            const uint64_t a4 = (ea + 3) / 4, z4 = eb / 4;
            const f4s z = {0.0f, 0.0f, 0.0f, 0.0f};
            if (a4 < z4) {
                for (uint64_t i = a4 + threadIdx.x; i < z4; i += kPT) __builtin_nontemporal_store(z, (f4s *)g + i);
                if (threadIdx.x < 4 * a4 - ea) g[ea + threadIdx.x] = 0.0f;
                if (threadIdx.x < eb - 4 * z4) g[4 * z4 + threadIdx.x] = 0.0f;
            } else {
                for (uint64_t i = ea + threadIdx.x; i < eb; i += kPT) g[i] = 0.0f;
            }
        } else {
            for (uint64_t i = ea + threadIdx.x; i < eb; i += kPT) g[i] = 0.0f;
        }
    }
    __syncthreads();  // the zeros before the values (mode 1: the zero stores have completed)
    const Place P{g, b, ia, mode == 0 ? img : nullptr, lq, &lqn, queue, qcount, qcap, host_word, epoch};
    const uint64_t E = wp + gp;
    const uint32_t m = p != kNone ? min(cnt, (uint32_t)kRecK) : 0u;
    static_assert(kRecK == 2 * kPG, "two records per lane");
    // mode 2: where each record's gap starts (the run before it ended): record j - 1's end by
    // shuffles within the segment's 16 lanes (record j is lane j % 16's r[0] or r[1]), E for the first
    const uint32_t end0 = r[0].y + r[0].z, end1 = r[1].y + r[1].z;
    const uint32_t prev0 = (uint32_t)__shfl((int)end0, (int)((lane + kPG - 1) % kPG), kPG);
    const uint32_t prev1 = (uint32_t)__shfl((int)end1, (int)((lane + kPG - 1) % kPG), kPG);
    const uint64_t from[2] = {lane == 0 ? E : E + prev0, lane == 0 ? E + prev0 : E + prev1};
    uint64_t stream_end = ~0ull;  // the end of the stream's last run, if this thread holds it
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const uint32_t j = lane + k * kPG;
        if (j >= m) break;
        const uint64_t gi = E + r[k].y;
        const uint32_t len = r[k].z;
        const size_t pos = r[k].x & ~1u;
        if (gi > total || total - gi < len || gi < ea || gi + len > eb) {  // (never outside the range)
            raise_bad(host_word, epoch);
            continue;
        }
        if (mode == 2) queue_span(from[k], 0, gi - from[k], 1u, queue, qcount, qcap, host_word, epoch);
        P.run(gi, pos + 8, len, r[k].x & 1u, r[k].w);
        if (pos + 8 + 2 * (size_t)len == nbytes) stream_end = gi + len;
    }
    if (cnt > (uint32_t)kRecK && lane == 0 && p != kNone) {
        // a walk of more than kRecK records (a true start refused nearby): the
        // rest walked again from the last stored one, stopping where sl_index stopped
        const uint4 e = my[kRecK - 1];  // the last stored record: {position, run start in the walk, length}
        size_t pos = (e.x & ~1u) + 8 + 2 * (size_t)e.z;
        uint64_t cur = (uint64_t)e.y + e.z;
        const size_t segend = 8 + (s + 1) * kSeg;
        for (;;) {
            if (pos >= nbytes) break;
            if (pos >= segend) {
                const size_t u = (pos - 8) / kSeg;
                const uint32_t pu = u >= S ? kNone : p0g[u];
                if (pu != kNone && pos >= pu) break;
            }
            if (nbytes - pos < 8) break;
            glb_u16 *h = (glb_u16 *)(b + pos);
            const uint32_t off = (uint32_t)h[0] | (uint32_t)h[1] << 16, len = (uint32_t)h[2] | (uint32_t)h[3] << 16;
            if ((nbytes - pos - 8) / 2 < len) break;
            const uint64_t gi = E + cur + off;
            if (gi > total || total - gi < len || gi < ea || gi + len > eb) { raise_bad(host_word, epoch); break; }
            if (mode == 2) queue_span(E + cur, 0, off, 1u, queue, qcount, qcap, host_word, epoch);
            P.run(gi, pos + 8, len, false, 0u);
            if (pos + 8 + 2 * (size_t)len == nbytes) stream_end = gi + len;
            cur += (uint64_t)off + len;
            pos += 8 + 2 * (size_t)len;
        }
    }
    // mode 2: the tail after the stream's last run (or all of g when there are no records)
    if (mode == 2 && stream_end != ~0ull) queue_span(stream_end, 0, total - stream_end, 1u, queue, qcount, qcap,
                                                      host_word, epoch);
    if (mode == 2 && S == 0 && threadIdx.x == 0) queue_span(0, 0, total, 1u, queue, qcount, qcap, host_word, epoch);
    if (mode != 0) return;
    __syncthreads();  // the image's short runs and the long-run queue
    const uint32_t nl = min(lqn, (uint32_t)kLQ);
    for (uint32_t k = 0; k < nl; k++) {  // long runs: the whole workgroup copies each
        const uint32_t a = lq[3 * k], vp = lq[3 * k + 1], n = lq[3 * k + 2];
        glb_u16 *q = (glb_u16 *)(b + vp);
        for (uint32_t i = threadIdx.x; i < n; i += kPT) img[a + i] = from_f16_sp(q[i]);
    }
    __syncthreads();
    // the range out, coalesced: whole 16-B vectors of the image where they lie inside [ea, eb), the
    // elements of the first and last vector that do one by one
    const uint32_t n = (uint32_t)(eb - ia), nv = (n + 3) / 4;
    const uint32_t skip = (uint32_t)(ea - ia);  // image elements before ea (another group's)
    if (vec) {
        for (uint32_t i = threadIdx.x; i < nv; i += kPT) {
            const uint32_t e0 = 4 * i;
            if (e0 >= skip && e0 + 4 <= n) {
                __builtin_nontemporal_store(img4[i], (f4s *)(g + ia) + i);
            } else {
                for (uint32_t k = 0; k < 4; k++)
                    if (e0 + k >= skip && e0 + k < n) g[ia + e0 + k] = img[e0 + k];
            }
        }
    } else {
        for (uint32_t i = threadIdx.x; i < n; i += kPT) g[ia + i] = img[i];
    }
}

// Queued chunks of long runs and of wide groups' gaps, one workgroup each (grid-stride).
__global__ __launch_bounds__(kSB) void sl_long(float *g, const uint8_t *b, const uint4 *queue,
                                               const uint32_t *qcount, uint32_t qcap) {
    const uint32_t nq = min(*qcount, qcap);
    for (uint32_t k = blockIdx.x; k < nq; k += gridDim.x) {
        const uint4 e = queue[k];
        if (e.w) {  // zeros
            for (uint32_t i = threadIdx.x; i < e.z; i += kSB) g[(size_t)e.x + i] = 0.0f;
        } else {
            glb_u16 *q = (glb_u16 *)(b + e.y);
            for (uint32_t i = threadIdx.x; i < e.z; i += kSB) g[(size_t)e.x + i] = from_f16_sp(q[i]);
        }
    }
}

// ------------------------------------------------- lift: pattern path ----
// The common stream parses with no speculation and no walks (round 3).  In
// grad_drop_into's output (protocol.rs:57-86) every run length is >= 1, every
// offset after the first >= 1 (runs are maximal), and every kept value is a
// nonzero f16 (|g| >= t >= f16::MIN_POSITIVE, protocol.rs:48).  When the gaps
// and runs are also shorter than 2^16 values, the only zero u16s of the stream
// are the high halves of the headers' two fields, so unit k (byte 8 + 2k)
// starts a record iff units k + 1 and k + 3 are zero: offset = unit k, length
// = unit k + 2.  (Another k with both zeros would need a header high half at
// k + 3 with k not a header: k = h + 2 puts a zero at h + 5, i.e. another
// header at h + 4 — a zero-length run.)  The candidates are then CHECKED to be
// the sequential parse, exactly and in parallel: the first is unit 0, each
// candidate's successor k + 4 + length is the next candidate or the end of the
// stream, and the offsets and lengths sum to at most total.  By induction from
// the head the reference's loop (protocol.rs:109-141) visits exactly these
// records, in order, with the same bounds checks passing.  A stream outside the
// shape (long gaps or runs, zero-length runs, zero payloads, malformed input)
// fails a check and the walk path below parses it, rewriting [0, total).
// Three launches: pl_index (per 8 KiB tile: candidates, in-tile successor
// checks, {count, sum of offset + length, first, exit}), pl_scan (one
// workgroup: the tiles' element prefixes and the cross-tile links), pl_place
// (per tile: its range of g — the gap before each record, the records' runs,
// the tail after the last — built in LDS from the staged tile and stored once).
constexpr int kPatU = 2048;                           // stream units (u16) per tile: 4 KiB
constexpr int kPatT = 256, kPatPer = kPatU / kPatT;   // 8 units per thread
constexpr int kPatImg = 6144;                         // pl_place's LDS image, floats (a tile's range is
                                                      // ~4.5 K values at 10 % kept)
constexpr int kPatHalo = 40;                          // staged past the tile: the last header's fields and
                                                      // every short run that starts in the tile
constexpr int kPatScanT = 1024;                       // pl_scan's one workgroup
constexpr uint32_t kPatNone = 0xFFFFFFFFu;
static_assert(kPatPer == 8, "a thread's 8 units and the 4 after them are one 16-B and one 8-B LDS read");
static_assert(kPatHalo >= 4 + kShortP, "short runs of the tile's records are staged whole");

// A thread's units and the 4 after them from the staged tile.
// the 4 units after a thread's 8: the next lane's by a lane shift (1: no 2-way conflicts of the 8-B
// read, measured no faster: 23.9-24.1 vs 23.7 us per lift, profiles/r05_s45_lift_ab.txt) or LDS (0)
#ifndef ONO_UNITS12_SHFL
#define ONO_UNITS12_SHFL 0
#endif
// The pattern lift's records read their units from LDS (a 16-B lane stride: 4-way bank conflicts, ~1.1
// conflict cycles per LDS instruction) — not from the registers units12 already holds, selected per lane
// (`Units12::sel`; 0.17 conflict cycles per instruction, but 25.9 vs 24.1 us per 64 MiB lift: the
// selects' VALU cost more than the conflicts, profiles/r05_s44_lift_ab.txt); 1 builds that form.
#ifndef ONO_PL_UNITS_REG
#define ONO_PL_UNITS_REG 0
#endif
__device__ __forceinline__ const uint16_t *lw4u16(const uint4 *p) { return (const uint16_t *)p; }
struct Units12 {
    uint32_t w[6];
    __device__ __forceinline__ uint32_t u(int i) const { return (w[i >> 1] >> ((i & 1) * 16)) & 0xFFFFu; }
    // unit i (< 12) for a lane-varying i: selects, not an indexed register array (that would be scratch)
    __device__ __forceinline__ uint32_t sel(uint32_t i) const {
        uint32_t x = w[0];
#pragma unroll
        for (int q = 1; q < 6; q++) {
            uint32_t y = w[q];
            asm volatile("" : "+v"(y));  // (else the chain is folded back into a scratch array load)
            x = (i >> 1) == (uint32_t)q ? y : x;
        }
        return (x >> ((i & 1) * 16)) & 0xFFFFu;
    }
};
// (every lane of the wave active) the 4 units after the thread's 8 are the next lane's first 4, taken
// by a lane shift; only lane 63 reads them from LDS — an 8-B read per lane at a 16-B stride put two
// lanes on every bank
__device__ __forceinline__ Units12 units12(const uint4 *lw4) {
    Units12 r;
    const uint4 a = lw4[threadIdx.x];
#if ONO_UNITS12_SHFL
    uint32_t c0 = (uint32_t)__shfl_down((int)a.x, 1, 64), c1 = (uint32_t)__shfl_down((int)a.y, 1, 64);
    if ((threadIdx.x & 63) == 63) {
#else
    uint32_t c0 = 0, c1 = 0;
    {
#endif
        const uint2 c = ((const uint2 *)lw4)[2 * threadIdx.x + 2];
        c0 = c.x;
        c1 = c.y;
    }
    r.w[0] = a.x; r.w[1] = a.y; r.w[2] = a.z; r.w[3] = a.w;
    r.w[4] = c0; r.w[5] = c1;
    return r;
}
// Candidate mask of the thread's units (k = base + 8 t + j, a header needs k + 4 <= M) and the sum of
// their offsets and lengths.
__device__ __forceinline__ uint32_t pat_mask(const Units12 &U, size_t k0, size_t M, uint32_t &sum) {
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < kPatPer; j++) m |= (U.u(j + 1) == 0u && U.u(j + 3) == 0u) ? 1u << j : 0u;
    if (k0 + 4 > M) m = 0;
    else if (M - k0 - 4 < (size_t)kPatPer - 1) m &= (2u << (M - k0 - 4)) - 1u;
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < kPatPer; j++) s += (m >> j & 1u) ? U.u(j) + U.u(j + 2) : 0u;
    sum = s;
    return m;
}
constexpr int kPatStage = kPatU + kPatHalo;  // units staged per tile
// the tile's units [base, base + kPatStage) of the stream's M (after the 8-byte total) into LDS
__device__ __forceinline__ size_t pat_stage(uint4 *lw4, const uint8_t *b, size_t base, size_t M) {
    const size_t n16 = min(M - base, (size_t)kPatStage);
    stage_bytes<kPatT, 2 * kPatStage>((uint16_t *)lw4, b, 8 + 2 * base, n16);
    return n16;
}

// rec[4 t ..]: candidates, sum of offset + length, first candidate, exit (the
// last candidate's successor: the next tile's first record or M).
// A thread's 12 units straight from the stream (one 16-B and one 8-B load when
// the stream is 8-B aligned: the 8-byte total keeps them so), unit by unit at
// the stream's end or for a stream at a 2-B boundary.
__device__ __forceinline__ Units12 units12_global(const uint8_t *b, size_t k0, size_t M) {
    Units12 r;
    const uint8_t *p = b + 8 + 2 * k0;
    if (k0 + 12 <= M && ((uintptr_t)b & 7) == 0) {
        const uint4 a = *(const uint4 *)p;
        const uint2 c = *(const uint2 *)(p + 16);
        r.w[0] = a.x; r.w[1] = a.y; r.w[2] = a.z; r.w[3] = a.w;
        r.w[4] = c.x; r.w[5] = c.y;
    } else {
#pragma unroll
        for (int i = 0; i < 6; i++) {
            const uint32_t lo = k0 + 2 * i < M ? ((const uint16_t *)p)[2 * i] : 0u;
            const uint32_t hi = k0 + 2 * i + 1 < M ? ((const uint16_t *)p)[2 * i + 1] : 0u;
            r.w[i] = lo | hi << 16;
        }
    }
    return r;
}
// unit j + 2 of the thread's units for a run-time j < kPatPer (a select chain: a register array
// indexed at run time would be moved to LDS and addressed through the dispatch packet)
__device__ __forceinline__ uint32_t unit_plus2(const Units12 &U, uint32_t j) {
    uint32_t v = U.u(2);
#pragma unroll
    for (int q = 1; q < kPatPer; q++) v = j == (uint32_t)q ? U.u(q + 2) : v;
    return v;
}

// rec[4 t ..]: candidates, sum of offset + length, first candidate, exit (the
// last candidate's successor: the next tile's first record or M).  The units
// come straight from HBM into registers (no LDS staging); the masks and their
// prefixes go through LDS for the successor checks.  TPB tiles per workgroup,
// every thread's loads for all of them issued before the first is used: the
// stream is small (~15 MB for a 64 MiB gradient at 10 % kept), so the kernel is
// a few rounds of load latency, and TPB = 2 halves the rounds.
template <int TPB> struct PatCnt {
    uint32_t v[2 * TPB];
};
template <int TPB>
__device__ __forceinline__ void block_scan_n(const uint32_t (&in)[2 * TPB], uint32_t (&ex)[2 * TPB],
                                             uint32_t (&tot)[2 * TPB]) {
    __shared__ uint32_t wt[2 * TPB][kPatT / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t inc[2 * TPB];
#pragma unroll
    for (int q = 0; q < 2 * TPB; q++) {
        inc[q] = wave_incl_sum_dpp(in[q]);
        if (lane == 63) wt[q][wave] = inc[q];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 2 * TPB; q++) {
        uint32_t pre = 0, all = 0;
#pragma unroll
        for (int w = 0; w < kPatT / 64; w++) {
            pre += w < wave ? wt[q][w] : 0u;
            all += wt[q][w];
        }
        ex[q] = pre + inc[q] - in[q];
        tot[q] = all;
    }
}
template <int TPB>
__global__ __launch_bounds__(kPatT) void pl_index(const uint8_t *b, size_t M, size_t T, uint32_t *rec, uint32_t *tsum,
                                                  uint32_t *qcount, uint32_t *wide, uint64_t *host_word,
                                                  uint64_t *badw, uint32_t epoch) {
    __shared__ uint16_t lmask[TPB][kPatT], lpre[TPB][kPatT];  // (masks of kPatPer bits)
    SP_CLOCK(sp_t0);
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // before pl_place: the total for the host, an empty queue
        host_word[1] = stream_total(b);
        *qcount = 0;
    }
    const uint32_t j0 = kPatPer * threadIdx.x;
    Units12 U[TPB];
#pragma unroll
    for (int q = 0; q < TPB; q++) {
        const size_t base = ((size_t)blockIdx.x * TPB + q) * kPatU;
        U[q] = base + j0 < M ? units12_global(b, base + j0, M) : Units12{};
    }
    uint32_t m[TPB], in[2 * TPB], ex[2 * TPB], tot[2 * TPB];
#pragma unroll
    for (int q = 0; q < TPB; q++) {
        const size_t base = ((size_t)blockIdx.x * TPB + q) * kPatU;
        uint32_t sum = 0;
        m[q] = base + j0 < M ? pat_mask(U[q], base + j0, M, sum) : 0u;
        in[2 * q] = (uint32_t)__builtin_popcount(m[q]);
        in[2 * q + 1] = sum;
    }
    block_scan_n<TPB>(in, ex, tot);
    SP_CLOCK(sp_tm);
#pragma unroll
    for (int q = 0; q < TPB; q++) {
        lmask[q][threadIdx.x] = (uint16_t)m[q];
        lpre[q][threadIdx.x] = (uint16_t)ex[2 * q];
    }
    __syncthreads();
    bool bad = false;
#pragma unroll
    for (int q = 0; q < TPB; q++) {
        const size_t t = (size_t)blockIdx.x * TPB + q, base = t * kPatU;
        if (t >= T) break;  // (uniform)
        const uint32_t ec = ex[2 * q], tc = tot[2 * q];
        uint32_t rank = ec;
        for (uint32_t mm = m[q]; mm && !bad; mm &= mm - 1, rank++) {
            const uint32_t j = (uint32_t)__builtin_ctz(mm), k = j0 + j;
            const uint32_t nx = k + 4 + unit_plus2(U[q], j);  // tile-local successor
            if (base + nx > M) { bad = true; break; }  // the run overruns the stream
            if (nx < (uint32_t)kPatU && base + nx < M) {
                const uint32_t m2 = lmask[q][nx / kPatPer], b2 = nx % kPatPer;
                const uint32_t p2 = lpre[q][nx / kPatPer] + (uint32_t)__builtin_popcount(m2 & ((1u << b2) - 1u));
                if (!(m2 >> b2 & 1u) || p2 != rank + 1) { bad = true; break; }
            } else {  // the end of the stream or another tile: only the tile's last candidate goes there
                if (rank + 1 != tc) { bad = true; break; }
                rec[4 * t + 3] = (uint32_t)(base + nx);
            }
        }
        if (m[q] && ec == 0) rec[4 * t + 2] = (uint32_t)(base + j0 + __builtin_ctz(m[q]));
        if (threadIdx.x == 0) {
            rec[4 * t] = tc;
            rec[4 * t + 1] = tot[2 * q + 1];
            tsum[t] = tot[2 * q + 1];  // (again, contiguous: pl_place sums the earlier tiles' from here)
            if (tc == 0) { rec[4 * t + 2] = kPatNone; rec[4 * t + 3] = kPatNone; }
        }
    }
    if (bad) raise_bad(badw, epoch);
#ifdef ONO_SP_STAMP
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x < 64) sp_stamp(g_sp_stamp_pli, blockIdx.x, sp_t0, sp_tm);
#endif
}
hipError_t launch_pl_index(const uint8_t *b, size_t M, size_t T, uint32_t *rec, uint32_t *tsum, uint32_t *qcount,
                           uint32_t *wide, uint64_t *host_word, uint64_t *badw, uint32_t epoch, hipStream_t s) {
    // (two tiles per workgroup, all their loads issued before the first use, measured slower in round 4:
    // 9.35 vs 8.1 us; the template keeps the form)
    hipLaunchKernelGGL(pl_index<1>, dim3((unsigned)T), dim3(kPatT), 0, s, b, M, T, rec, tsum, qcount, wide, host_word,
                       badw, epoch);
    return hipGetLastError();
}

// E[t] = the element index tile t's range starts at: one workgroup scans the
// tiles' sums, 4 per thread, kPatScanT x 4 tiles per step (DPP wave scans; the
// u32 partial sums are exact when the u64 total is at most total < 2^32, which
// is checked).  E[T] = where the last run ends.
constexpr int kPatScanPer = 4;
__global__ __launch_bounds__(kPatScanT) void pl_scan(const uint8_t *b, const uint32_t *rec, size_t T, uint64_t *E,
                                                     uint64_t *badw, uint32_t epoch) {
    __shared__ uint32_t wtot[kPatScanT / 64];
    const uint64_t total = stream_total(b);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t carry = 0;
    for (size_t c0 = 0; c0 < T; c0 += (size_t)kPatScanT * kPatScanPer) {
        const size_t i0 = c0 + (size_t)kPatScanPer * threadIdx.x;
        uint32_t v[kPatScanPer];
#pragma unroll
        for (int q = 0; q < kPatScanPer; q++) v[q] = i0 + q < T ? ((const uint4 *)rec)[i0 + q].y : 0u;
        uint32_t own = 0;
#pragma unroll
        for (int q = 0; q < kPatScanPer; q++) own += v[q];
        const uint32_t inc = wave_incl_sum_dpp(own);
        if (lane == 63) wtot[wave] = inc;
        __syncthreads();
        uint32_t before = 0;
        uint64_t all = 0;
#pragma unroll
        for (int w = 0; w < kPatScanT / 64; w++) {
            before += w < wave ? wtot[w] : 0u;
            all += wtot[w];
        }
        __syncthreads();
        uint64_t e = carry + before + (inc - own);
#pragma unroll
        for (int q = 0; q < kPatScanPer; q++) {
            if (i0 + q < T) E[i0 + q] = e;
            e += v[q];
        }
        carry += all;
    }
    if (threadIdx.x == 0) {
        E[T] = carry;
        if (carry > total) raise_bad(badw, epoch);
    }
}

// The non-empty tile before tile `from` (exclusive), or -1: the workgroup
// tests 256 tiles at a time, nearest first (a run spanning many tiles).
__device__ int64_t prev_nonempty(const uint32_t *rec, size_t from) {
    __shared__ int64_t best[kPatT / 64];
    size_t hi = from;  // candidates [0, hi)
    while (hi > 0) {
        const size_t i = hi - 1 - threadIdx.x;
        int64_t v = threadIdx.x < hi && rec[4 * i] > 0 ? (int64_t)i : -1;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) v = max(v, (int64_t)__shfl_xor((long long)v, d, 64));
        if ((threadIdx.x & 63) == 0) best[threadIdx.x >> 6] = v;
        __syncthreads();
        int64_t r = -1;
#pragma unroll
        for (int w = 0; w < kPatT / 64; w++) r = max(r, best[w]);
        __syncthreads();
        if (r >= 0) return r;
        hi = hi > (size_t)kPatT ? hi - kPatT : 0;
    }
    return -1;
}

// Tile t's range of g: [E_t, E_t+1) — [E_T-1, total) for the last tile, which
// also holds the tail — with its zeros and values, and the cross-tile links:
// the tile's first record is the exit of the nearest non-empty tile before it
// (or the head, unit 0); the last tile's (or the last non-empty one's) exit is M.
// A range of up to kPatImg values (every tile of a 10 %-kept stream) is built in
// LDS in one pass — zeros, each record's run placed by the lane that holds it
// (short runs from the staged units, long ones by the workgroup) — and stored
// as whole 16-B vectors.  A wider range (sparse streams) is flagged for pl_wide.
constexpr size_t kPatDirect = 4096;  // up to this many tiles pl_place sums the earlier tiles itself
// One tile with a wide range (above kPatImg: sparse streams), placed by one
// workgroup: up to kPatPasses windows of kPatImg values built in LDS one after
// another; wider still (few tiles hold all of g) and allow_queue, the gaps and
// the tail queued as zero chunks for sl_long's full grid and the values
// scattered (long runs queued); without allow_queue (the stream-ordered lift,
// which launches nothing after it) every window in turn, however many.
constexpr int kPatPasses = 8;
__device__ __forceinline__ void wide_tile(float *g, const uint8_t *b, size_t M, size_t T, int vec, size_t t,
                                          uint64_t E0, uint32_t sum_t, uint64_t total, bool allow_queue,
                                          uint2 *img8, uint4 *lw4, uint32_t *lq, uint32_t *lqn, uint4 *queue,
                                          uint32_t *qcount, uint32_t qcap, uint64_t *host_word, uint64_t *badw,
                                          uint32_t epoch) {
    uint16_t *img = (uint16_t *)img8;
    const uint16_t *lw = (const uint16_t *)lw4;
    const size_t base = t * kPatU;
    const uint64_t ea = min(E0, total);
    uint64_t eb = t + 1 == T ? total : min(E0 + sum_t, total);
    eb = max(eb, ea);
    __syncthreads();  // earlier reads of the staged units
    pat_stage(lw4, b, base, M);
    __syncthreads();
    const Units12 U = units12(lw4);
    const uint32_t j0 = kPatPer * threadIdx.x;
    uint32_t sum;
    const uint32_t m = pat_mask(U, base + j0, M, sum);
    uint32_t ec, es, tc, ts;
    block_scan2<kPatT>((uint32_t)__builtin_popcount(m), sum, ec, es, tc, ts);
    const uint64_t ia = vec ? ea & ~3ull : ea, span = eb - ia;
    const uint64_t npass = (span + kPatImg - 1) / kPatImg;
    if (allow_queue && npass > (uint64_t)kPatPasses) {
        uint64_t cur = E0 + es;
        for (uint32_t mm = m; mm; mm &= mm - 1) {
            const uint32_t k = j0 + (uint32_t)__builtin_ctz(mm), off = lw[k], len = lw[k + 2];
            const uint64_t gi = cur + off;
            if (gi < ea || gi + len > eb || base + k + 4 + len > M) { raise_bad(badw, epoch); break; }
            queue_span(cur, 0, off, 1u, queue, qcount, qcap, host_word, epoch, host_word + 3);
            if (len <= (uint32_t)kShortP)
                for (uint32_t i = 0; i < len; i++) g[gi + i] = from_f16_sp(lw[k + 4 + i]);
            else
                queue_span(gi, 8 + 2 * (base + k + 4), len, 0u, queue, qcount, qcap, host_word, epoch,
                           host_word + 3);
            cur = gi + len;
        }
        const bool holds_last = m != 0 && ec + (uint32_t)__builtin_popcount(m) == tc;
        if (t + 1 == T && (holds_last || (tc == 0 && threadIdx.x == 0)))
            queue_span(E0 + ts, 0, total > E0 + ts ? total - (E0 + ts) : 0, 1u, queue, qcount, qcap, host_word,
                       epoch, host_word + 3);
        return;
    }
    const uint64_t skip = ea - ia;
    for (uint64_t p = 0; p < npass; p++) {
        const uint64_t w0 = p * kPatImg, w1 = min(w0 + kPatImg, span);
        const uint32_t wn = (uint32_t)(w1 - w0);
        for (uint32_t i = threadIdx.x; i < (wn + 3) / 4; i += kPatT) img8[i] = make_uint2(0u, 0u);
        if (threadIdx.x == 0) *lqn = 0;
        __syncthreads();
        uint64_t cur = E0 + es;
        for (uint32_t mm = m; mm; mm &= mm - 1) {
            const uint32_t k = j0 + (uint32_t)__builtin_ctz(mm), off = lw[k], len = lw[k + 2];
            const uint64_t gi = cur + off;
            cur = gi + len;
            if (gi < ea || gi + len > eb || base + k + 4 + len > M) { raise_bad(badw, epoch); break; }
            const uint64_t r0 = gi - ia, a = max(r0, w0), e = min(r0 + len, w1);
            if (a >= e) continue;
            const uint32_t c = (uint32_t)(e - a), u0 = k + 4 + (uint32_t)(a - r0), ai = (uint32_t)(a - w0);
            if (len <= (uint32_t)kShortP) {
                for (uint32_t i = 0; i < c; i++) img[ai + i] = lw[u0 + i];
            } else {
                const uint32_t q = atomicAdd(lqn, 1u);
                if (q < (uint32_t)kLQ) {
                    lq[3 * q] = ai;
                    lq[3 * q + 1] = (uint32_t)(8 + 2 * (base + u0));
                    lq[3 * q + 2] = c;
                } else {
                    for (uint32_t i = 0; i < c; i++) img[ai + i] = ((glb_u16 *)(b + 8 + 2 * (base + u0)))[i];
                }
            }
        }
        __syncthreads();
        const uint32_t nl = min(*lqn, (uint32_t)kLQ);
        for (uint32_t q = 0; q < nl; q++) {
            const uint32_t a = lq[3 * q], vp = lq[3 * q + 1], c = lq[3 * q + 2];
            glb_u16 *src = (glb_u16 *)(b + vp);
            for (uint32_t i = threadIdx.x; i < c; i += kPatT) img[a + i] = src[i];
        }
        __syncthreads();
        float *dst = g + ia + w0;
        for (uint32_t i = threadIdx.x; i < wn; i += kPatT)
            if (w0 + i >= skip) dst[i] = from_f16_sp(img[i]);
        __syncthreads();
    }
}

// pl_place's prologue reduction, all DPP (no 64-bit lane shuffles): the sum of the threads' partial sums of
// the earlier tiles' sums (each < 2^31: at most 16 tile sums of < 2^27) as two 16-bit-split 32-bit sums, exact
// in 64 bits; the largest `kidx` (the nearest non-empty earlier tile, index + 1) and the `exit` of the thread
// that holds it (kidx values are distinct or 0).  Two block syncs.
__device__ __forceinline__ void block_sum_nearest(uint64_t part, uint32_t kidx, uint32_t exit, uint64_t &S,
                                                  uint32_t &kmax, uint32_t &kexit) {
    __shared__ uint32_t slo[kPatT / 64], shi[kPatT / 64], smx[kPatT / 64], sx;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t p = (uint32_t)part;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_sum_dpp(p & 0xFFFFu), 63);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_sum_dpp(p >> 16), 63);
    const uint32_t mx = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_max_dpp(kidx), 63);
    if (lane == 0) {
        slo[wave] = lo;
        shi[wave] = hi;
        smx[wave] = mx;
    }
    __syncthreads();
    uint64_t tl = 0, th = 0;
    uint32_t m = 0;
#pragma unroll
    for (int w = 0; w < kPatT / 64; w++) {
        tl += slo[w];
        th += shi[w];
        m = max(m, smx[w]);
    }
    if (m != 0 && kidx == m) sx = exit;
    __syncthreads();
    S = (th << 16) + tl;
    kmax = m;
    kexit = m ? sx : 0u;
}

// (32-bit element and unit arithmetic: total <= cap < 2^32 and M < 2^31 on the device path; the one
// sum that could wrap in a malformed stream, the last tile's, is checked in 64 bits)
// ASYNC (the stream-ordered lift): nothing is launched after it, so a wide range is placed here
// (wide_tile without the queue) and total > cap refutes the call instead of being read by the host.
template <bool ASYNC>
__global__ __launch_bounds__(kPatT) void pl_place(float *g, const uint8_t *b, size_t M, size_t T, size_t cap, int vec,
                                                  uint64_t *E, const uint32_t *rec, const uint32_t *tsum,
                                                  uint32_t *wide, uint64_t *host_word, uint64_t *badw,
                                                  uint32_t epoch) {
    __shared__ uint4 img16[kPatImg / 8];  // the range as f16 bits (12 KiB: 8 workgroups per CU), widened on the way out
    __shared__ uint4 lw4[kPatStage / 8 + 1];
    __shared__ uint32_t lq[3 * kLQ], lqn;
    uint2 *img8 = (uint2 *)img16;
    uint16_t *img = (uint16_t *)img16;
    const uint16_t *lw = (const uint16_t *)lw4;
    const uint32_t t = blockIdx.x, base = t * (uint32_t)kPatU, M32 = (uint32_t)M, T32 = (uint32_t)T;
    const bool direct = T <= kPatDirect;  // (uniform) else E[] from pl_scan
    SP_CLOCK(sp_t0);
    // the prologue's loads issued together: the tile's record, its range (E from pl_scan, or the earlier
    // tiles' sums), the record of each of the 256 tiles before it (the nearest non-empty one's exit is
    // the link into this tile)
    const uint4 me = ((const uint4 *)rec)[t];
    // (the earlier tiles' sums as 16-B vectors, 4 loads per thread: tsum holds a multiple of 4 entries)
    constexpr int kSumVec = (int)(kPatDirect / (4 * kPatT));
    uint4 sums[kSumVec];
    uint64_t E0 = 0, E1 = 0;
    if (direct) {
#pragma unroll
        for (int q = 0; q < kSumVec; q++) {
            const uint32_t i = 4 * (threadIdx.x + (uint32_t)q * kPatT);
            sums[q] = i < t ? *(const uint4 *)(tsum + i) : make_uint4(0, 0, 0, 0);
        }
    } else {
        E0 = E[t];
        E1 = E[t + 1];
    }
    const uint4 near = threadIdx.x < t ? ((const uint4 *)rec)[t - 1 - threadIdx.x] : make_uint4(0, 0, 0, 0);
    const uint64_t total = stream_total(b);
    pat_stage(lw4, b, base, M);
    if (total > cap) {  // ONO_E_SIZE: nothing is written
        if (ASYNC && t == 0 && threadIdx.x == 0) raise_bad(badw, epoch);
        return;
    }
    if (threadIdx.x == 0) lqn = 0;
    {
        uint64_t part = 0;
        if (direct) {
#pragma unroll
            for (int q = 0; q < kSumVec; q++) {
                const uint32_t i = 4 * (threadIdx.x + (uint32_t)q * kPatT);
                part += (i < t ? sums[q].x : 0u) + (i + 1 < t ? sums[q].y : 0u) + (i + 2 < t ? sums[q].z : 0u) +
                        (i + 3 < t ? sums[q].w : 0u);
            }
        }
        // the nearest non-empty tile among the 256 before t: index + 1 (0: none), its exit
        const uint32_t kidx = threadIdx.x < t && near.x > 0 ? t - threadIdx.x : 0u;
        uint64_t S;
        uint32_t kmax, kexit;
        block_sum_nearest(part, kidx, near.w, S, kmax, kexit);  // (its sync also covers the staged units)
        uint32_t pexit = kexit;
        bool found = kmax != 0;
        if (!found && t > (uint32_t)kPatT) {  // none among those 256
            const int64_t q = prev_nonempty(rec, t - kPatT);
            found = q >= 0;
            if (found) pexit = rec[4 * q + 3];
        }
        bool bad = me.x > 0 && (found ? pexit != me.z : me.z != 0u);
        if (t + 1 == T32) bad |= me.x > 0 ? me.w != M32 : !found || pexit != M32;
        if (direct) {
            E0 = S;
            E1 = E0 + me.y;
            if (t + 1 == T32) bad |= E1 > total;  // the offsets and lengths sum to at most total
        }
        if (bad && threadIdx.x == 0) raise_bad(badw, epoch);
    }
    SP_CLOCK(sp_tm);
    const uint32_t total32 = (uint32_t)total;
    const uint32_t ea = (uint32_t)min(E0, total);
    const uint32_t eb = max(t + 1 == T32 ? total32 : (uint32_t)min(E1, total), ea);
    const uint32_t ia = vec ? ea & ~3u : ea;
    const uint32_t n = min(eb - ia, (uint32_t)kPatImg + 1);
    const bool is_wide = eb > ea && n > (uint32_t)kPatImg;
    if constexpr (ASYNC) {
        if (is_wide) {  // (uniform)
            wide_tile(g, b, M, T, vec, t, E0, me.y, total, false, img8, lw4, lq, &lqn, nullptr, nullptr, 0,
                      host_word, badw, epoch);
            return;
        }
    } else if (threadIdx.x == 0) {
        wide[t] = is_wide;  // (every tile writes its flag: nothing to reset between lifts)
        if (is_wide) {
            if (direct) E[t] = E0;
            *(volatile uint64_t *)(host_word + 4) = epoch;
        }
    }
    if (eb == ea || is_wide) return;  // (uniform) an empty tile inside a run; a wide range: pl_wide places it
    for (uint32_t i = threadIdx.x; i < (n + 7) / 8; i += kPatT) img16[i] = make_uint4(0u, 0u, 0u, 0u);
    const Units12 U = units12(lw4);
    const uint32_t j0 = kPatPer * threadIdx.x;
    uint32_t sum;
    const uint32_t m = pat_mask(U, base + j0, M, sum);
    uint32_t ec, es, tc, ts;
    block_scan2<kPatT>((uint32_t)__builtin_popcount(m), sum, ec, es, tc, ts);  // (its sync: the zeros)
    uint32_t cur = (uint32_t)E0 + es;  // where the run before the thread's first record ended
    for (uint32_t mm = m; mm; mm &= mm - 1) {
#if ONO_PL_UNITS_REG
        const uint32_t e = (uint32_t)__builtin_ctz(mm), k = j0 + e, off = U.sel(e), len = U.sel(e + 2);
#else
        const uint32_t e = (uint32_t)__builtin_ctz(mm), k = j0 + e, off = lw[k], len = lw[k + 2];
#endif
        const uint32_t gi = cur + off;
        // (overflow-free: in a refuted stream cur + off may wrap; then gi < ea or it lies past eb)
        if (gi < ea || gi > eb || len > eb - gi || cur > eb || base + k + 4 + len > M32) {
            raise_bad(badw, epoch);  // only a refuted stream
            break;
        }
        uint16_t *d = img + (gi - ia);
        if (len <= (uint32_t)kShortP) {  // staged whole (kPatHalo)
#if ONO_PL_UNITS_REG
            for (uint32_t i = 0; i < len; i++) d[i] = e + 4 + i < 12u ? (uint16_t)U.sel(e + 4 + i) : lw[k + 4 + i];
#else
            for (uint32_t i = 0; i < len; i++) d[i] = lw[k + 4 + i];
#endif
        } else {
            const uint32_t q = atomicAdd(&lqn, 1u);
            const uint32_t vp = 8 + 2 * (base + k + 4);
            if (q < (uint32_t)kLQ) {
                lq[3 * q] = gi - ia;
                lq[3 * q + 1] = vp;
                lq[3 * q + 2] = len;
            } else {
                for (uint32_t i = 0; i < len; i++) d[i] = ((glb_u16 *)(b + vp))[i];
            }
        }
        cur = gi + len;
    }
    __syncthreads();  // the short runs and the long-run queue
    const uint32_t nl = min(lqn, (uint32_t)kLQ);
    if (nl) {  // (uniform) long runs: the whole workgroup copies each
        for (uint32_t q = 0; q < nl; q++) {
            const uint32_t a = lq[3 * q], vp = lq[3 * q + 1], c = lq[3 * q + 2];
            glb_u16 *src = (glb_u16 *)(b + vp);
            for (uint32_t i = threadIdx.x; i < c; i += kPatT) img[a + i] = src[i];
        }
        __syncthreads();
    }
    // the range out, widened to f32: whole 16-B vectors inside [ea, eb), then the partial first and
    // last vectors
    const uint32_t skip = ea - ia;
    float *gi0 = g + ia;
    if (vec) {
        const uint32_t v0 = skip ? 1u : 0u, v1 = n / 4;  // whole vectors [v0, v1)
        for (uint32_t i = v0 + threadIdx.x; i < v1; i += kPatT) {
            const uint2 h = img8[i];
            const f4s x = {from_f16_sp((uint16_t)h.x), from_f16_sp((uint16_t)(h.x >> 16)), from_f16_sp((uint16_t)h.y),
                           from_f16_sp((uint16_t)(h.y >> 16))};
            __builtin_nontemporal_store(x, (f4s *)gi0 + i);  // (write-through stores measured slower here: 25 vs 18.7 us)
        }
        if (threadIdx.x < 4) {
            const uint32_t e = threadIdx.x;
            if (skip && e >= skip && e < n) gi0[e] = from_f16_sp(img[e]);  // the first vector's part in range
            const uint32_t l = 4 * v1 + e;
            if (l < n && l >= 4 * v0) gi0[l] = from_f16_sp(img[l]);        // the last vector's part
        }
    } else {
        for (uint32_t i = threadIdx.x; i < n; i += kPatT) gi0[i] = from_f16_sp(img[i]);
    }
#ifdef ONO_SP_STAMP
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x < 64) sp_stamp(g_sp_stamp_plp, blockIdx.x, sp_t0, sp_tm);
#endif
}

// The stream-ordered lift in ONE launch (ono_sparse_lift_dev_async, up to kPatDirect tiles): each
// workgroup (tile t = blockIdx.x) stages its tile, finds and checks its candidates as pl_index does, publishes the
// tile's record — {sum of offset + length}, {exit, kPatNone without a candidate}, each an 8-byte
// granule {value, tag} written by one agent-scope store, so a reader needs no ordering — and adds its
// sum and an arrival to its chunk's line in each of kFusedRep replicas (kPatChunk tiles per 128-B
// line; one 64-bit agent-scope add: the sum in the low 40 bits, arrivals above; a reader polls one).  Its range start E_t is then the sum of the earlier
// chunks (each polled until all its tiles arrived) and of its chunk's earlier tiles (each polled
// until its granules carry this launch's tag); the link into it is the exit of the nearest earlier
// tile that holds a record.  Every poll is bounded: one that times out refutes the call (the caller
// takes the blocking lift), so no workgroup waits forever.  Then it places its range as pl_place
// does.  pl_index's launch, the boundary and pl_place's far prologue loads are gone.
// A tile waits only for lower tiles, and each XCD starts its workgroups in blockIdx order (observed,
// not promised by HIP: a tile's ticket from one counter, which promises it, measured ~88 tickets/us —
// 43 us for 3767 tiles, 77 us a lift); were that order ever broken, a poll would time out and the
// caller would take the blocking lift.  The tag is the call's epoch (so the stream-ordered lift is
// not for graph capture: a replay repeats it); a launch zeroes the chunk lines of the next.
constexpr int kStageU4 = kPatStage / 8 + 1;
constexpr int kPatChunk = 64;         // tiles per chunk line (kPatDirect / kPatChunk = 64 chunks: one per lane)
constexpr int kFusedLine = 16;        // u64 per chunk line (128 B)
#ifndef ONO_FUSED_REP
#define ONO_FUSED_REP 2
#endif
constexpr int kFusedRep = ONO_FUSED_REP;  // replicas of the chunk lines: a tile adds to all, a reader polls one
static_assert(kPatDirect / kPatChunk <= 64 && kPatChunk <= 64, "pl_fused's look-back: one chunk or tile per lane");
constexpr uint32_t kPollMax = 1u << 14;  // polls before a look-back gives up (~0.5-1 us each: ~10 ms)
// between polls: ~1000 cycles (a poll every 53 ns from every resident workgroup measured 77 us a lift:
// the polled lines' channels stall every other load)
#ifndef ONO_POLL_SLEEP
#define ONO_POLL_SLEEP 16
#endif
constexpr int kPollSleep = ONO_POLL_SLEEP;
// Residency bound: every workgroup counts itself in (one device-scope add) as it
// starts; a look-back that is still waiting while the count stays short of the grid and has not moved
// for kArriveTicks of the 100 MHz wall clock gives the call up (the status word), and so does one that
// sees the status raised.  Short work of another stream (a two-launch lift, a few tens of us) frees
// slots and the count moves on; a kernel of another stream or process that holds CU slots for long then
// costs ~100 us and a refusal (the caller's blocking lift does the work), not the ~10 ms poll limit and
// a wait for that kernel.
// The count is sharded (round 5): workgroup b adds to line b % 64, and the last of a line's workgroups
// to arrive resets it and adds one to the top word, which the look-back reads — one word taking every
// workgroup's add serialised them at ~88 per us (the guide's dequeue row): 1256 workgroups, +14 us
// before the last could start its look-back (the 64 MiB lift 22.9 -> 36.8 us per call,
// profiles/r05_mid_sp_phases.txt; sharded 23.9-24.1 us, profiles/r05_s45_lift_ab.txt; the add's value
// used only after the first tile is indexed 23.6-23.9 us against round 4's 22.7-23.2 on the same box,
// r05_s48).  (No-return adds summed by the check instead: 26.4-26.9 us — the check's 64 loads per
// waiting lane, r05_s46; a check every 64 polls instead of 16: no change, r05_s48.)
constexpr uint64_t kArriveTicks = 10000;  // 100 us without a new arrival
#ifndef ONO_ARRIVE_EVERY
#define ONO_ARRIVE_EVERY 16
#endif
constexpr uint32_t kArriveEvery = ONO_ARRIVE_EVERY;  // polls between two residency checks (~8 us)
constexpr uint32_t kArriveShards = 64;     // lines of the count (16 u64 each), then the top word's line
// ONO_LIFT_PROGRESS (default): no count at all — a waiting lane gives the call up when the words it polls
// (its chunk line's arrival count, its tile's granules) have not changed for kArriveTicks: a producer
// that runs publishes within microseconds of starting, so a standstill that long means it is not
// resident (the same bound as the count's, without its adds: see DESIGN §3)
#ifndef ONO_LIFT_PROGRESS
#define ONO_LIFT_PROGRESS 1
#endif
// (two halves: the add is issued with the tile's loads, its returned value used only after the first tile
// is indexed, so no wave waits for it)
__device__ __forceinline__ uint64_t arrive_add(uint64_t *arrive) {
#if defined(ONO_NO_ARRIVE) || ONO_LIFT_PROGRESS  // (no residency count)
    return ~0ull;
#endif
    return __hip_atomic_fetch_add(arrive + (size_t)(blockIdx.x % kArriveShards) * 16, (uint64_t)1, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void arrive_done(uint64_t *arrive, uint64_t old) {
    const uint32_t G = gridDim.x, sh = blockIdx.x % kArriveShards;
    const uint64_t cnt = (G - sh + kArriveShards - 1) / kArriveShards;  // this line's workgroups
    if (old + 1 == cnt) {  // the line's last: every add of this launch to it is in
        __hip_atomic_store(arrive + (size_t)sh * 16, (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(arrive + (size_t)kArriveShards * 16, (uint64_t)1, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
}
__device__ __forceinline__ uint64_t ld_agent(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
struct FusedGrid {
    const uint64_t *arrive;  // the stream's count of complete arrival lines (the top word, monotonic)
    uint64_t target;         // its value once this launch's whole grid has started
    const uint64_t *badw;    // the call's status word (raise_bad)
    uint32_t epoch;
    uint64_t seen = 0, since = 0;  // the count last read, and when it last moved
    __device__ bool give_up() {
        if (*(const volatile uint64_t *)badw == (uint64_t)epoch) return true;  // refused elsewhere
#ifdef ONO_NO_ARRIVE
        return false;
#endif
        const uint64_t c = ld_agent(arrive), now = wall_clock64();
        if (c >= target) return false;  // the whole grid is resident: the awaited tiles will come
        if (c != seen || since == 0) {
            seen = c;
            since = now;
            return false;
        }
        return now - since > kArriveTicks;
    }
    // the progress form (ONO_LIFT_PROGRESS): the lane's polled words (key) unchanged for kArriveTicks
    __device__ bool stalled(uint64_t key) {
        if (*(const volatile uint64_t *)badw == (uint64_t)epoch) return true;  // refused elsewhere
        const uint64_t now = wall_clock64();
        if (key != seen || since == 0) {
            seen = key;
            since = now;
            return false;
        }
        return now - since > kArriveTicks;
    }
    __device__ bool check(uint64_t key) {
#if ONO_LIFT_PROGRESS
        return stalled(key);
#else
        (void)key;
        return give_up();
#endif
    }
};
__device__ __forceinline__ void st_agent(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// pl_fused's staging (an 8-B aligned stream), 8 B per load: every tile's loads issued up front,
// the first tile's first (a scheduling barrier keeps them ahead: the wait for them lets the later
// tiles' loads stay in flight while the first tile is indexed and published), unconditional and
// clamped into the tile — or onto the total when the tile has no 8-B word — so that no wait comes
// before the last issue.  Tile q of the workgroup is blockIdx.x + q * gridDim.x.
constexpr int kStageK = (kPatStage / 4 + kPatT - 1) / kPatT;  // 8-B loads per thread per tile
template <int TPW>
__device__ __forceinline__ void pat_stage_issue(uint2 (&v)[TPW][kStageK], uint32_t (&n16)[TPW], const uint8_t *b,
                                                size_t M, size_t T) {
#pragma unroll
    for (int q = 0; q < TPW; q++) {
        const size_t t = blockIdx.x + (size_t)q * gridDim.x, base = t * kPatU;
        n16[q] = t < T ? (uint32_t)min(M - base, (size_t)kPatStage) : 0u;
        const uint32_t n8 = (n16[q] + 3) / 4;  // (the last word may hold units past M: same page, unused)
        const uint2 *src = n8 ? (const uint2 *)(b + 8 + 2 * base) : (const uint2 *)b;
#pragma unroll
        for (int k = 0; k < kStageK; k++) {
            const uint32_t i = threadIdx.x + (uint32_t)k * kPatT;
            v[q][k] = src[i < n8 ? i : 0u];
        }
        if (q == 0) __builtin_amdgcn_sched_barrier(0);
    }
}
// tile q's loaded words into LDS (no loads of its own: a load loop here would make every later wait
// a wait for all loads in flight)
__device__ __forceinline__ void pat_stage_write(uint4 *lw4, const uint2 (&v)[kStageK], uint32_t n16) {
    uint2 *dst = (uint2 *)lw4;
#pragma unroll
    for (int k = 0; k < kStageK; k++) {
        const uint32_t i = threadIdx.x + (uint32_t)k * kPatT;
        if (i < (n16 + 3) / 4) dst[i] = v[k];
    }
}

// pl_fused's look-back for tile t, one wave: E_t (the sum of the earlier chunks' sums, each polled in
// replica `rep` until all its tiles arrived, and of the earlier tiles of t's chunk, each polled until
// its granules carry the call's tag: one round of loads for both, repeated for the lanes still
// waiting) and the exit of the nearest earlier tile that holds a record.  False: a poll timed out.
__device__ __forceinline__ bool fused_lookback(uint32_t t, uint32_t tagv, const uint64_t *frec, const uint64_t *fchunk,
                                               uint32_t gcap, uint32_t rep, uint64_t &E, bool &found,
                                               uint32_t &pexit, FusedGrid fg) {
    const uint32_t lane = threadIdx.x & 63, c = t / kPatChunk, c0 = c * kPatChunk;
    bool timeout = false;
    const bool wchunk = lane < c, wtile = c0 + lane < t;
    const uint64_t *w = fchunk + ((size_t)rep * gcap + lane) * kFusedLine;
    const uint64_t *r = frec + 2 * (size_t)(c0 + lane);
    uint64_t v = 0, a = 0, x3 = 0;
    for (uint32_t it = 0;; it++) {
        if (wchunk) v = ld_agent(w);
        if (wtile) {
            a = ld_agent(r);
            x3 = ld_agent(r + 1);
        }
        const bool ready = (!wchunk || (v >> 40) == (uint64_t)kPatChunk) &&
                           (!wtile || ((a >> 32) == tagv && (x3 >> 32) == tagv));
        if (ready) break;
        if (it > kPollMax || (it % kArriveEvery == kArriveEvery - 1 && fg.check(v ^ (a * 0x9E3779B97F4A7C15ull) ^ x3))) {
            timeout = true;
            break;
        }
        __builtin_amdgcn_s_sleep(kPollSleep);
    }
    uint64_t part = (wchunk ? v & ((1ull << 40) - 1) : 0ull) + (wtile ? (uint32_t)a : 0u);
    const uint32_t ex = (uint32_t)x3;
    // the lanes' parts (each < 2^40) summed exactly
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) part += (uint64_t)__shfl_xor((long long)part, d, 64);
    E = part;
    const uint64_t hold = __ballot(wtile && ex != kPatNone);
    found = hold != 0;
    pexit = found ? (uint32_t)__builtin_amdgcn_readlane((int)ex, 63 - __clzll((long long)hold)) : 0u;
    // none in this chunk: earlier chunks, 64 tiles at a time, nearest first (all published)
    for (int64_t hi = (int64_t)c0; !found && hi > 0 && !timeout; hi -= 64) {
        const int64_t i = hi - 1 - (int64_t)lane;
        uint32_t xe = kPatNone;
        if (i >= 0) {
            const uint64_t *rr = frec + 2 * (size_t)i + 1;
            uint64_t x = ld_agent(rr);
            for (uint32_t it = 0; (x >> 32) != tagv; it++) {
                if (it > kPollMax || (it % kArriveEvery == kArriveEvery - 1 && fg.check(x))) { timeout = true; break; }
                __builtin_amdgcn_s_sleep(kPollSleep);
                x = ld_agent(rr);
            }
            xe = (uint32_t)x;
        }
        const uint64_t h = __ballot(i >= 0 && xe != kPatNone);
        if (h) {
            found = true;
            pexit = (uint32_t)__builtin_amdgcn_readlane((int)xe, __ffsll((unsigned long long)h) - 1);
        }
    }
    return __ballot(timeout) == 0;
}

// TPW tiles per workgroup, tile q = blockIdx.x + q * gridDim.x: every tile staged, indexed and published
// first, then each in turn looked back and placed — the first tiles' ranges depend only on the first
// tiles, published early, so their stores start while the later tiles' look-backs are still waiting.
template <int TPW>
__global__ __launch_bounds__(kPatT) __attribute__((amdgpu_waves_per_eu(6))) void pl_fused(
    float *g, const uint8_t *b, size_t M, size_t T, size_t cap, int vec,
                                                  uint64_t *frec, uint64_t *fchunk, uint64_t *fchunk_next,
                                                  uint32_t gcap, uint64_t *host_word, uint64_t *badw, uint32_t epoch, uint64_t *arrive, uint64_t arrive_target,
                                                  uint64_t *done_word, uint64_t *done_arrive, uint64_t done_target, uint32_t done_sig,
                                                  int force_bad) {
    __shared__ uint4 img16[kPatImg / 8];  // a range as f16 bits (12 KiB), widened on the way out
    __shared__ uint4 lw4[TPW][kStageU4];
    __shared__ uint32_t lq[3 * kLQ], lqn;
    __shared__ uint16_t lmask[kPatT], lpre[kPatT];
    __shared__ uint32_t s_first[TPW], s_exit[TPW], s_bad, s_pexit, s_found;
    __shared__ uint64_t s_E0;
    uint2 *img8 = (uint2 *)img16;
    uint16_t *img = (uint16_t *)img16;
    SP_CLOCK(sp_t0);
    const uint32_t M32 = (uint32_t)M, T32 = (uint32_t)T, G = gridDim.x;
    if (threadIdx.x == 0) {
#pragma unroll
        for (int q = 0; q < TPW; q++) s_first[q] = s_exit[q] = kPatNone;
        s_bad = 0;
    }
    const uint32_t tagv = epoch;  // (never 0: frec starts zeroed)
    if (force_bad && blockIdx.x == 0 && threadIdx.x == 0) raise_bad(badw, epoch);  // (ono_sparse_lift_debug_refuse)
    uint2 v[TPW][kStageK];
    uint32_t n16[TPW];
    // the total (b is 8-B aligned: the host launches pl_fused for no other stream), issued first, from a
    // lane-dependent address that is always b (cap < 2^32 on this path): a uniform load would be moved
    // to a scalar register at once, waiting for it before the tiles' loads are issued
    const uint64_t total = *(const uint64_t *)(b + 8 * (threadIdx.x * (cap >> 62)));
    __builtin_amdgcn_sched_barrier(0);
    pat_stage_issue<TPW>(v, n16, b, M, T);
    // counted in once its loads are in flight
    uint64_t arr_old = 0;
    if (threadIdx.x == 0) arr_old = arrive_add(arrive);
    // pl_index's part per tile: candidates, their counts and sums, the successor checks inside the tile;
    // then the tile published: its two granules {sum}, {exit: kPatNone for no candidate}, and its
    // chunk's sum and arrival in every replica
    const uint32_t j0 = kPatPer * threadIdx.x;
    uint32_t m[TPW], es[TPW], tc[TPW], ts[TPW];
#pragma unroll
    for (int q = 0; q < TPW; q++) {
        const uint32_t t = blockIdx.x + q * G, base = t * (uint32_t)kPatU;
        m[q] = es[q] = tc[q] = ts[q] = 0;
        if (t >= T32) continue;  // (uniform)
        pat_stage_write(lw4[q], v[q], n16[q]);
        __syncthreads();
        const Units12 U = units12(lw4[q]);
        uint32_t sum, ec;
        m[q] = base + j0 < M32 ? pat_mask(U, base + j0, M, sum) : (sum = 0, 0u);
        block_scan2<kPatT>((uint32_t)__builtin_popcount(m[q]), sum, ec, es[q], tc[q], ts[q]);
        lmask[threadIdx.x] = (uint16_t)m[q];
        lpre[threadIdx.x] = (uint16_t)ec;
        if (m[q] && ec == 0) s_first[q] = base + j0 + (uint32_t)__builtin_ctz(m[q]);
        __syncthreads();
        bool bad = false;
        uint32_t rank = ec;
        for (uint32_t mm = m[q]; mm; mm &= mm - 1, rank++) {
            const uint32_t e = (uint32_t)__builtin_ctz(mm), k = j0 + e;
#if ONO_PL_UNITS_REG
            const uint32_t nx = k + 4 + U.sel(e + 2);  // tile-local successor
#else
            const uint32_t nx = k + 4 + lw4u16(lw4[q])[k + 2];  // tile-local successor
#endif
            if (base + nx > M32) { bad = true; break; }  // the run overruns the stream
            if (nx < (uint32_t)kPatU && base + nx < M32) {
                const uint32_t m2 = lmask[nx / kPatPer], b2 = nx % kPatPer;
                const uint32_t p2 = lpre[nx / kPatPer] + (uint32_t)__builtin_popcount(m2 & ((1u << b2) - 1u));
                if (!(m2 >> b2 & 1u) || p2 != rank + 1) { bad = true; break; }
            } else {  // the end of the stream or another tile: only the tile's last candidate goes there
                if (rank + 1 != tc[q]) { bad = true; break; }
                s_exit[q] = base + nx;
            }
        }
        if (bad) s_bad = 1;
        __syncthreads();  // (lmask, lpre and the scan's words are reused by the next tile; s_exit is read)
        if (threadIdx.x < kFusedRep) {
            if (threadIdx.x == 0) {
                const uint64_t tag = (uint64_t)tagv << 32;
                uint64_t *r = frec + 2 * (size_t)t;
                st_agent(r, tag | ts[q]);
                st_agent(r + 1, tag | (tc[q] ? s_exit[q] : kPatNone));
            }
            atomicAdd((unsigned long long *)(fchunk + ((size_t)threadIdx.x * gcap + t / kPatChunk) * kFusedLine),
                      (unsigned long long)ts[q] | 1ull << 40);
        }
    }
    if (threadIdx.x == 0) arrive_done(arrive, arr_old);
    if (s_bad && threadIdx.x == 0) raise_bad(badw, epoch);
    // (checked after the tiles are published, before any look-back: uniform over the grid, so nobody
    // waits; checked first, the compiler would sink the later tiles' loads behind the total's)
    if (total > cap) {  // ONO_E_SIZE: nothing is written
        if (blockIdx.x == 0 && threadIdx.x == 0) raise_bad(badw, epoch);
        // the next launch's chunk lines are zeroed on this path too: the host flips the pair either way,
        // and a line left holding this launch's counts would look complete to the next-but-one launch
        for (uint32_t i = blockIdx.x * kPatT + threadIdx.x; i < kFusedRep * gcap; i += G * kPatT)
            fchunk_next[(size_t)i * kFusedLine] = 0;
        if (done_word) grid_complete(done_word, done_arrive, done_target, done_sig);
        return;
    }
    const uint32_t total32 = (uint32_t)total;
#pragma unroll
    for (int q = 0; q < TPW; q++) {  // the tiles in turn, the image reused
        const uint32_t t = blockIdx.x + q * G, base = t * (uint32_t)kPatU;
        if (t >= T32) break;  // (uniform)
        if (threadIdx.x < 64) {
            uint64_t E;
            bool f;
            uint32_t px;
            const bool ok = fused_lookback(t, tagv, frec, fchunk, gcap, blockIdx.x % kFusedRep, E, f, px,
                                           FusedGrid{arrive + (size_t)kArriveShards * 16, arrive_target, badw, epoch});
            if (threadIdx.x == 0) {
                s_E0 = E;
                s_found = ok && f ? 1u : 0u;
                s_pexit = px;
                if (!ok) raise_bad(badw, epoch);
            }
        }
        __syncthreads();
#ifdef ONO_SP_STAMP
        if (q == 0) {
            SP_CLOCK(sp_tl);
            if (threadIdx.x == 0) g_sp_stamp_plf[blockIdx.x] = make_uint4(0u, 0u, (unsigned)(sp_tl - sp_t0), 0u);
        }
#endif
        const uint64_t E0 = s_E0, E1 = E0 + ts[q];
        const bool found = s_found != 0;
        const uint32_t pexit = s_pexit;
        {
            bool bad = tc[q] > 0 && (found ? pexit != s_first[q] : s_first[q] != 0u);
            if (t + 1 == T32) bad |= (tc[q] > 0 ? s_exit[q] != M32 : !found || pexit != M32) || E1 > total;
            if (bad && threadIdx.x == 0) raise_bad(badw, epoch);
        }
        const uint32_t ea = (uint32_t)min(E0, total);
        const uint32_t eb = max(t + 1 == T32 ? total32 : (uint32_t)min(E1, total), ea);
        const uint32_t ia = vec ? ea & ~3u : ea;
        const uint32_t n = min(eb - ia, (uint32_t)kPatImg + 1);
        const bool is_wide = eb > ea && n > (uint32_t)kPatImg;
        if (is_wide) {  // (uniform) window by window
            wide_tile(g, b, M, T, vec, t, E0, ts[q], total, false, img8, lw4[q], lq, &lqn, nullptr, nullptr, 0,
                      host_word, badw, epoch);
        } else if (eb != ea) {
            const uint16_t *lw = (const uint16_t *)lw4[q];
            for (uint32_t i = threadIdx.x; i < (n + 7) / 8; i += kPatT) img16[i] = make_uint4(0u, 0u, 0u, 0u);
            if (threadIdx.x == 0) lqn = 0;
#if ONO_PL_UNITS_REG
            const Units12 U = units12(lw4[q]);  // (the thread's units from registers below)
#endif
            __syncthreads();
            uint32_t cur = (uint32_t)E0 + es[q];  // where the run before the thread's first record ended
            for (uint32_t mm = m[q]; mm; mm &= mm - 1) {
#if ONO_PL_UNITS_REG
                const uint32_t e = (uint32_t)__builtin_ctz(mm), k = j0 + e, off = U.sel(e), len = U.sel(e + 2);
#else
                const uint32_t e = (uint32_t)__builtin_ctz(mm), k = j0 + e, off = lw[k], len = lw[k + 2];
#endif
                const uint32_t gi = cur + off;
                if (gi < ea || gi > eb || len > eb - gi || cur > eb || base + k + 4 + len > M32) {
                    raise_bad(badw, epoch);  // only a refuted stream
                    break;
                }
                uint16_t *d = img + (gi - ia);
                if (len <= (uint32_t)kShortP) {  // staged whole (kPatHalo)
#if ONO_PL_UNITS_REG
                    for (uint32_t i = 0; i < len; i++) d[i] = e + 4 + i < 12u ? (uint16_t)U.sel(e + 4 + i) : lw[k + 4 + i];
#else
                    for (uint32_t i = 0; i < len; i++) d[i] = lw[k + 4 + i];
#endif
                } else {
                    const uint32_t qq = atomicAdd(&lqn, 1u);
                    const uint32_t vp = 8 + 2 * (base + k + 4);
                    if (qq < (uint32_t)kLQ) {
                        lq[3 * qq] = gi - ia;
                        lq[3 * qq + 1] = vp;
                        lq[3 * qq + 2] = len;
                    } else {
                        for (uint32_t i = 0; i < len; i++) d[i] = ((glb_u16 *)(b + vp))[i];
                    }
                }
                cur = gi + len;
            }
            __syncthreads();  // the short runs and the long-run queue
            const uint32_t nl = min(lqn, (uint32_t)kLQ);
            if (nl) {  // (uniform) long runs: the whole workgroup copies each
                for (uint32_t qq = 0; qq < nl; qq++) {
                    const uint32_t a = lq[3 * qq], vp = lq[3 * qq + 1], cn = lq[3 * qq + 2];
                    glb_u16 *src = (glb_u16 *)(b + vp);
                    for (uint32_t i = threadIdx.x; i < cn; i += kPatT) img[a + i] = src[i];
                }
                __syncthreads();
            }
            const uint32_t skip = ea - ia;
            float *gi0 = g + ia;
            if (vec) {
                const uint32_t v0 = skip ? 1u : 0u, v1 = n / 4;  // whole vectors [v0, v1)
                for (uint32_t i = v0 + threadIdx.x; i < v1; i += kPatT) {
                    const uint2 h = img8[i];
                    const f4s x = {from_f16_sp((uint16_t)h.x), from_f16_sp((uint16_t)(h.x >> 16)),
                                   from_f16_sp((uint16_t)h.y), from_f16_sp((uint16_t)(h.y >> 16))};
                    __builtin_nontemporal_store(x, (f4s *)gi0 + i);
                }
                if (threadIdx.x < 4) {
                    const uint32_t e = threadIdx.x;
                    if (skip && e >= skip && e < n) gi0[e] = from_f16_sp(img[e]);
                    const uint32_t l = 4 * v1 + e;
                    if (l < n && l >= 4 * v0) gi0[l] = from_f16_sp(img[l]);
                }
            } else {
                for (uint32_t i = threadIdx.x; i < n; i += kPatT) gi0[i] = from_f16_sp(img[i]);
            }
        }
        __syncthreads();  // (the image and the look-back's words are reused by the next tile)
    }
    // the next launch's chunk lines back to zero (the previous launch, which used them, is done; at the
    // end: a store loop ahead of the first waits would make them wait for every load in flight)
    for (uint32_t i = blockIdx.x * kPatT + threadIdx.x; i < kFusedRep * gcap; i += G * kPatT)
        fchunk_next[(size_t)i * kFusedLine] = 0;
    // the TCP ring's lift: the last workgroup to finish tells the host (with every refusal before it)
    if (done_word) grid_complete(done_word, done_arrive, done_target, done_sig);
#ifdef ONO_SP_STAMP
    SP_CLOCK(sp_tm);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x < 64) sp_stamp(g_sp_stamp_plp, blockIdx.x, sp_t0, sp_tm);
#endif
}

// The tiles pl_place flagged, one workgroup each, grid-stride over the tiles.
__global__ __launch_bounds__(kPatT) void pl_wide(float *g, const uint8_t *b, size_t M, size_t T, int vec,
                                                 const uint64_t *E, const uint32_t *tsum, const uint32_t *wide,
                                                 uint4 *queue, uint32_t *qcount, uint32_t qcap, uint64_t *host_word,
                                                 uint64_t *badw, uint32_t epoch) {
    __shared__ uint2 img8[kPatImg / 4];
    __shared__ uint4 lw4[kPatStage / 8 + 1];
    __shared__ uint32_t lq[3 * kLQ], lqn;
    const uint64_t total = stream_total(b);
    for (size_t t = blockIdx.x; t < T; t += gridDim.x) {
        if (!wide[t]) continue;  // (uniform)
        wide_tile(g, b, M, T, vec, t, E[t], tsum[t], total, true, img8, lw4, lq, &lqn, queue, qcount, qcap,
                  host_word, badw, epoch);
    }
}

// The lift's completion: one lane stores the call's epoch into a host-mapped
// word once every earlier launch on the stream has finished; the host spins on
// that word instead of a stream synchronisation (see host_wait).
__global__ void sp_signal(uint64_t *host_word, uint32_t epoch) {
    if (threadIdx.x == 0) __hip_atomic_store(host_word, (uint64_t)epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// the totals into the host-mapped words (the exact-size path of a small buffer), one wave
// (agg: the call's aggregates; state != NULL: the count + emit form, whose array sp_count named in state[1])
__global__ void sp_totals_out(const uint4 *agg, size_t half, const uint32_t *state, uint32_t G, uint64_t *host_tot) {
    if (state && (state[1] & 1u)) agg += half;
    const uint2 t = chunk_totals(agg, G);
    if (threadIdx.x == 0) {
        host_tot[0] = t.x;
        host_tot[1] = t.y;
    }
}

// Scratch of the encoder (tile records, prefixes, the tile images, two host-
// mapped words for the result), kept per (device, stream) and grown on
// demand: the stream-ordered allocations it replaces cost more than the
// kernels at 64 MiB.  Per stream, so stream-ordered drops on different
// streams never share it (on one stream they are ordered anyway).
struct Scratch {
    uint32_t calls = 0;       // the blocking drop's completion signal: a per-call tag in host_tot[2]
    size_t tiles_cap = 0;
    uint2 *rec = nullptr;     // 2 x tiles_cap: recA, then recB
    // two arrays of agg_cap chunk aggregates: call k accumulates into agg[parity] and zeroes the
    // other one for call k + 1 (zeroed when allocated; flipped once a call's sp_image is launched)
    uint4 *agg = nullptr;
    size_t agg_cap = 0;
    int parity = 0;
    uint16_t *img = nullptr;  // img_cap slots of kSlotU16 units (5 B per value): sp_image / sp_move
    size_t img_cap = 0;
    uint32_t *mask = nullptr;  // mask_cap tiles of 64 keep words (N / 8 bytes): sp_count / sp_emit
    uint16_t *cv = nullptr;    // mask_cap tile slots of kTile f16 (the kept values, compact): sp_count / sp_emit
    size_t mask_cap = 0;
    uint64_t *host_tot = nullptr, *host_tot_dev = nullptr;  // [F, R, the completion tag, the error word]
    // the one-launch form (sp_drop1): 4 granules per tile and per group of tiles (zeroed when
    // allocated, and when the epoch wraps), the call's epoch
    uint64_t *desc = nullptr;
    size_t desc_cap = 0;
    uint32_t depoch = 0;
    // the blocking one launch's in-kernel completion: workgroups counted in (device, never reset), and the
    // count the call before this one ended at
    uint64_t *arrive = nullptr;
    uint64_t arrive_base = 0;
    // count + emit: the aggregate parity on the device ([0] the array sp_count adds into, flipped by
    // sp_emit; [1] the array of the call in flight, for sp_totals_out), zeroed with agg
    uint32_t *state = nullptr;
    // the host's copy of state[0] while every call on the stream was uncaptured (par_known): sp_emit then takes
    // it as an argument and loads one array; after a capture only the device knows it (sp_emit<.., true>)
    bool par_known = true;
    uint32_t hpar = 0;
    // a graph captured a call on this stream: its kernels hold these arrays, so they are never freed or
    // regrown in place (a larger call moves them to `retired` and allocates new ones)
    bool captured = false;
    // sp_count ran without its sp_emit (a failed launch): the aggregates are re-zeroed before the next call
    bool dirty = false;
    std::vector<void *> retired;
};
std::mutex g_scratch_mu;
std::map<std::pair<int, hipStream_t>, Scratch> g_scratch;

int scratch_for(size_t ntiles, hipStream_t stream, Scratch **out, bool image = true, bool emit = false) {
    int dev = 0;
    ONO_HIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) return set_error(ONO_E_ARG, "device %d", dev);
    Scratch &sc = g_scratch[{dev, stream}];
    if (!sc.host_tot) {
        ONO_HIP(hipHostMalloc((void **)&sc.host_tot, 4 * sizeof(uint64_t), hipHostMallocMapped | hipHostMallocCoherent));
        ONO_HIP(hipHostGetDevicePointer((void **)&sc.host_tot_dev, sc.host_tot, 0));
        sc.host_tot[3] = 0;
    }
    if (!sc.arrive) {
        ONO_HIP(hipMalloc((void **)&sc.arrive, 64));
        ONO_HIP(hipMemsetAsync(sc.arrive, 0, 64, stream));
        sc.arrive_base = 0;
    }
    if (!image) {  // sp_drop1's granules instead of the slot image
        const size_t want = std::max<size_t>(ntiles + (ntiles + kDropGroup - 1) / kDropGroup, 1);  // tiles, groups
        if (want > sc.desc_cap) {
            (void)hipFree(sc.desc);
            sc.desc = nullptr;
            sc.desc_cap = 0;
            ONO_HIP(hipMalloc((void **)&sc.desc, 4 * want * sizeof(uint64_t)));
            ONO_HIP(hipMemsetAsync(sc.desc, 0, 4 * want * sizeof(uint64_t), stream));
            sc.desc_cap = want;
        }
        *out = &sc;
        return ONO_OK;
    }
    // a captured graph's arrays are retired, not freed (the graph may be replayed as long as it exists)
    auto drop_arr = [&sc](void *p) {
        if (!p) return;
        if (sc.captured) sc.retired.push_back(p);
        else (void)hipFree(p);
    };
    if (ntiles > sc.tiles_cap || !sc.state) {
        drop_arr(sc.rec);
        drop_arr(sc.agg);
        drop_arr(sc.state);
        sc.rec = nullptr;
        sc.agg = nullptr;
        sc.state = nullptr;
        sc.tiles_cap = sc.agg_cap = 0;
        const size_t tc = std::max<size_t>(ntiles, 1), gcap = (tc + kRecChunk - 1) / kRecChunk;
        ONO_HIP(hipMalloc((void **)&sc.rec, 2 * tc * sizeof(uint2)));
        ONO_HIP(hipMalloc((void **)&sc.agg, gcap * kAggStride * sizeof(uint4)));  // (both arrays: kAggHalf)
        ONO_HIP(hipMemsetAsync(sc.agg, 0, gcap * kAggStride * sizeof(uint4), stream));
        ONO_HIP(hipMalloc((void **)&sc.state, 16 * sizeof(uint32_t)));
        ONO_HIP(hipMemsetAsync(sc.state, 0, 16 * sizeof(uint32_t), stream));
        sc.tiles_cap = tc;
        sc.agg_cap = gcap;
        sc.parity = 0;
        sc.dirty = false;
        sc.par_known = true;
        sc.hpar = 0;
    }
    if (!emit && ntiles > sc.img_cap) {
        drop_arr(sc.img);
        sc.img = nullptr;
        sc.img_cap = 0;
        ONO_HIP(hipMalloc((void **)&sc.img, ntiles * kSlotU16 * sizeof(uint16_t)));
        sc.img_cap = ntiles;
    }
    if (emit && (ntiles > sc.mask_cap || !sc.mask)) {
        drop_arr(sc.mask);
        drop_arr(sc.cv);
        sc.mask = nullptr;
        sc.cv = nullptr;
        sc.mask_cap = 0;
        const size_t tc = std::max<size_t>(ntiles, 1);
        ONO_HIP(hipMalloc((void **)&sc.mask, tc * 64 * sizeof(uint32_t)));
        ONO_HIP(hipMalloc((void **)&sc.cv, tc * kTile * sizeof(uint16_t)));
        sc.mask_cap = tc;
    }
    *out = &sc;
    return ONO_OK;
}
// Under stream capture nothing may be allocated or zeroed (a memset would become a graph node that every
// replay runs; an allocation is not allowed while the stream captures): the call's arrays must exist from
// an earlier uncaptured call on the stream.  Returns the scratch, or NULL.
Scratch *scratch_ready(size_t ntiles, hipStream_t stream) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    auto it = g_scratch.find({dev, stream});
    if (it == g_scratch.end()) return nullptr;
    Scratch &sc = it->second;
    if (!sc.host_tot || !sc.state || !sc.mask || sc.dirty || ntiles > sc.tiles_cap || ntiles > sc.mask_cap) return nullptr;
    return &sc;
}

struct LiftScratch {
    size_t seg_cap = 0, win_cap = 0, q_cap = 0, buf_cap = 0;
    uint32_t *seg = nullptr;   // 4 x seg_cap: p0, gpre, rcnt, reached (epoch stamps, zeroed when allocated)
    uint4 *ent = nullptr;      // kRecK x seg_cap: the walks' records
    uint32_t *win = nullptr;   // wsum (W), then the long-run queue's count
    uint4 *queue = nullptr;    // q_cap chunks of long runs
    uint32_t epoch = 0;
    uint8_t *buf = nullptr;
    size_t pt_cap = 0;
    uint32_t *prec = nullptr;  // pattern path: 4 x pt_cap tile records, then pt_cap tile sums
    uint64_t *pE = nullptr;    // pattern path: pt_cap + 1 element prefixes
    uint32_t *pwide = nullptr; // pattern path: per tile, 1 = a wide range (for pl_wide)
    // [0] walk refuted / malformed (= epoch), [1] total, [2] pattern refuted (= epoch), [3] pattern queued a
    // chunk, [4] pattern listed a wide tile
    uint64_t *host_word = nullptr, *host_word_dev = nullptr;
};
LiftScratch g_lift[64];
// The stream-ordered lift's scratch, per (device, stream): calls on one stream are ordered, calls on
// different streams never share it.
struct PatScratch {
    size_t cap = 0;
    uint32_t *prec = nullptr;  // 4 x cap tile records, then cap tile sums
    uint64_t *pE = nullptr;    // cap + 1 element prefixes (pl_scan, wide tiles)
    uint32_t *pwide = nullptr; // (unused flags: pl_place<true> places wide tiles itself)
    uint64_t *aw = nullptr;    // 8 device words standing in for the blocking lift's host words
    uint32_t epoch = 0;
    // pl_fused: per tile 2 granules {value, epoch} (zeroed when allocated), two arrays of chunk lines
    // (kFusedRep replicas each) in turn (a launch zeroes the other for the next)
    size_t fcap = 0, fgcap = 0;
    uint64_t *frec = nullptr, *fchunk = nullptr;
    int fpar = 0;
    uint64_t *arrive = nullptr;  // pl_fused's arrival count: kArriveShards lines + the top word (zeroed once)
    uint64_t arrive_base = 0;    // the top word once every earlier launch's grid has started
    uint64_t *done_arrive = nullptr;  // pl_fused's completion count (a caller's word; grows, never reset)
    uint64_t done_base = 0;
};
std::map<std::pair<int, hipStream_t>, PatScratch> g_pat;
std::atomic<size_t> g_lift_fallbacks{0};      // lifts the host parsed (walk path refuted, or malformed)
std::atomic<uint32_t> g_lift_force_refuse{0};  // one-launch lifts still to be refused (a test hook)
std::atomic<size_t> g_lift_pattern_misses{0}; // lifts the pattern path handed to the walk path
std::atomic<int> g_lift_mode{0};              // 0: pattern, then walk, then host; 1: walk, then host

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

}  // namespace

namespace ono {
// f16 bits -> f32 on the host, as half 2.7.1 (and gfx950's v_cvt_f32_f16): exact, NaN -> sign |
// quiet bit | payload << 13
static float f16_to_f32_host(uint16_t h) {
    const uint32_t sign = (uint32_t)(h >> 15) << 31, e = (h >> 10) & 0x1Fu, m = h & 0x3FFu;
    uint32_t bits;
    if (e == 0x1F) bits = sign | (m ? 0x7FC00000u | m << 13 : 0x7F800000u);
    else if (e) bits = sign | (e + 112u) << 23 | m << 13;
    else if (!m) bits = sign;
    else {  // subnormal: m * 2^-24, normalised
        int sh = 0;
        uint32_t mm = m;
        while (!(mm & 0x400u)) { mm <<= 1; sh++; }
        bits = sign | (uint32_t)(113 - sh) << 23 | (mm & 0x3FFu) << 13;
    }
    float f;
    memcpy(&f, &bits, 4);
    return f;
}

// A SparseGrad whose total exceeds what its receiver uses (the scatter adds
// over the shorter length, worker_ring.rs:141-143): the reference's sequential
// parse validates the whole stream (its errors), but only values [0, L) are
// materialised — out[0, min(total, L)) on the host.  A frame's claimed total
// never sizes a device allocation.
int sparse_lift_prefix_host(const uint8_t *buf, size_t nbytes, float *out, size_t L, size_t *got) {
    uint64_t total = 0;
    if (nbytes < 8) return set_error(ONO_E_PROTO, "Missing total length bytes at grad lift");
    for (int q = 0; q < 8; q++) total |= (uint64_t)buf[q] << (8 * q);
    std::vector<uint64_t> start, cumF;
    int rc = lift_parse_host(buf, nbytes, total, start, cumF);
    if (rc) return rc;
    const size_t k = (size_t)std::min<uint64_t>(total, L);
    std::fill(out, out + k, 0.0f);
    for (size_t j = 0; j < start.size() && start[j] < k; j++) {
        const size_t len = (j + 1 < start.size() ? cumF[j + 1] : (nbytes - 8 - 8 * start.size()) / 2) - cumF[j];
        const uint8_t *v = buf + 16 + 8 * j + 2 * cumF[j];
        for (size_t i = 0; i < len && start[j] + i < k; i++) out[start[j] + i] = f16_to_f32_host((uint16_t)(v[2 * i] | v[2 * i + 1] << 8));
    }
    *got = (size_t)std::min<uint64_t>(total, (uint64_t)SIZE_MAX);
    return ONO_OK;
}
}  // namespace ono

namespace {
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

// The blocking calls' wait (lift, drop): a one-lane signal kernel behind the
// launches and a spin on its host-mapped word (a stream synchronisation's
// wake-up is the larger part of a blocking call's host time otherwise: 38.3-
// 39.0 against 42.4-42.7 us per 64 MiB lift, same box); after ~2 s without the
// signal (a faulted kernel) the stream synchronisation reports the error.
hipError_t host_spin(hipStream_t s, uint64_t *word_host, uint32_t epoch);
hipError_t host_wait(hipStream_t s, uint64_t *word_host, uint64_t *word_dev, uint32_t epoch) {
    volatile uint64_t *w = word_host;
    *w = 0;  // (a lift may wait more than once under one epoch)
    hipLaunchKernelGGL(sp_signal, dim3(1), dim3(64), 0, s, word_dev, epoch);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return host_spin(s, word_host, epoch);
}
// the spin of host_wait, on a word the stream's own kernel stores (sp_drop1's in-kernel completion)
hipError_t host_spin(hipStream_t s, uint64_t *word_host, uint32_t epoch) {
    volatile uint64_t *w = word_host;
    // A tight spin for the lift's own few tens of microseconds; beyond that the
    // stream had other work queued ahead of the call (training kernels before a
    // TCP hop's drop or lift), so the thread backs off — pause, then yield —
    // instead of burning a core while it holds the scratch lock, and past 2 s
    // it blocks in the runtime.
    const auto t0 = std::chrono::steady_clock::now();
    int mode = 0;  // 0 spin, 1 pause, 2 yield
    for (uint32_t i = 0; *w != epoch; i++) {
        if (mode == 1) __builtin_ia32_pause();
        else if (mode == 2) std::this_thread::yield();
        if ((i & 255) != 0) continue;
        const auto dt = std::chrono::steady_clock::now() - t0;
        if (dt > std::chrono::seconds(2)) return hipStreamSynchronize(s);
        mode = dt > std::chrono::microseconds(200) ? 2 : dt > std::chrono::microseconds(50) ? 1 : 0;
    }
    return hipSuccess;
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
    const size_t S = (nbytes - 8 + kSeg - 1) / kSeg, W = (S + kLW - 1) / kLW;
    if (!L.host_word) {
        ONO_HIP(hipHostMalloc((void **)&L.host_word, 8 * sizeof(uint64_t), hipHostMallocMapped | hipHostMallocCoherent));
        ONO_HIP(hipHostGetDevicePointer((void **)&L.host_word_dev, L.host_word, 0));
    }
    bool restamp = false;
    if (S > L.seg_cap) {
        (void)hipFree(L.seg);
        (void)hipFree(L.ent);
        L.seg = nullptr;
        L.ent = nullptr;
        L.seg_cap = 0;
        ONO_HIP(hipMalloc((void **)&L.seg, 4 * S * sizeof(uint32_t)));
        ONO_HIP(hipMalloc((void **)&L.ent, kRecK * S * sizeof(uint4)));
        L.seg_cap = S;
        restamp = true;
    }
    const size_t Wg = std::max<size_t>(1, W);  // (an empty stream still gets one: it resets the long-run queue)
    int rc = grow(&L.win, L.win_cap, Wg + 1);
    // chunks of runs longer than kShortP: at most one per kLongChunk values plus one per such run
    // queued chunks: of runs longer than kShortP (one per kLongChunk values plus one per such run) and of
    // the gaps of groups wider than kZeroMax (one per kLongChunk zeros plus one per record, and the tail)
    const size_t qcap = (nbytes - 8) / 8 + (nbytes - 8) / (8 + 2 * (kShortP + 1)) + 2 * (cap / kLongChunk) + 4;
    if (!rc) rc = grow(&L.queue, L.q_cap, qcap);
    if (rc) return rc;
    if (++L.epoch == 0) {  // stamps of 2^32 lifts ago could match again
        L.epoch = 1;
        restamp = true;
    }
    const size_t C = L.seg_cap;
    uint32_t *p0 = L.seg, *gpre = L.seg + C, *rcnt = L.seg + 2 * C, *reached = L.seg + 3 * C;
    if (restamp) ONO_HIP(hipMemsetAsync(reached, 0, C * sizeof(uint32_t), s));
    uint32_t *wsum = L.win, *qcount = L.win + Wg;
    volatile uint64_t *word = L.host_word;
    const uint32_t epoch = L.epoch;
    const int vec = ((uintptr_t)g & 15) == 0;
    // the pattern path first (streams of an even length with at least one unit)
    const size_t M = (nbytes - 8) / 2;
    if (g_lift_mode.load() == 0 && M > 0 && (nbytes & 1) == 0) {
        const size_t T = (M + kPatU - 1) / kPatU;
        if (T > L.pt_cap) {
            const size_t Tc = (T + 3) & ~(size_t)3;  // tile sums read as 16-B vectors
            (void)hipFree(L.prec);
            (void)hipFree(L.pE);
            (void)hipFree(L.pwide);
            L.prec = nullptr;
            L.pE = nullptr;
            L.pwide = nullptr;
            L.pt_cap = 0;
            ONO_HIP(hipMalloc((void **)&L.prec, 5 * Tc * sizeof(uint32_t)));  // records, then the sums again
            ONO_HIP(hipMalloc((void **)&L.pE, (Tc + 1) * sizeof(uint64_t)));
            ONO_HIP(hipMalloc((void **)&L.pwide, Tc * sizeof(uint32_t)));
            L.pt_cap = Tc;
        }
        word[1] = word[2] = word[3] = word[4] = 0;
        uint32_t *tsum = L.prec + 4 * L.pt_cap;
        ONO_HIP(launch_pl_index(dbuf, M, T, L.prec, tsum, qcount, L.pwide, L.host_word_dev, L.host_word_dev + 2, epoch,
                                s));
        if (T > kPatDirect)
            hipLaunchKernelGGL(pl_scan, dim3(1), dim3(kPatScanT), 0, s, dbuf, L.prec, T, L.pE, L.host_word_dev + 2, epoch);
        hipLaunchKernelGGL(pl_place<false>, dim3((unsigned)T), dim3(kPatT), 0, s, g, dbuf, M, T, cap, vec, L.pE, L.prec, tsum,
                           L.pwide, L.host_word_dev, L.host_word_dev + 2, epoch);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = host_wait(s, L.host_word + 5, L.host_word_dev + 5, epoch);
        if (e != hipSuccess) return hip_error(e, "sparse lift", __FILE__, __LINE__);
        const uint64_t total = word[1];
        if (total > cap) return size_error(total);
        if (word[2] != epoch && word[4] == epoch) {  // tiles with wide ranges (a sparse stream)
            hipLaunchKernelGGL(pl_wide, dim3((unsigned)std::min<size_t>(T, 2048)), dim3(kPatT), 0, s, g, dbuf, M, T,
                               vec, L.pE, tsum, L.pwide, L.queue, qcount, (uint32_t)qcap, L.host_word_dev,
                               L.host_word_dev + 2, epoch);
            e = hipGetLastError();
            if (e == hipSuccess) e = host_wait(s, L.host_word + 5, L.host_word_dev + 5, epoch);
            if (e != hipSuccess) return hip_error(e, "sparse lift", __FILE__, __LINE__);
        }
        if (word[2] != epoch) {
            if (word[3] == epoch) {  // long runs or wide gaps were queued
                hipLaunchKernelGGL(sl_long, dim3((unsigned)std::min<size_t>(2048, qcap)), dim3(kSB), 0, s, g, dbuf,
                                   L.queue, qcount, (uint32_t)qcap);
                e = hipGetLastError();
                if (e == hipSuccess) e = host_wait(s, L.host_word + 5, L.host_word_dev + 5, epoch);
                if (e != hipSuccess) return hip_error(e, "sparse lift", __FILE__, __LINE__);
            }
            *out_len = total;
            return ONO_OK;
        }
        g_lift_pattern_misses.fetch_add(1);  // not the pattern: the walk path parses it
    }
    word[0] = 0;
    word[1] = 0;
    hipLaunchKernelGGL(sl_index, dim3((unsigned)Wg), dim3(kLW), 0, s, dbuf, nbytes, S, epoch, p0, gpre, rcnt, L.ent,
                       reached, wsum, qcount, L.host_word_dev);
    hipLaunchKernelGGL(sl_place, dim3((unsigned)std::max<size_t>(1, (S + kPSeg - 1) / kPSeg)), dim3(kPT), 0, s, g,
                       dbuf, nbytes, S, cap, vec, epoch, p0, gpre, rcnt, L.ent, reached, wsum, L.queue, qcount,
                       (uint32_t)qcap, L.host_word_dev);
    hipLaunchKernelGGL(sl_long, dim3((unsigned)std::min<size_t>(2048, qcap)), dim3(kSB), 0, s, g, dbuf, L.queue,
                       qcount, (uint32_t)qcap);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = host_wait(s, L.host_word + 5, L.host_word_dev + 5, epoch);
    if (e != hipSuccess) return hip_error(e, "sparse lift", __FILE__, __LINE__);
    const uint64_t total = word[1];
    if (total > cap) return size_error(total);
    *out_len = total;
    if (word[0] != epoch) return ONO_OK;
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
// +inf), so this is an exact radix select over u32 keys.  Two launches when
// the sample is drawn: sp_gather_keys spreads the m random reads g[idx[i]]
// over many workgroups (one CU alone took 9-18 us for them) and leaves the
// keys where the indices were; sp_threshold then selects in one workgroup of
// eight waves, 32 keys per lane in registers, two bits per step from the top (round 5, bit-sliced): a
// lane's 32 keys are transposed into 32 bit planes (bit 31 - q of plane p = bit p of key q), so one step is four AND / popcount pairs on the lane's
// candidate mask for the whole 32 keys instead of 32 compares per bit; the counts of the digits
// 00 / 01 / 10 among the candidates are summed by two DPP reductions per wave (two counts packed in
// 16-bit halves) and across the eight waves in LDS, and the digit chosen by the rank still sought:
// 16 steps of a few hundred cycles.  (The compare-per-key form was VALU-bound on its one CU — 16384
// keys x 3 ops x 31 bits — at 20.5 us per call, the TCP ring's largest codec kernel.)  (Round 4's
// form, LDS-atomic histograms in 1024 threads, spent ~60 us in contended bins: the exponent byte of
// N(0, s) gradients puts most keys in a few of them.)
constexpr int kThrT = 512;
constexpr uint32_t kSampleMax = 16384;  // SAMPLE_SIZE, protocol.rs:13-19
constexpr int kThrK = (int)kSampleMax / kThrT;
static_assert(kThrK == 32, "a lane's keys are one 32 x 32 bit matrix");
constexpr int kGatherT = 256;
__device__ __forceinline__ uint32_t abs_key(float x) { return __builtin_bit_cast(uint32_t, x) & 0x7FFFFFFFu; }
// idx: device memory, or the caller's pinned host buffer read in place (no copy engine in between)
__global__ __launch_bounds__(kGatherT) void sp_gather_keys(const float *g, const uint32_t *idx, uint32_t *keys,
                                                           uint32_t m) {
    const uint32_t i = blockIdx.x * kGatherT + threadIdx.x;
    if (i < m) keys[i] = abs_key(g[idx[i]]);
}
// 32 x 32 bit transpose in registers (Hacker's Delight 7-3): afterwards bit 31 - c of A[r] is bit 31 - r
// of the former A[c]
__device__ __forceinline__ void transpose32(uint32_t (&A)[32]) {
    uint32_t m = 0x0000FFFFu;
#pragma unroll
    for (int j = 16; j != 0; j >>= 1, m ^= (m << j)) {
#pragma unroll
        for (int k = 0; k < 32; k = (k + j + 1) & ~j) {
            const uint32_t t = (A[k] ^ (A[k + j] >> j)) & m;
            A[k] ^= t;
            A[k + j] ^= t << j;
        }
    }
}
// keys: the gathered keys, or NULL: the sample is g[0, m) itself.  (Round 6 measured gathering g[idx[i]] here
// instead of in sp_gather_keys, one launch less: +10 us per SparseCapable push of the config-1 TCP ring — one
// workgroup's 16384 scattered loads cost more than the gather's launch; profiles/r06_s4_tcp_variants.jsonl.)
// The select stops early once the chosen digit leaves a single candidate (typically after 10-12 of the 16
// steps: 16384 samples near the 90th percentile differ within ~12 mantissa bits); that key is the answer, and
// the lane holding it reads it back from its bit planes (round 6: 9.5 vs 11.0 us per select, config-1 push,
// tools/thr_bench, profiles/r06_s26_thr_bench.json — where four bits a step, four waves of 64 keys a lane,
// and the gather and the select in one launch (the last workgroup to arrive selecting) all measured slower).
__global__ __launch_bounds__(kThrT) void sp_threshold(const uint32_t *keys, const float *g, uint32_t m, uint32_t k,
                                                      float *t_out) {
    __shared__ uint32_t wc[2][kThrT / 64][2];
    const int wave = threadIdx.x / 64;
    uint32_t A[32], C = 0;  // keys, then planes (plane p = A[31 - p]); candidates: bit 31 - q for key q
#pragma unroll
    for (int q = 0; q < kThrK; q++) {
        const uint32_t i = threadIdx.x + (uint32_t)q * kThrT;
        A[q] = i < m ? (keys ? keys[i] : abs_key(g[i])) : 0u;
        C |= i < m ? 1u << (31 - q) : 0u;
    }
    transpose32(A);
    uint32_t prefix = 0, kk = k, cand = m;
    bool one = false;
    // bits 30..1 two at a time (bit 31 is clear in every key), then bit 0
#pragma unroll
    for (int s = 0; s < 16; s++) {
        const int hi = 30 - 2 * s, lo = hi - 1;  // s == 15: hi = 0, lo = -1 (one bit)
        const uint32_t P1 = A[31 - hi], P0 = lo >= 0 ? A[31 - lo] : 0u;
        const uint32_t c0 = C & ~P1;
        const uint32_t x = (uint32_t)__popc(c0 & ~P0) | (uint32_t)__popc(c0 & P0) << 16;
        const uint32_t y = (uint32_t)__popc(C & P1 & ~P0);
        const uint32_t X = wsum(x), Y = lo >= 0 ? wsum(y) : 0u;
        const int par = s & 1;  // two count arrays: the next step's writes never meet this step's reads
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
        if (lo < 0) {  // one bit: n00 = candidates with a 0 there
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
        if (cand == 1 && lo > 0) {  // (uniform) one key left
            one = true;
            break;
        }
    }
    const float mp = 6.103515625e-05f;  // f16::MIN_POSITIVE
    uint32_t key = prefix;
    if (one) {
        if (!C) return;  // (the lane that holds the candidate writes)
        const int q = __builtin_clz(C);  // its bit is 31 - q: bit p of that key is bit 31 - q of plane p
        key = 0;
#pragma unroll
        for (int p = 0; p < 31; p++) key |= ((A[31 - p] >> (31 - q)) & 1u) << p;
    } else if (threadIdx.x != 0) {
        return;
    }
    const float t = __builtin_bit_cast(float, key);
    t_out[0] = key > 0x7F800000u ? mp : (t > mp ? t : mp);
}
// the select over g[0, m) (idx NULL) or over g[idx[i]] (keys: m device words for the gathered keys; idx
// may be the same buffer; in HBM or pinned host memory)
hipError_t launch_threshold(const float *g, const uint32_t *idx, uint32_t *keys, uint32_t m, uint32_t k, float *t_out,
                            hipStream_t s) {
    if (idx)
        hipLaunchKernelGGL(sp_gather_keys, dim3((m + kGatherT - 1) / kGatherT), dim3(kGatherT), 0, s, g, idx, keys, m);
    hipLaunchKernelGGL(sp_threshold, dim3(1), dim3(kThrT), 0, s, idx ? (const uint32_t *)keys : nullptr, g, m, k,
                       t_out);
    return hipGetLastError();
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

// The launches of the encoder.  nbytes_dev != NULL: the stream-ordered
// form (the buffer holds the worst case, nothing waits; sp_move stores the
// wire length there).  Otherwise blocking: the host reads the
// totals at the end (and, for a buffer below the worst case, once before the
// write pass to check the size).
// tiles per sp_image workgroup (a power of two <= kRecChunk: all in one chunk).  Round 4 measured
// 1 / 2 / 8 / 16 at 41.9 / 37.1 / 37.4 / 51.4 us per drop against 35.1 for 4.
constexpr size_t kImageTpw = 4;
static_assert(kRecChunk % kImageTpw == 0, "a workgroup's tiles share one chunk aggregate");

// ONO_DROP_FUSED=0 keeps the two launches (sp_image + sp_move): measurement, A/B
bool drop_fused() {
    static const bool v = [] {
        const char *e = getenv("ONO_DROP_FUSED");
        return !(e && !strcmp(e, "0"));
    }();
    return v;
}
// The two launches above the one-launch size: sp_count + sp_emit (default: 30.2 vs 34.0 us per 64 MiB
// drop, profiles/r05_s69_*); ONO_DROP_FORM=image: sp_image + sp_move (the round-4 form, kept for A/B)
bool drop_emit() {
    static const bool v = [] {
        const char *e = getenv("ONO_DROP_FORM");
        return !(e && !strcmp(e, "image"));
    }();
    return v;
}
// sp_count's grid: ONO_COUNT_WGS workgroups per CU (default 4), at most one per kCountTpw tiles
size_t count_grid(size_t ntiles) {
    static const size_t per = [] {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        const char *e = getenv("ONO_COUNT_WGS");
        const size_t w = e && *e ? (size_t)strtoul(e, nullptr, 10) : 4;
        return (size_t)cus * (w ? w : 1);
    }();
    return std::max<size_t>(1, std::min(per, (ntiles + kCountTpw - 1) / kCountTpw));
}
// ONO_EMIT_STAGE=0: sp_emit stores every unit straight to the wire (default: through an LDS stage)
bool emit_stage() {
    static const bool v = [] {
        const char *e = getenv("ONO_EMIT_STAGE");
        return !(e && !strcmp(e, "0"));
    }();
    return v;
}
// ONO_DROP_FALLBACK_POLLS: sp_drop1's polls before its fallback (tests set 0: every descriptor not
// there at the first read is computed by the waiting wave)
uint32_t drop_fallback_polls() {
    static const uint32_t v = [] {
        const char *e = getenv("ONO_DROP_FALLBACK_POLLS");
        return e && *e ? (uint32_t)strtoul(e, nullptr, 10) : kDropFallbackPolls;
    }();
    return v;
}

// the largest gradient (in tiles) the one launch takes; above it the two launches (measured by
// tools/drop_sizes.py; ONO_DROP_ONE_LAUNCH_TILES overrides)
size_t drop_one_launch_tiles() {
    static const size_t v = [] {
        const char *e = getenv("ONO_DROP_ONE_LAUNCH_TILES");
        return e && *e ? (size_t)strtoull(e, nullptr, 10) : kDropOneLaunchTiles;
    }();
    return v;
}

// the error word an encoder left (host_tot[3]), cleared
int take_drop_error(Scratch *sc, const char *when) {
    volatile uint64_t *w = sc->host_tot;
    const uint64_t code = w[3];
    if (!code) return ONO_OK;
    w[3] = 0;
    return set_error(ONO_E_IO, "sparse drop%s: %s", when,
                     code == kDropErrStale ? "chunk aggregates disagree with their tile records (not zero when the "
                                             "call began); nothing was written past the buffer"
                                           : "a tile's range would pass the end of the buffer; it was not written");
}

// ONO_TCP_TRACE=1 (measurement): host time of the one-launch drop's calls — entry to the launch call, the
// launch call, the launch's return to the completion seen — printed at exit
struct DropHostTrace {
    std::atomic<uint64_t> calls{0}, pre_ns{0}, launch_ns{0}, wait_ns{0};
    ~DropHostTrace() {
        const uint64_t c = calls.load();
        if (!c || !getenv("ONO_TCP_TRACE")) return;
        fprintf(stderr, "ONO_TCP_TRACE one-launch drop, %llu calls, us each: before the launch %.2f, the launch %.2f, "
                "until complete %.2f\n", (unsigned long long)c, pre_ns.load() / 1e3 / c, launch_ns.load() / 1e3 / c,
                wait_ns.load() / 1e3 / c);
    }
};
DropHostTrace g_drop_trace;
bool drop_trace_on() {
    static const bool v = getenv("ONO_TCP_TRACE") != nullptr;
    return v;
}
inline uint64_t ns_since(std::chrono::steady_clock::time_point a) {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - a).count();
}

int drop_launch(uint8_t *buf, size_t cap, size_t *nbytes, uint64_t *nbytes_dev, const float *g, size_t n,
                float threshold, hipStream_t s, const float *t_dev = nullptr) {
    const auto t_entry = std::chrono::steady_clock::now();
    const size_t ntiles = n ? (n + kTile - 1) / kTile : 0;
    const bool vec = ((uintptr_t)g & 15u) == 0;
    const bool worst_case_fits = cap >= ono_sparse_max_bytes(n);
    // The maps and allocations of one call at a time; released before the launches: a stream's scratch is
    // its own (calls on one stream are ordered by the caller) and never freed, so launches and waits need no
    // lock — held through its spin it made every other ring's drop or lift in the process wait for this one's
    // GPU work (two TCP workers of one process, config 1: ~11 us of each drop call before its launch, r06_s31)
    std::unique_lock<std::mutex> lk(g_scratch_mu);
    Scratch *sc = nullptr;
    hipStreamCaptureStatus cap_st = hipStreamCaptureStatusNone;
    const bool capturing = hipStreamIsCapturing(s, &cap_st) == hipSuccess && cap_st != hipStreamCaptureStatusNone;
    if (capturing) {
        // Captured: the stream-ordered two launches (count + emit), whose only state between calls is on
        // the device (the aggregate parity), over arrays an earlier uncaptured call on this stream made.
        // Not the one launch (a replay would repeat its epoch), not a blocking call (it waits for its
        // result), no allocation or memset (r05: a captured form with memset nodes faulted on replay).
        if (!nbytes_dev) return set_error(ONO_E_ARG, "the blocking sparse drop cannot be captured (use the stream-ordered one)");
        if (!drop_emit()) return set_error(ONO_E_ARG, "the image-form drop (ONO_DROP_FORM=image) cannot be captured");
        if (ntiles == 0) {  // the total alone (sp_drop1's empty case reads no descriptor and no scratch)
            hipLaunchKernelGGL(sp_drop1, dim3(1), dim3(kIT), 0, s, g, n, (size_t)0, threshold, t_dev, vec,
                               (uint64_t *)nullptr, 0u, 0u, buf, cap, (uint64_t *)nullptr, nbytes_dev,
                               (uint64_t *)nullptr, (uint64_t)0, 0u);
            ONO_HIP(hipGetLastError());
            return ONO_OK;
        }
        sc = scratch_ready(ntiles, s);
        if (!sc)
            return set_error(ONO_E_ARG, "sparse drop under capture: call it once on this stream outside the capture "
                                        "first (its scratch for %zu tiles is made there)", ntiles);
        sc->captured = true;
        sc->par_known = false;  // from now on replays flip the device parity behind the host's back
    }
    const bool emit = drop_emit();
    if (!capturing) {
        // the two-launch arrays whatever the form this call takes, so that a capture on this stream finds
        // them (up to 256 tiles ~1.1 MB)
        int rc = scratch_for(ntiles, s, &sc, true, emit);
        if (rc) return rc;
        if ((rc = take_drop_error(sc, " (an earlier call on this stream)"))) return rc;
        if (sc->dirty) {  // an earlier sp_count without its sp_emit: both arrays and the parity from zero
            ONO_HIP(hipMemsetAsync(sc->agg, 0, sc->agg_cap * kAggStride * sizeof(uint4), s));
            ONO_HIP(hipMemsetAsync(sc->state, 0, 16 * sizeof(uint32_t), s));
            sc->dirty = false;
            sc->parity = 0;
            if (!sc->captured) {  // (a graph's replays still flip the device parity)
                sc->par_known = true;
                sc->hpar = 0;
            }
        }
    }
    // the one-launch form when the buffer holds the worst case (it writes as it goes) and the stream is
    // not being captured (a replayed graph would repeat the epoch: the last replay's descriptors would
    // read as this one's)
    if (!capturing && drop_fused() && worst_case_fits && ntiles <= drop_one_launch_tiles()) {
        int rc = scratch_for(ntiles, s, &sc, false);
        if (rc) return rc;
        if (++sc->depoch == 0 || sc->depoch >= 0x7FFFFFFFu) {  // tags 2 e, 2 e + 1 stay nonzero and distinct
            ONO_HIP(hipMemsetAsync(sc->desc, 0, 4 * sc->desc_cap * sizeof(uint64_t), s));
            sc->depoch = 1;
        }
        const uint32_t grid = (uint32_t)std::max<size_t>(ntiles, 1);
        // blocking: the kernel signals its own completion (drop1_complete) — no signal launch, no stream wait
        uint32_t sig = 0;
        uint64_t target = 0;
        const bool in_kernel = drop1_signal_in_kernel();
        if (!nbytes_dev && in_kernel) {
            if (++sc->calls == 0) sc->calls = 1;
            sig = sc->calls;
            target = sc->arrive_base + grid - 1;
            *(volatile uint64_t *)(sc->host_tot + 2) = 0;
        }
        lk.unlock();  // (the launch and the wait use this stream's scratch only)
        const bool tr = drop_trace_on();
        const auto t_pre = std::chrono::steady_clock::now();
        hipLaunchKernelGGL(sp_drop1, dim3(grid), dim3(kIT), 0, s, g, n, ntiles, threshold, t_dev, vec, sc->desc,
                           sc->depoch, drop_fallback_polls(), buf, cap, sc->host_tot_dev, nbytes_dev, sc->arrive,
                           target, sig);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return hip_error(e, "sparse drop", __FILE__, __LINE__);
        if (nbytes_dev) return ONO_OK;
        const auto t_launched = std::chrono::steady_clock::now();
        volatile uint64_t *tot = sc->host_tot;
        if (in_kernel) {
            sc->arrive_base += grid;
            e = host_spin(s, sc->host_tot + 2, sig);
        } else {
            if (++sc->calls == 0) sc->calls = 1;
            e = host_wait(s, sc->host_tot + 2, sc->host_tot_dev + 2, sc->calls);
        }
        if (tr) {
            g_drop_trace.calls++;
            g_drop_trace.pre_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t_pre - t_entry).count();
            g_drop_trace.launch_ns +=
                (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t_launched - t_pre).count();
            g_drop_trace.wait_ns += ns_since(t_launched);
        }
        if (e != hipSuccess) return hip_error(e, "sparse drop", __FILE__, __LINE__);
        if ((rc = take_drop_error(sc, ""))) return rc;
        *nbytes = 8 + 8 * (size_t)tot[1] + 2 * (size_t)tot[0];
        return ONO_OK;
    }
    lk.unlock();  // (from here on the call uses this stream's scratch only)
    uint2 *recA = sc->rec, *recB = sc->rec + sc->tiles_cap;
    const size_t nchunks = (ntiles + kRecChunk - 1) / kRecChunk;
    const size_t half = kAggHalf;  // (the second array, within each chunk's line)
    // the image form keeps its parity on the host (it is never captured); count + emit on the device
    uint4 *agg = sc->agg + sc->parity * half;
    uint4 *agg_next = sc->agg + (1 - sc->parity) * half;
    volatile uint64_t *tot = sc->host_tot;  // pinned, written by the device
    if (!nbytes_dev) tot[0] = tot[1] = 0;
    hipError_t e = hipSuccess;
    if (ntiles && emit) {
        hipLaunchKernelGGL(sp_count, dim3((unsigned)count_grid(ntiles)), dim3(kSB), 0, s, g, n, ntiles, threshold, t_dev, vec,
                           sc->mask, sc->cv, recA, sc->agg, (uint32_t)sc->agg_cap, sc->state);
        e = hipGetLastError();
        if (e == hipSuccess) sc->dirty = true;  // until its sp_emit is launched
    } else if (ntiles) {
        const size_t grid = (ntiles + kImageTpw - 1) / kImageTpw;
        hipLaunchKernelGGL(sp_image, dim3((unsigned)grid), dim3(kIT), 0, s, g, n, ntiles, (uint32_t)kImageTpw, threshold,
                           t_dev, vec, sc->img, recA, recB, agg, agg_next, (uint32_t)sc->agg_cap);
        e = hipGetLastError();
        if (e == hipSuccess) sc->parity ^= 1;  // agg_next is zeroed for the next call
    }
    if (e == hipSuccess && !worst_case_fits) {  // the exact size first (one extra host round trip; never captured)
        hipLaunchKernelGGL(sp_totals_out, dim3(1), dim3(64), 0, s, emit ? sc->agg : agg, half,
                           emit ? (const uint32_t *)sc->state : nullptr, (uint32_t)nchunks, sc->host_tot_dev);
        e = hipStreamSynchronize(s);
        // (count + emit: no sp_emit follows, so the call stays `dirty` and the next one re-zeroes)
        if (e == hipSuccess && 8 + 8 * tot[1] + 2 * tot[0] > cap)
            return set_error(ONO_E_SIZE, "sparse encoding needs %zu bytes, buffer holds %zu",
                             (size_t)(8 + 8 * tot[1] + 2 * tot[0]), cap);
    }
    if (e != hipSuccess) return hip_error(e, "sparse encode", __FILE__, __LINE__);
    const size_t mblocks = std::max<size_t>(1, (ntiles + kSB / 64 - 1) / (kSB / 64));
#ifdef ONO_EXP_COUNT
    if (emit) return 0;  // measurement builds: sp_count alone
#endif
    const bool dp = !sc->par_known;
    const uint32_t hp = sc->hpar;
    if (emit) {
        auto k = emit_stage() ? (dp ? sp_emit<true, true> : sp_emit<true, false>)
                              : (dp ? sp_emit<false, true> : sp_emit<false, false>);
        hipLaunchKernelGGL(k, dim3((unsigned)mblocks), dim3(kSB), 0, s, sc->cv, n, ntiles, sc->mask, recA, sc->agg,
                           sc->state, hp, buf, cap, sc->host_tot_dev, nbytes_dev);
    }
    else
        hipLaunchKernelGGL(sp_move, dim3((unsigned)mblocks), dim3(kSB), 0, s, sc->img, recA, recB, agg, ntiles, n, buf,
                           cap, sc->host_tot_dev, nbytes_dev);
    e = hipGetLastError();
    if (e != hipSuccess) return hip_error(e, "sparse write", __FILE__, __LINE__);
    if (emit) {
        sc->dirty = false;
        sc->hpar ^= 1u;  // (sp_emit flipped state[0])
    }
    if (nbytes_dev) return ONO_OK;
    if (++sc->calls == 0) sc->calls = 1;
    e = host_wait(s, sc->host_tot + 2, sc->host_tot_dev + 2, sc->calls);
    if (e != hipSuccess) return hip_error(e, "sparse write", __FILE__, __LINE__);
    int rc = take_drop_error(sc, "");
    if (rc) return rc;
    *nbytes = 8 + 8 * (size_t)tot[1] + 2 * (size_t)tot[0];
    return ONO_OK;
}

// Test hook (ono_sparse_drop_debug_stale): adds `add` to the kept values and runs of every chunk aggregate
// in the array the stream's next sp_count adds into — an aggregate that was not zero when the call began,
// the hazard the writers' bounds and sp_emit's record check exist for.
__global__ void sp_poison(uint4 *agg2, size_t half, const uint32_t *state, uint32_t G, uint32_t add) {
    uint4 *agg = agg2 + (size_t)(state[0] & 1u) * half;
    for (uint32_t j = threadIdx.x; j < G; j += blockDim.x) {
        uint4 a = agg[(size_t)j * kAggStride];
        a.x += add;
        a.y += add;
        agg[(size_t)j * kAggStride] = a;
    }
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

int ono_sparse_drop_check(void *stream) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    ONO_HIP(hipStreamSynchronize(s));
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    int dev = 0;
    ONO_HIP(hipGetDevice(&dev));
    auto it = g_scratch.find({dev, s});
    if (it == g_scratch.end() || !it->second.host_tot) return ONO_OK;
    return take_drop_error(&it->second, "");
}

int ono_sparse_drop_debug_stale(void *stream, uint32_t add) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    int dev = 0;
    ONO_HIP(hipGetDevice(&dev));
    auto it = g_scratch.find({dev, s});
    if (it == g_scratch.end() || !it->second.state)
        return set_error(ONO_E_ARG, "no count + emit drop has run on this stream");
    Scratch &sc = it->second;
    hipLaunchKernelGGL(sp_poison, dim3(1), dim3(256), 0, s, sc.agg, (size_t)kAggHalf, (const uint32_t *)sc.state,
                       (uint32_t)sc.agg_cap, add);
    ONO_HIP(hipGetLastError());
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


}  // extern "C"

namespace ono {

// (sample.len() as f32 * (1.0 - r)) as usize, clamped to the last index (protocol.rs:33-49)
static size_t threshold_rank(size_t m, float r) {
    const float kf = (float)m * (1.0f - r);
    size_t k = kf <= 0.0f ? 0 : (size_t)kf;
    return k > m - 1 ? m - 1 : k;
}

// The TCP ring's push in stream order (ono_tcp.cpp): the threshold into t_dev, the drop and the masks
// reading it there — no host round trip between them.  idx_dev: the m sample indices in device memory
// (the caller checked them against n), or NULL for the whole chunk (m == n <= 16384).
hipError_t stream_wait(hipStream_t s, uint64_t *word_host, uint64_t *word_dev, uint32_t epoch) {
    return host_wait(s, word_host, word_dev, epoch);
}
hipError_t stream_spin(hipStream_t s, uint64_t *word_host, uint32_t epoch) { return host_spin(s, word_host, epoch); }

int sparse_threshold_dev(float *t_dev, const float *g, size_t n, const uint32_t *idx, uint32_t *keys, size_t m, float r,
                         hipStream_t s) {
    if (!(r > 0.0f && r <= 1.0f)) return set_error(ONO_E_ARG, "ratio %g outside (0, 1]", (double)r);
    if (m == 0 || m > kSampleMax || (!idx && m != n))
        return set_error(ONO_E_ARG, "sample of %zu values from %zu", m, n);
    ONO_HIP(launch_threshold(g, idx, keys, (uint32_t)m, (uint32_t)threshold_rank(m, r), t_dev, s));
    return ONO_OK;
}
int sparse_drop_tdev(uint8_t *buf, size_t cap, size_t *nbytes, const float *g, size_t n, const float *t_dev,
                     hipStream_t s) {
    int rc = drop_args(g, n, buf, cap);
    if (rc) return rc;
    return drop_launch(buf, cap, nbytes, nullptr, g, n, 0.0f, s, t_dev);
}
hipError_t launch_hop_post(float *dst, const float *src, size_t k, int add, float *mg, size_t mn, const float *t_dev,
                           int zero_kept, hipStream_t s, size_t L, const uint32_t *idx, const uint32_t *offs,
                           uint32_t *keys) {
    const size_t b1 = ((keys ? L : k) + kSB - 1) / kSB, b2 = (mn + kSB - 1) / kSB;
    if (b1 + b2 == 0) return hipSuccess;
    hipLaunchKernelGGL(sp_hop_post, dim3((unsigned)(b1 + b2)), dim3(kSB), 0, s, dst, src, k, add, mg, mn, t_dev,
                       zero_kept, (uint32_t)b1, idx, offs, keys);
    return hipGetLastError();
}
// the select alone over m keys already gathered (sp_hop_post gathered them)
int sparse_select_keys_dev(float *t_dev, const uint32_t *keys, size_t m, float r, hipStream_t s) {
    if (!(r > 0.0f && r <= 1.0f)) return set_error(ONO_E_ARG, "ratio %g outside (0, 1]", (double)r);
    if (m == 0 || m > kSampleMax) return set_error(ONO_E_ARG, "sample of %zu values", m);
    hipLaunchKernelGGL(sp_threshold, dim3(1), dim3(kThrT), 0, s, keys, (const float *)nullptr, (uint32_t)m,
                       (uint32_t)threshold_rank(m, r), t_dev);
    ONO_HIP(hipGetLastError());
    return ONO_OK;
}
hipError_t launch_sparse_mask_tdev(float *g, size_t n, const float *t_dev, int zero_kept, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(sp_mask, dim3((unsigned)((n + kSB - 1) / kSB)), dim3(kSB), 0, s, g, n, 0.0f, t_dev, zero_kept);
    return hipGetLastError();
}

}  // namespace ono

extern "C" {

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
    const size_t k = threshold_rank(m, r);
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
    ONO_HIP(launch_threshold(g, idx_host ? T.idx : nullptr, T.idx, (uint32_t)m, (uint32_t)k, T.t_dev, s));
    ONO_HIP(hipGetLastError());
    ONO_HIP(hipStreamSynchronize(s));
    *t_out = *(volatile float *)T.t_host;
    return ONO_OK;
}

}  // extern "C"
namespace {
// the stream-ordered lift in one launch (pl_fused) up to kPatDirect tiles; ONO_LIFT_FUSED=0 keeps the
// pl_index + pl_place launches (measurement), =2 takes the one launch even under stream capture (a
// diagnostic: shows what the capture guard prevents)
int lift_fused_mode() {
    static const int v = [] {
        const char *e = getenv("ONO_LIFT_FUSED");
        return e ? atoi(e) : 1;
    }();
    return v;
}
bool lift_fused() { return lift_fused_mode() != 0; }
// one tile per workgroup up to this many tiles (and the device's slots), three above (measurement builds
// move the switch)
#ifndef ONO_FUSED_ONE_MAX
#define ONO_FUSED_ONE_MAX 0xFFFFFFFFu
#endif
// pl_fused's workgroups co-resident on this device (one or three tiles each): occupancy x CUs, asked
// once per device.  A tile waits for tiles of higher workgroups (the earlier tiles of later stripes),
// so the grid must fit whole; a kernel of another stream that takes the slots delays it until a poll
// times out (~10 ms) and the call is refused (the caller's blocking lift then does the work).
size_t fused_slots(int tpw) {
    static std::mutex mu;
    static std::map<std::pair<int, int>, size_t> memo;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    std::lock_guard<std::mutex> lk(mu);
    auto it = memo.find({dev, tpw});
    if (it != memo.end()) return it->second;
    int per_cu = 0, cus = 0;
    const hipError_t e1 = tpw == 1 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, pl_fused<1>, kPatT, 0)
                                   : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, pl_fused<3>, kPatT, 0);
    const hipError_t e2 = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const size_t slots = e1 == hipSuccess && e2 == hipSuccess && per_cu > 0 && cus > 0 ? (size_t)per_cu * cus : 0;
    memo[{dev, tpw}] = slots;
    return slots;
}
// The one-launch lifts of different streams must not hold slots the others wait for: a tile waits for
// tiles of higher workgroups, so grids that together overfill the device could each wait for workgroups
// that cannot start until a poll times out (~10 ms) and the calls are refused.  Each stream's last
// one-launch grid is remembered; while one stream alone uses the form nothing is recorded (an event after
// every launch measured 26.5 vs 22.7 us per lift back to back).  A stream's launch takes the one launch
// when the grids of the other streams that may still run (no event yet, or one not reached) and its own
// fit in half the device's slots together (or nothing of theirs may still run) — round 5 allowed one such
// lift per device at a time, so two workers
// sharing a GPU (the TCP bench, the ring tests) lifted every other frame in two launches, 17-19 vs 8-9 us
// for a config-1 frame (profiles/r06_s17); ONO_LIFT_FUSED_SHARE=0 restores that rule (measurement).
bool lift_fused_share() {
    static const bool v = [] {
        const char *e = getenv("ONO_LIFT_FUSED_SHARE");
        return !(e && !strcmp(e, "0"));
    }();
    return v;
}
// ONO_LIFT_SMALL_TRACKED=1 (measurement): small one-launch grids are tracked as the large ones
bool small_lifts_untracked() {
    static const bool v = [] {
        const char *e = getenv("ONO_LIFT_SMALL_TRACKED");
        return !(e && !strcmp(e, "1"));
    }();
    return v;
}
struct FusedLast {
    hipEvent_t ev = nullptr;
    bool recorded = false;
    size_t grid = 0;
    std::chrono::steady_clock::time_point at;  // (the launch: an unrecorded one counts for 50 ms)
};
struct FusedDev {
    std::map<hipStream_t, FusedLast> last;
    bool multi = false;
};
std::map<int, FusedDev> g_fused_last;  // (under g_scratch_mu)
bool fused_device_free(int dev, hipStream_t s, size_t grid, size_t slots) {
    FusedDev &D = g_fused_last[dev];
    size_t busy = 0, others = 0;
    for (auto it = D.last.begin(); it != D.last.end();) {
        FusedLast &f = it->second;
        if (it->first == s || !f.grid) { ++it; continue; }
        others++;
        // an unrecorded launch (made while its stream was the only one) cannot be asked; after 50 ms it is taken
        // as finished — were it not, the grids would wait for each other until a poll gives up and the call is
        // refused (the blocking lift then does it): slower, never wrong
        const bool done = f.recorded ? hipEventQuery(f.ev) != hipErrorNotReady
                                     : std::chrono::steady_clock::now() - f.at > std::chrono::milliseconds(50);
        if (done) {
            f.grid = 0;
            if (D.last.size() > 64) {  // streams come and go: forget the finished ones
                (void)hipEventDestroy(f.ev);
                it = D.last.erase(it);
                continue;
            }
        } else {
            busy += f.grid;
        }
        ++it;
    }
    if (!others) return true;
    if (!D.multi) {  // a second stream: from now on every one-launch lift on the device is recorded
        D.multi = true;
        if (!lift_fused_share()) return false;
    }
    // nothing of the others may still run: the whole device (the caller checked that the grid fits it);
    // else both grids in half of it
    if (busy == 0 || !lift_fused_share()) return busy == 0;
    return busy + grid <= slots / 2;
}
void fused_device_mark(int dev, hipStream_t s, size_t grid) {
    FusedDev &D = g_fused_last[dev];
    FusedLast &f = D.last[s];
    f.grid = grid;
    f.recorded = false;
    f.at = std::chrono::steady_clock::now();
    if (!D.multi) return;
    if (!f.ev && hipEventCreateWithFlags(&f.ev, hipEventDisableTiming) != hipSuccess) {
        f.ev = nullptr;
        return;
    }
    f.recorded = hipEventRecord(f.ev, s) == hipSuccess;
}
}  // namespace
extern "C" {

int ono_sparse_lift_dev_async(float *g, size_t cap, const uint8_t *buf_dev, size_t nbytes, uint64_t *status,
                              uint64_t *ticket, void *stream) {
    return ono::lift_dev_async(g, cap, buf_dev, nbytes, status, ticket, reinterpret_cast<hipStream_t>(stream), nullptr);
}

}  // extern "C"

namespace ono {

// ono_sparse_lift_dev_async; done (the TCP ring's hop): when the lift is one launch, its last workgroup
// stores done->sig into done->word (host-mapped, zeroed here) and done->in_kernel is set — the caller spins on
// the word instead of a signal launch behind the lift
int lift_dev_async(float *g, size_t cap, const uint8_t *buf_dev, size_t nbytes, uint64_t *status, uint64_t *ticket,
                   hipStream_t s, LiftDone *done) {
    if (done) done->in_kernel = false;
    if (!status || !ticket || (!buf_dev && nbytes)) return set_error(ONO_E_ARG, "NULL argument");
    if (nbytes < 8) return set_error(ONO_E_PROTO, "The given sparse buffer is smaller than TOTAL_LEN_SIZE");
    std::unique_lock<std::mutex> lk(g_scratch_mu);  // (the maps and the device's one-launch record)
    int dev = 0;
    ONO_HIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) return set_error(ONO_E_ARG, "device %d", dev);
    PatScratch &P = g_pat[{dev, s}];
    if (!P.aw) {
        ONO_HIP(hipMalloc((void **)&P.aw, 8 * sizeof(uint64_t)));
        ONO_HIP(hipMemsetAsync(P.aw, 0, 8 * sizeof(uint64_t), s));
    }
    if (++P.epoch == 0) P.epoch = 1;
    const uint32_t epoch = P.epoch;
    *ticket = epoch;
    const size_t M = (nbytes - 8) / 2;
    // the pattern path's domain (as lift_device's); any other stream is refused at once
    if (M == 0 || (nbytes & 1) || nbytes >= 0xFFFFFFF0ull || cap >= 0xFFFFFFFFull || ((uintptr_t)buf_dev & 1)) {
        hipLaunchKernelGGL(sp_signal, dim3(1), dim3(64), 0, s, status, epoch);
        ONO_HIP(hipGetLastError());
        return ONO_OK;
    }
    const size_t T = (M + kPatU - 1) / kPatU;
    if (T > P.cap) {  // (hipFree waits for the work that still uses the old arrays)
        const size_t Tc = (T + 3) & ~(size_t)3;  // tile sums read as 16-B vectors
        (void)hipFree(P.prec);
        (void)hipFree(P.pE);
        (void)hipFree(P.pwide);
        P.prec = nullptr;
        P.pE = nullptr;
        P.pwide = nullptr;
        P.cap = 0;
        ONO_HIP(hipMalloc((void **)&P.prec, 5 * Tc * sizeof(uint32_t)));
        ONO_HIP(hipMalloc((void **)&P.pE, (Tc + 1) * sizeof(uint64_t)));
        ONO_HIP(hipMalloc((void **)&P.pwide, Tc * sizeof(uint32_t)));
        P.cap = Tc;
    }
    uint32_t *tsum = P.prec + 4 * P.cap, *qcount = (uint32_t *)(P.aw + 6);
    const int vec = ((uintptr_t)g & 15) == 0;
    // one launch (pl_fused) when every workgroup fits on the device at once: one tile each, or three
    // (an 8-B aligned stream of at most kPatDirect tiles)
    // Not under stream capture: a replayed graph repeats the epoch, and the granules of the previous
    // replay would pass for this one's (the two launches carry no such state).
    hipStreamCaptureStatus cap_st = hipStreamCaptureStatusNone;
    const bool capturing = lift_fused_mode() != 2 && hipStreamIsCapturing(s, &cap_st) == hipSuccess &&
                           cap_st != hipStreamCaptureStatusNone;
    const bool one = T <= std::min(fused_slots(1), (size_t)ONO_FUSED_ONE_MAX);
    const size_t grid = one ? T : (T + 2) / 3;
    // A small grid (at most 1/64 of the slots: a config-1 frame's 13 workgroups) is neither asked about nor
    // recorded: one stream runs its lifts one at a time, so it takes dozens of streams lifting at once to fill
    // half the device with them, and a small grid that does find the device full of a waiting one's
    // workgroups ends, like any stalled one, refused after ~100 us of standstill (the caller's blocking lift
    // then does it) — never wrong.  The event query and record cost ~3 us of host time per lift between two
    // workers of one process (r06_s32).
    const bool small = one && grid <= fused_slots(1) / 64 && small_lifts_untracked();
    if (T <= kPatDirect && ((uintptr_t)buf_dev & 7) == 0 && lift_fused() && !capturing &&
        (T + 2) / 3 <= fused_slots(3) &&
        (small || fused_device_free(dev, s, grid, one ? fused_slots(1) : fused_slots(3)))) {
        if (T > P.fcap) {
            const size_t gc = (T + kPatChunk - 1) / kPatChunk;
            (void)hipFree(P.frec);
            (void)hipFree(P.fchunk);
            P.frec = P.fchunk = nullptr;
            P.fcap = P.fgcap = 0;
            ONO_HIP(hipMalloc((void **)&P.frec, 2 * T * sizeof(uint64_t)));
            ONO_HIP(hipMemsetAsync(P.frec, 0, 2 * T * sizeof(uint64_t), s));
            ONO_HIP(hipMalloc((void **)&P.fchunk, 2 * kFusedRep * gc * kFusedLine * sizeof(uint64_t)));
            ONO_HIP(hipMemsetAsync(P.fchunk, 0, 2 * kFusedRep * gc * kFusedLine * sizeof(uint64_t), s));
            P.fcap = T;
            P.fgcap = gc;
            P.fpar = 0;
        }
        if (!P.arrive) {  // kArriveShards lines + the top word's line, 128 B each
            ONO_HIP(hipMalloc((void **)&P.arrive, (kArriveShards + 1) * 16 * sizeof(uint64_t)));
            ONO_HIP(hipMemsetAsync(P.arrive, 0, (kArriveShards + 1) * 16 * sizeof(uint64_t), s));
        }
        uint64_t *cur = P.fchunk + (size_t)P.fpar * kFusedRep * P.fgcap * kFusedLine;
        uint64_t *next = P.fchunk + (size_t)(1 - P.fpar) * kFusedRep * P.fgcap * kFusedLine;
        const uint64_t target = P.arrive_base + std::min<size_t>(grid, kArriveShards);  // complete lines
        int force = 0;
        for (uint32_t k = g_lift_force_refuse.load(); k && !force;)
            if (g_lift_force_refuse.compare_exchange_weak(k, k - 1)) force = 1;
        uint64_t *dw = nullptr, dtarget = 0;
        uint32_t dsig = 0;
        if (done && done->word_dev) {
            if (!P.done_arrive) {
                ONO_HIP(hipMalloc((void **)&P.done_arrive, 16 * sizeof(uint64_t)));
                ONO_HIP(hipMemsetAsync(P.done_arrive, 0, 16 * sizeof(uint64_t), s));
            }
            dw = done->word_dev;
            dsig = done->sig;
            dtarget = P.done_base + grid - 1;
            *(volatile uint64_t *)done->word_host = 0;
        }
        if (small) lk.unlock();  // (nothing of the device's record to update after the launch)
        if (one)
            hipLaunchKernelGGL(pl_fused<1>, dim3((unsigned)grid), dim3(kPatT), 0, s, g, buf_dev, M, T, cap, vec, P.frec,
                               cur, next, (uint32_t)P.fgcap, P.aw, status, epoch, P.arrive, target, dw, P.done_arrive,
                               dtarget, dsig, force);
        else
            hipLaunchKernelGGL(pl_fused<3>, dim3((unsigned)grid), dim3(kPatT), 0, s, g, buf_dev, M, T, cap, vec,
                               P.frec, cur, next, (uint32_t)P.fgcap, P.aw, status, epoch, P.arrive, target, dw,
                               P.done_arrive, dtarget, dsig, force);
        ONO_HIP(hipGetLastError());
        P.arrive_base = target;
        if (dw) {
            P.done_base += grid;
            done->in_kernel = true;
        }
        P.fpar ^= 1;
        if (!small) fused_device_mark(dev, s, grid);
        return ONO_OK;
    }
    lk.unlock();  // (the two launches use this stream's scratch only)
    ONO_HIP(launch_pl_index(buf_dev, M, T, P.prec, tsum, qcount, P.pwide, P.aw, status, epoch, s));
    if (T > kPatDirect)
        hipLaunchKernelGGL(pl_scan, dim3(1), dim3(kPatScanT), 0, s, buf_dev, P.prec, T, P.pE, status, epoch);
    hipLaunchKernelGGL(pl_place<true>, dim3((unsigned)T), dim3(kPatT), 0, s, g, buf_dev, M, T, cap, vec, P.pE, P.prec,
                       tsum, P.pwide, P.aw, status, epoch);
    ONO_HIP(hipGetLastError());
    return ONO_OK;
}

}  // namespace ono

extern "C" {

size_t ono_sparse_lift_fallbacks(void) { return g_lift_fallbacks.load(); }
int ono_sparse_lift_debug_refuse(uint32_t count) {
    return (int)std::min<uint32_t>(g_lift_force_refuse.exchange(count), 0x7FFFFFFFu);
}
size_t ono_sparse_lift_pattern_misses(void) { return g_lift_pattern_misses.load(); }
int ono_sparse_lift_set_mode(int mode) {
    if (mode != 0 && mode != 1) return set_error(ONO_E_ARG, "lift mode %d (0: pattern path first, 1: walk path)", mode);
    g_lift_mode.store(mode);
    return ONO_OK;
}

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
                       reinterpret_cast<hipStream_t>(stream), g, n, threshold, (const float *)nullptr, zero_kept);
    ONO_HIP(hipGetLastError());
    return ONO_OK;
}

}  // extern "C"
