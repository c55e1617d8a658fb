// ono_kernels.hip — gfx950 elementwise kernels of the gradient-bucket reduction.
//
// Every kernel here is a pure HBM stream (10-16 B of traffic
// per element against <= 10 VALU ops), so the design goal is bytes in flight,
// not arithmetic:
//   * 16-B per lane f32 accesses (global_load_dwordx4 / global_store_dwordx4),
//     8-B per lane for f16 wire buffers, one 64-lane wave = 1 KiB per f32
//     instruction, consecutive lanes on consecutive addresses;
//   * one vector per thread, one-wave workgroups, a one-shot grid: the
//     hardware keeps the bytes in flight through wave count (measured, see
//     the skeleton below and tools/stream_variants.hip);
//   * non-temporal stores for outputs, non-temporal loads for read-once inputs;
//   * misaligned chunk starts (split_chunks offsets are arbitrary) are handled
//     by a <= 3-element scalar head and tail, so the body stays vectorised
//     whenever all operands share the same 4-element phase;
//   * no LDS: no element is read twice, so staging through LDS would only add
//     instructions ("Why no LDS / MFMA").
// Numerics: -ffp-contract=off, IEEE division and sqrt (hipcc default
// -fhip-fp32-correctly-rounded-divide-sqrt), denormals preserved; f16 by
// v_cvt_f16_f32 (round-to-nearest-even) with the `half` crate's NaN rule.
#include <hip/hip_runtime.h>

#include <type_traits>
#include <utility>

#include <atomic>
#include <cstdlib>
#include <cstring>

#include "ono_device.h"
#include "ono_internal.h"

namespace ono {
namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef uint16_t h4 __attribute__((ext_vector_type(4)));

constexpr int kBlock = 64;  // one wave per workgroup: +1-4 % over 256 on every shape (tools/stream_variants.hip)

// ------------------------------------------------------------------ f16 ----
// half 2.7.1 f32_to_f16 / f16_to_f32 are v_cvt_f16_f32 (RNE, overflow -> inf,
// subnormals kept) and v_cvt_f32_f16 (exact) as they stand: the crate's NaN
// rules (f32 -> f16: sign | 0x7E00 | mantissa >> 13; f16 -> f32: sign |
// 0x7FC00000 | mantissa << 13) are exactly what gfx950's conversions produce —
// checked for all 2^16 f16 patterns and all 2^24 - 2 f32 NaN patterns
// (tools/skeleton_variants.hip "nan", profiles/r02_nan_rule.txt), and pinned by
// the exhaustive parity tests (every f32 bit pattern through the encoder, every
// f16 pattern through the decoder, tests/test_gpu_kernels.py).  Spelling the
// NaN rule out in VALU cost the decode 4 % of its HBM rate.
__device__ __forceinline__ uint16_t to_f16(float x) { return __builtin_bit_cast(uint16_t, (_Float16)x); }
__device__ __forceinline__ float from_f16(uint16_t b) { return (float)__builtin_bit_cast(_Float16, b); }

// wire traits: f16 (uint16_t) or f32 (float) messages
template <class W> struct Wire;
template <> struct Wire<uint16_t> {
    typedef h4 V;
    static __device__ __forceinline__ uint16_t enc(float x) { return to_f16(x); }
    static __device__ __forceinline__ float dec(uint16_t h) { return from_f16(h); }
    static __device__ __forceinline__ V enc4(f4 x) {
        V r;
        r.x = to_f16(x.x); r.y = to_f16(x.y); r.z = to_f16(x.z); r.w = to_f16(x.w);
        return r;
    }
    static __device__ __forceinline__ f4 dec4(V h) {
        f4 r;
        r.x = from_f16(h.x); r.y = from_f16(h.y); r.z = from_f16(h.z); r.w = from_f16(h.w);
        return r;
    }
};
template <> struct Wire<float> {
    typedef f4 V;
    static __device__ __forceinline__ float enc(float x) { return x; }
    static __device__ __forceinline__ float dec(float x) { return x; }
    static __device__ __forceinline__ V enc4(f4 x) { return x; }
    static __device__ __forceinline__ f4 dec4(V x) { return x; }
};

template <int M> __device__ __forceinline__ float scl(float x, float v) {
    if constexpr (M == SCALE_NONE) return x;
    else if constexpr (M == SCALE_RECIP) return x * v;
    else return x / v;
}
template <int M> __device__ __forceinline__ f4 scl4(f4 x, float v) {
    if constexpr (M == SCALE_NONE) return x;
    else if constexpr (M == SCALE_RECIP) return x * v;
    else return x / v;
}

template <class T> __device__ __forceinline__ T ld(const T *p) { return *p; }
// read-once inputs that this launch does not write back: non-temporal loads
// (+3-4 % on kR1W streams; a plain load is better when the same lines are
// rewritten in the launch, e.g. residual read-then-zero: tools/stream_variants.hip)
template <class T> __device__ __forceinline__ T ldn(const T *p) { return __builtin_nontemporal_load(p); }
template <class T> __device__ __forceinline__ void st(T *p, T v) { *p = v; }
// write-once outputs that nobody re-reads in this launch: non-temporal
template <class T> __device__ __forceinline__ void st_nt(T *p, T v) { __builtin_nontemporal_store(v, p); }
// Outputs of the ops that consume the residual (read it, zero it, pass the
// result on): streaming stores at agent scope, `global_store … nt sc1` (the
// builtin above gives `nt` alone), after nt loads.  Producers that accumulate
// into a buffer the next kernel reads (acc_residual, the store's f16
// accumulate) keep plain loads + `nt` stores: those leave the residual in the
// Infinity Cache for the pull, which the consumer policy would forfeit
// (tools/stream_variants.hip mode t: acc + pull on one reused bucket, 224.8 us
// per step with this split vs 253-257 us with the consumer policy everywhere).
// The pull shape (1R2W) back to back over fresh 256 MiB buffers (mode c):
// 125-129 us with plain loads + `nt` stores, 119-121 us with nt loads +
// `nt sc1`; on one reused bucket after acc_residual (mode t) 103.7 -> 100 us.
// On the kR1W / 1R1W ops and the optimizer it measured worse, so those keep
// st_nt.  Vector stores only (no scalar-cache writes).  The
// compiler's hazard recognizer cannot see into the asm, so it carries the gfx9
// store-data hazard itself: no VALU may overwrite the data VGPRs of a > 8-byte
// store for 2 wait states on gfx940+ (`s_nop 1`).  vmcnt waits the compiler
// emits for its own loads only grow stricter with these stores outstanding;
// the "memory" clobber keeps them after every load of the op (ops load first).
template <class T> __device__ __forceinline__ void st_sc1(T *p, T v) { __builtin_nontemporal_store(v, p); }
__device__ __forceinline__ void st_sc1(f4 *p, f4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" : : "v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st_sc1(h4 *p, h4 v) {
    asm volatile("global_store_dwordx2 %0, %1, off nt sc1" : : "v"(p), "v"(__builtin_bit_cast(uint64_t, v))
                 : "memory");
}

// --------------------------------------------------------- stream skeleton
// Element range [0, n) split as [0, head) scalar | [head, head+4*nvec) 4-wide | tail scalar.
// One 16-B vector per thread over a one-shot grid (ceil(nvec/64) one-wave workgroups):
// measured on MI355X with rotating > 1.5 GiB working sets (tools/stream_variants.hip),
// this beats grid-stride loops with 2-4 vectors in flight per thread by 8-40 %
// for every 1R2W / kR1W shape of this path; the hardware keeps enough bytes in
// flight through wave count, not per-thread unrolling.  The grid-stride form
// is kept for grids beyond the launch limit.
// Ops whose stores other processes / devices read next (after a flag barrier
// in a later launch) end every wave with op.finish(): see peer_stores_done().
template <class Op, class = void> struct HasFinish : std::false_type {};
template <class Op> struct HasFinish<Op, std::void_t<decltype(std::declval<const Op &>().finish())>> : std::true_type {};
template <class Op> __device__ __forceinline__ void finish_wave(const Op &op) {
    if constexpr (HasFinish<Op>::value) op.finish();
}
// Ops that cap how many of their one-wave workgroups share a CU say so with
// occ() (0 = no cap); the launch then reserves enough dynamic LDS per
// workgroup (unused; 160 KiB per CU) that no more than occ() fit.  Applied to
// buckets of at least kOccElems; ONO_EW_OCC=<cap> overrides every op's cap
// (32 = none) for measurement (tools/occ_sweep.sh).
template <class Op, class = void> struct HasOcc : std::false_type {};
template <class Op> struct HasOcc<Op, std::void_t<decltype(std::declval<const Op &>().occ())>> : std::true_type {};
constexpr size_t kOccElems = size_t(4) << 20;
inline unsigned lds_for_occ(int occ) {
    return occ <= 0 || occ >= 32 ? 0u : (unsigned)(160u * 1024u * 2u / (2u * (unsigned)occ + 1u));
}
int occ_override() {
    static int v = [] {
        const char *e = getenv("ONO_EW_OCC");
        int x = e ? atoi(e) : 0;
        return x > 0 ? x : 0;
    }();
    return v;
}
template <class Op> unsigned ew_lds(const Op &op, size_t n) {
    if (const int o = occ_override()) return lds_for_occ(o);
    if constexpr (HasOcc<Op>::value) return n >= kOccElems ? lds_for_occ(op.occ()) : 0u;
    return 0u;
}

// The write-only fill uses 256-thread workgroups instead (block() = 256): a
// one-shot grid of one-wave workgroups is bounded by the dispatcher's workgroup
// rate — an empty kernel over the 65,536 one-wave workgroups of a 64 MiB bucket
// takes 14.9 us — and a 64 MiB fill then runs at 0.52 of 8 TB/s against 0.81
// with 256-thread workgroups (tools/launch_phases.hip,
// profiles/r04_launch_phases_s3.txt, tools/pk_ab.py).  Every other shape moves
// enough bytes per workgroup that 64 threads stay best (+1-4 %; the f16 decode
// too, on the bench's data).  ONO_EW_WIDE=0 runs the fill on 64 threads (A/B).
template <class Op, class = void> struct HasBlock : std::false_type {};
template <class Op> struct HasBlock<Op, std::void_t<decltype(Op::block())>> : std::true_type {};
template <class Op> constexpr int block_of() {
    if constexpr (HasBlock<Op>::value) return Op::block();
    else return kBlock;
}
// ONO_EW_WIDE=0: the 256-thread ops run with 64-thread workgroups too (measurement A/B)
bool wide_blocks() {
    static const bool v = [] {
        const char *e = getenv("ONO_EW_WIDE");
        return !(e && !strcmp(e, "0"));
    }();
    return v;
}

// LOOP = false: the grid covers every vector (the one-shot grid), so no loop
// at all — one guarded vector per lane (dec 2.5 %, sum8 1 % faster than the
// loop form, tools/skeleton_variants.hip; profiles/r02_skeleton_variants.txt).
template <class Op, bool LOOP, int B = block_of<Op>()>
__global__ __launch_bounds__(B) void ew_kernel(Op op, size_t head, size_t nvec, size_t n) {
    const size_t tid = (size_t)blockIdx.x * B + threadIdx.x;
    const size_t tail0 = head + 4 * nvec;
    if (tid < head) op.scalar(tid);
    if (tid < n - tail0) op.scalar(tail0 + tid);
    if constexpr (LOOP) {
        const size_t stride = (size_t)gridDim.x * B;
        for (size_t v = tid; v < nvec; v += stride) op.store(head + 4 * v, op.load(head + 4 * v));
    } else {
        if (tid < nvec) op.store(head + 4 * tid, op.load(head + 4 * tid));
    }
    finish_wave(op);
}

// scalar-only fallback for operands whose 4-element phases differ
template <class Op, int B = block_of<Op>()>
__global__ __launch_bounds__(B) void ew_scalar_kernel(Op op, size_t n) {
    const size_t stride = (size_t)gridDim.x * B;
    for (size_t i = (size_t)blockIdx.x * B + threadIdx.x; i < n; i += stride) op.scalar(i);
    finish_wave(op);
}

// ---------------------------------------------------------------- grid ----
struct DevInfo {
    int cus = 0;
};
DevInfo g_dev[64];

// Grid cap in workgroups per CU (0 = one-shot grid, the measured optimum);
// ONO_EW_BLOCKS_PER_CU overrides it for experiments.
int blocks_per_cu() {
    static int v = [] {
        const char *e = getenv("ONO_EW_BLOCKS_PER_CU");
        int x = e ? atoi(e) : 0;
        return x > 0 ? x : 0;
    }();
    return v;
}

int device_cus() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (g_dev[dev].cus == 0) {
        int c = 0;
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0)
            c = 256;
        g_dev[dev].cus = c;
    }
    return g_dev[dev].cus;
}

inline unsigned phase_of(const void *p, size_t esz) {
    return (unsigned)(((uintptr_t)p / esz) & 3u);
}

// An op whose kernel tells the host it is done (the TCP ring's dense hop, whose frame the op writes into
// pinned memory): each wave waits for its stores, lane 0 releases at system scope (the frame can sit dirty in
// its XCD's L2, as sp_drop1's) and counts the wave in; the last wave of the launch stores `sig` into the
// host-mapped word the host spins on — instead of a stream synchronisation's wake-up after the kernel.
template <class Op> struct Signaled : Op {
    uint64_t *word, *arrive;
    uint64_t target;
    uint32_t sig;
    __device__ __forceinline__ void finish() const {
        if constexpr (HasFinish<Op>::value) Op::finish();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if ((threadIdx.x & 63) == 0) {
            __atomic_thread_fence(__ATOMIC_RELEASE);
            const uint64_t old = __hip_atomic_fetch_add(arrive, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (old == target) __hip_atomic_store(word, (uint64_t)sig, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
};

// Launch `op` over n elements.  phases: the 4-element phase of every operand.
template <class Op, int B = block_of<Op>()>
hipError_t launch_ew_arr(const Op &op, size_t n, const unsigned *phases, int nph, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if constexpr (B != kBlock) {
        if (!wide_blocks()) return launch_ew_arr<Op, kBlock>(op, n, phases, nph, s);
    }
    unsigned ph = phases[0];
    bool same = true;
    for (int i = 0; i < nph; i++) same &= (phases[i] == ph);
    const int bpc = blocks_per_cu();
    const size_t cap = bpc > 0 ? (size_t)device_cus() * (size_t)bpc * kBlock / B : (size_t)0x7FFFFFFF;
    const unsigned lds = ew_lds(op, n);
    if (!same) {
        size_t blocks = (n + B - 1) / B;
        if (blocks > cap) blocks = cap;
        hipLaunchKernelGGL((ew_scalar_kernel<Op, B>), dim3((unsigned)blocks), dim3(B), lds, s, op, n);
        return hipGetLastError();
    }
    size_t head = (4 - ph) & 3u;
    if (head > n) head = n;
    size_t nvec = (n - head) / 4;
    size_t work = nvec > 4 ? nvec : 4; // threads needed (>= head/tail lanes)
    size_t blocks = (work + B - 1) / B;
    if (blocks < 1) blocks = 1;
    if (blocks > cap) {
        hipLaunchKernelGGL((ew_kernel<Op, true, B>), dim3((unsigned)cap), dim3(B), lds, s, op, head, nvec, n);
        return hipGetLastError();
    }
    hipLaunchKernelGGL((ew_kernel<Op, false, B>), dim3((unsigned)blocks), dim3(B), lds, s, op, head, nvec, n);
    return hipGetLastError();
}

template <class Op>
hipError_t launch_ew(const Op &op, size_t n, std::initializer_list<unsigned> phases, hipStream_t s) {
    return launch_ew_arr(op, n, phases.begin(), (int)phases.size(), s);
}
// launch_ew whose launch signals its end (Signaled over the same grid as launch_ew_arr's; done->base counts
// the waves launched so far on its counter); done NULL: launch_ew
template <class Op>
hipError_t launch_ew(const Op &op, size_t n, std::initializer_list<unsigned> phases, hipStream_t s, KernelDone *done) {
    if (!done || n == 0) return launch_ew(op, n, phases, s);
    constexpr int B0 = block_of<Op>();
    const int B = (B0 != kBlock && !wide_blocks()) ? kBlock : B0;
    const unsigned *ph = phases.begin();
    const int nph = (int)phases.size();
    bool same = true;
    for (int i = 0; i < nph; i++) same &= (ph[i] == ph[0]);
    const int bpc = blocks_per_cu();
    const size_t cap = bpc > 0 ? (size_t)device_cus() * (size_t)bpc * kBlock / B : (size_t)0x7FFFFFFF;
    size_t blocks;
    if (!same) {
        blocks = std::min((n + B - 1) / B, cap);
    } else {
        size_t head = (4 - ph[0]) & 3u;
        if (head > n) head = n;
        const size_t nvec = (n - head) / 4, work = nvec > 4 ? nvec : 4;
        blocks = std::min(std::max<size_t>((work + B - 1) / B, 1), cap);
    }
    const uint64_t waves = (uint64_t)blocks * (uint64_t)(B / 64);
    Signaled<Op> so;
    static_cast<Op &>(so) = op;
    so.word = done->word_dev;
    so.arrive = done->arrive;
    so.sig = done->sig;
    so.target = done->base + waves - 1;
    done->base += waves;
    return launch_ew_arr(so, n, ph, nph, s);
}

// ============================================================== ops =======
// sum-and-scale over K inputs (K compile-time), left fold in input order.
// Read-once inputs (NTL) at the 64 MiB bucket of BASELINE config 2, measured
// in round 3 (tools/sum_variants.hip, profiles/r03_sum_variants.txt; same box,
// medians of 3-5 passes):
//   K >= 4: ONE load in flight per wave (each input's vector requested once
//           the previous one has returned) and at most 28 of these one-wave
//           workgroups per CU (5.6 KiB of dynamic LDS each, unused): K = 8
//           99.9 -> 91.7 us (0.756 -> 0.823 of 8 TB/s), K = 4 55.9 -> 52.9 us
//           (0.750 -> 0.794).  All K loads issued at once — what the compiler
//           does by itself — is the slowest form; two or three in flight
//           measured like all of them; the cap alone (26-30 per CU) adds 1-2 %
//           to one load in flight, and costs every other shape.  (Found through
//           a load-order rotation that happened to serialize its loads through
//           one register set.)
//   K == 2: the two inputs land in LDS by LDS-DMA (global_load_lds_dwordx4
//           nt, no VGPR round trip) and are added from there: 32.3 -> 32.0 us
//           (0.778 -> 0.787); one load in flight measured no different there.
struct Ptrs {
    const float *p[ONO_MAX_INPUTS];
};
// SER: the serialized form (K >= 4, buckets of at least kSerialElems, where
// bandwidth, not one wave's latency, decides; smaller buckets keep every load
// in flight).
constexpr size_t kSerialElems = kOccElems;
template <int K, int M, bool NTL, bool SER = false> struct SumScaleOp {
    __host__ int occ() const { return SER ? 28 : 0; }  // one-wave workgroups per CU
    Ptrs in;
    float *out;
    float v;
    typedef f4 R;
    __device__ __forceinline__ void scalar(size_t i) const {
        float a = in.p[0][i];
#pragma unroll
        for (int j = 1; j < K; j++) a += in.p[j][i];
        out[i] = scl<M>(a, v);
    }
    __device__ __forceinline__ f4 get(int j, size_t i) const {
        if constexpr (NTL) return ldn((const f4 *)(in.p[j] + i));
        else return ld((const f4 *)(in.p[j] + i));
    }
    __device__ __forceinline__ R load(size_t i) const {
        if constexpr (NTL && K == 2) {
            __shared__ f4 lds[2][kBlock];  // lane l's 16 B of input j land at lds[j][l]
#pragma unroll
            for (int j = 0; j < 2; j++)
                __builtin_amdgcn_global_load_lds((const void *)(in.p[j] + i),
                                                 (__attribute__((address_space(3))) void *)&lds[j][0], 16, 0, 2);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            return lds[0][threadIdx.x] + lds[1][threadIdx.x];
        } else if constexpr (SER) {
            static_assert(NTL && K >= 4, "the serialized form reads K >= 4 read-once inputs");
            // one load in flight per wave: each input's vector is requested
            // once the previous one has returned (fold in input order)
            f4 a = get(0, i);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
            for (int j = 1; j < K; j++) {
                const f4 x = get(j, i);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                a += x;
            }
            return a;
        } else {
            f4 a = get(0, i);
#pragma unroll
            for (int j = 1; j < K; j++) a += get(j, i);
            return a;
        }
    }
    __device__ __forceinline__ void store(size_t i, R a) const { st_nt((f4 *)(out + i), scl4<M>(a, v)); }
};

// The chunk owner's reduction in the direct (all-to-all) schedule.  in[k] is
// rank (c+k)'s slice of chunk c, k = 0..K-1, the owner's own residual last.
//   p = in[0];  p = in[k] + wire(p) for k = 1..K-1
// reproduces the reference's hop chain (worker_ring.rs:122-143: each hop adds
// the received wire value into the local f32 chunk), wire() being the f16
// round trip (f16 wire) or the identity (f32 wire).  Then grad = p / d (:166 +
// :101-105), out = enc(p) for the all-gather (f16 wire; f32 wire: a copy of
// grad when out is set — the xGMI schedule's exchange buffer), and the slices
// that were "sent" are zeroed (:133, :191-193): the own one, or all of them
// when every rank is co-resident (zall).  Scale mode and zall are uniform
// run-time flags (uniform branches, no divergence).
struct Outs {
    void *p[ONO_MAX_INPUTS];
};
// ZALL is a template parameter (the load policy of every slice is decided at
// compile time; a plain load where an nt load belongs cost the owner chain at
// n = 8 about 20 %: profiles/r02_opt_variants.txt, "chain8 L0" vs "L1").
template <int K, class W, bool ZALL> struct DirectOp {
    typedef typename Wire<W>::V WV;
    // outs read by other ranks after the next flag barrier: every wave waits
    // for its stores to complete at system scope before it ends
    __device__ __forceinline__ void finish() const {
        if (sys_out) peer_stores_done();
    }
    Ptrs in;
    float *grad;
    Outs out;  // nout copies of the result (f16 message / f32 grad value): local and/or peer HBM
    int nout;
    int sys_out;  // outs are peer HBM: system-coherent (sc0 sc1) stores, see ono_device.h
    float v;
    int mode;  // SCALE_RECIP or SCALE_DIV
    typedef f4 R;
    __device__ __forceinline__ float wq(float p) const { return Wire<W>::dec(Wire<W>::enc(p)); }
    __device__ __forceinline__ f4 wq4(f4 p) const { return Wire<W>::dec4(Wire<W>::enc4(p)); }
    __device__ __forceinline__ void scalar(size_t i) const {
        float p = in.p[0][i];
#pragma unroll
        for (int k = 1; k < K; k++) p = in.p[k][i] + wq(p);
        const float gv = mode == SCALE_RECIP ? p * v : p / v;
        grad[i] = gv;
        const W m = sizeof(W) == 2 ? Wire<W>::enc(p) : Wire<W>::enc(gv);
        for (int j = 0; j < nout; j++) {
            if (sys_out) st_sys(static_cast<W *>(out.p[j]) + i, m);
            else static_cast<W *>(out.p[j])[i] = m;
        }
        if constexpr (ZALL) {
#pragma unroll
            for (int k = 0; k < K; k++) const_cast<float *>(in.p[k])[i] = 0.0f;
        } else {
            const_cast<float *>(in.p[K - 1])[i] = 0.0f;
        }
    }
    // Received slices are read once (nt loads); slices zeroed in this pass
    // (the own one, or all with ZALL) take plain loads.  The two forms are
    // separate straight-line loops: a `k < K - 1 ? ldn : ld` inside one loop
    // was merged by the compiler into a single plain load before unrolling.
    __device__ __forceinline__ R load(size_t i) const {
        f4 x[K];
        if constexpr (ZALL) {
#pragma unroll
            for (int k = 0; k < K; k++) x[k] = ld((const f4 *)(in.p[k] + i));
        } else {
#pragma unroll
            for (int k = 0; k < K - 1; k++) x[k] = ldn((const f4 *)(in.p[k] + i));
            x[K - 1] = ld((const f4 *)(in.p[K - 1] + i));
        }
        f4 p = x[0];
#pragma unroll
        for (int k = 1; k < K; k++) p = x[k] + wq4(p);
        return p;
    }
    __device__ __forceinline__ void store(size_t i, R p) const {
        const f4 gv = mode == SCALE_RECIP ? p * v : p / v;
        st_nt((f4 *)(grad + i), gv);
        const WV m = sizeof(W) == 2 ? Wire<W>::enc4(p) : Wire<W>::enc4(gv);
        for (int j = 0; j < nout; j++) {
            if (sys_out) st_sys((WV *)(static_cast<W *>(out.p[j]) + i), m);
            else st_nt((WV *)(static_cast<W *>(out.p[j]) + i), m);
        }
        const f4 z = {0.0f, 0.0f, 0.0f, 0.0f};
        if constexpr (ZALL) {
#pragma unroll
            for (int k = 0; k < K; k++) st_nt((f4 *)const_cast<float *>(in.p[k] + i), z);
        } else {
            st_nt((f4 *)const_cast<float *>(in.p[K - 1] + i), z);
        }
    }
};

// acc += in.  KEEP: the accumulator is read again soon (the ring's residual:
// acc_residual per batch, then pull_grads) — plain loads leave it in the
// Infinity Cache (acc + pull on one reused 64 MiB bucket: 55.8 us per step vs
// 62.2 with nt loads, tools/kernel_variants.hip "train").  Otherwise (a
// one-off accumulate over fresh buffers) both operands stream with nt loads
// (64 MiB: 72 -> 79 % of 8 TB/s, "acc ... ntacc").
template <bool KEEP> struct AccOp {
    float *acc;
    const float *in;
    struct R { f4 a, b; };
    __device__ __forceinline__ void scalar(size_t i) const { acc[i] += in[i]; }
    __device__ __forceinline__ R load(size_t i) const {
        if constexpr (KEEP) return R{ld((const f4 *)(acc + i)), ldn((const f4 *)(in + i))};
        else return R{ldn((const f4 *)(acc + i)), ldn((const f4 *)(in + i))};
    }
    __device__ __forceinline__ void store(size_t i, R r) const { st_nt((f4 *)(acc + i), r.a + r.b); }
};

template <int M> struct ScaleZeroOp { // dst = src / d; zero = 0
    float *dst;
    const float *src;
    float *zero;
    float v;
    __host__ int occ() const { return zero ? 24 : 0; }
    typedef f4 R;
    __device__ __forceinline__ void scalar(size_t i) const {
        float x = src[i];
        dst[i] = scl<M>(x, v);
        if (zero) zero[i] = 0.0f;
    }
    __device__ __forceinline__ R load(size_t i) const { return ldn((const f4 *)(src + i)); }
    __device__ __forceinline__ void store(size_t i, R x) const {
        st_sc1((f4 *)(dst + i), scl4<M>(x, v));
        if (zero) st_sc1((f4 *)(zero + i), f4{0.0f, 0.0f, 0.0f, 0.0f});
    }
};

// dst = src (1R1W) and dst = value (0R1W): the library's own pure streams on
// the same skeleton — the copy ceiling the path's kernels are read against
// (bench.py copy_ceiling) and the plan interpreter's device copies / zero
// fills (ONO_PLAN_COPY / ONO_PLAN_MEMSET), in place of the runtime's blit
// kernels.  Read-once source: nt loads.  The copy's stores are `nt sc1`
// (tools/launch_phases.hip, profiles/r04_launch_phases_s1.txt: 64 MiB 22.02 ->
// 21.18 us, 256 MiB 80.58 -> 78.49 us; the boundary to the next launch 1.9 ->
// 1.2 us, as no dirty L2 lines are left to write back).
template <class T> struct CopyOp {
    typedef typename Wire<T>::V V;
    T *dst;
    const T *src;
    typedef V R;
    __device__ __forceinline__ void scalar(size_t i) const { dst[i] = src[i]; }
    __device__ __forceinline__ R load(size_t i) const { return ldn((const V *)(src + i)); }
    __device__ __forceinline__ void store(size_t i, R x) const { st_sc1((V *)(dst + i), x); }
};
// The fill: 256-thread workgroups and `nt sc1` stores (64 MiB 16.0 -> 10.95
// us, 256 MiB 57.5 -> 39.7 us, against the runtime's fill kernel 11.4 / 40.2).
template <class T> struct FillOp {
    typedef typename Wire<T>::V V;
    static constexpr int block() { return 256; }
    T *dst;
    T value;
    typedef int R;
    __device__ __forceinline__ void scalar(size_t i) const { dst[i] = value; }
    __device__ __forceinline__ R load(size_t) const { return 0; }
    __device__ __forceinline__ void store(size_t i, R) const {
        V x;
        x.x = value; x.y = value; x.z = value; x.w = value;
        st_sc1((V *)(dst + i), x);
    }
};

template <class W> struct EncodeOp {
    typedef typename Wire<W>::V WV;
    W *out;
    const float *in;
    typedef f4 R;
    __device__ __forceinline__ void scalar(size_t i) const { out[i] = Wire<W>::enc(in[i]); }
    __device__ __forceinline__ R load(size_t i) const { return ldn((const f4 *)(in + i)); }
    __device__ __forceinline__ void store(size_t i, R x) const { st_nt((WV *)(out + i), Wire<W>::enc4(x)); }
};

template <class W, int M> struct DecodeScaleOp {
    typedef typename Wire<W>::V WV;
    // (64-thread workgroups: 256 measured 17.46 vs 17.69 us on the tool's data but 18.4 vs 17.6 us on the
    // bench's synthetic f16 gradients, tools/pk_ab.py, profiles/r04_pk_ab_s6.txt)
    float *out;
    const W *in;
    float v;
    typedef WV R;
    __device__ __forceinline__ void scalar(size_t i) const { out[i] = scl<M>(Wire<W>::dec(in[i]), v); }
    __device__ __forceinline__ R load(size_t i) const { return ldn((const WV *)(in + i)); }
    __device__ __forceinline__ void store(size_t i, R h) const {
        st_nt((f4 *)(out + i), scl4<M>(Wire<W>::dec4(h), v));
    }
};

template <class W> struct EncodeZeroOp {
    typedef typename Wire<W>::V WV;
    W *out;
    float *chunk;
    __host__ int occ() const { return 24; }
    typedef f4 R;
    __device__ __forceinline__ void scalar(size_t i) const {
        out[i] = Wire<W>::enc(chunk[i]);
        chunk[i] = 0.0f;
    }
    __device__ __forceinline__ R load(size_t i) const { return ldn((const f4 *)(chunk + i)); }
    __device__ __forceinline__ void store(size_t i, R x) const {
        st_sc1((WV *)(out + i), Wire<W>::enc4(x));
        st_sc1((f4 *)(chunk + i), f4{0.0f, 0.0f, 0.0f, 0.0f});
    }
};

template <class W> struct DecodeAddOp {
    typedef typename Wire<W>::V WV;
    float *acc;
    const W *in;
    struct R { f4 a; WV h; };
    __device__ __forceinline__ void scalar(size_t i) const { acc[i] += Wire<W>::dec(in[i]); }
    __device__ __forceinline__ R load(size_t i) const {
        return R{ld((const f4 *)(acc + i)), ldn((const WV *)(in + i))};
    }
    __device__ __forceinline__ void store(size_t i, R r) const { st_nt((f4 *)(acc + i), r.a + Wire<W>::dec4(r.h)); }
};

template <class W> struct AddEncodeZeroOp {
    typedef typename Wire<W>::V WV;
    W *out;
    float *acc;
    const W *in;
    __host__ int occ() const { return 24; }
    struct R { f4 a; WV h; };
    __device__ __forceinline__ void scalar(size_t i) const {
        float x = acc[i] + Wire<W>::dec(in[i]);
        out[i] = Wire<W>::enc(x);
        acc[i] = 0.0f;
    }
    __device__ __forceinline__ R load(size_t i) const {
        return R{ldn((const f4 *)(acc + i)), ldn((const WV *)(in + i))};
    }
    __device__ __forceinline__ void store(size_t i, R r) const {
        f4 x = r.a + Wire<W>::dec4(r.h);
        st_sc1((WV *)(out + i), Wire<W>::enc4(x));
        st_sc1((f4 *)(acc + i), f4{0.0f, 0.0f, 0.0f, 0.0f});
    }
};

template <class W, int M> struct AddFinishOp {
    typedef typename Wire<W>::V WV;
    float *grad;
    W *out;
    float *acc;
    const W *in;
    float v;
    __host__ int occ() const { return 16; }
    struct R { f4 a; WV h; };
    __device__ __forceinline__ void scalar(size_t i) const {
        float x = acc[i] + Wire<W>::dec(in[i]);
        grad[i] = scl<M>(x, v);
        out[i] = Wire<W>::enc(x);
        acc[i] = 0.0f;
    }
    __device__ __forceinline__ R load(size_t i) const {
        return R{ldn((const f4 *)(acc + i)), ldn((const WV *)(in + i))};
    }
    __device__ __forceinline__ void store(size_t i, R r) const {
        f4 x = r.a + Wire<W>::dec4(r.h);
        st_sc1((f4 *)(grad + i), scl4<M>(x, v));
        st_sc1((WV *)(out + i), Wire<W>::enc4(x));
        st_sc1((f4 *)(acc + i), f4{0.0f, 0.0f, 0.0f, 0.0f});
    }
};

// ---------------------------------------------------------- synthetic ----
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
struct SynthOp {
    float *out;
    uint64_t key;
    size_t offset;
    typedef int R;
    __device__ __forceinline__ float gen(size_t j) const {
        const uint64_t G = 0x9E3779B97F4A7C15ULL;
        uint64_t i = (uint64_t)(offset + j);
        uint64_t h1 = mix64(key + G * (i + 1));
        uint64_t h2 = mix64(h1 ^ 0xD1B54A32D192ED03ULL);
        uint32_t cls = (uint32_t)((h1 >> 32) % 100u);
        uint32_t sign = (uint32_t)(h2 >> 63);
        if (cls == 0) return __builtin_bit_cast(float, sign << 31);
        if (cls == 1) {
            float x = (float)(uint32_t)((h2 >> 8) & 0x3FFFFu) * 0x1p-32f;
            return sign ? -x : x;
        }
        if (cls == 2) {
            uint32_t e = (uint32_t)((h2 >> 8) % 13u);
            uint32_t m10 = (uint32_t)((h2 >> 16) & 0x3FFu);
            return __builtin_bit_cast(float, (sign << 31) | ((e + 117u) << 23) | (m10 << 13) | 0x1000u);
        }
        int32_t s4 = (int32_t)(h2 & 0xFFFF) + (int32_t)((h2 >> 16) & 0xFFFF) +
                     (int32_t)((h2 >> 32) & 0xFFFF) + (int32_t)((h2 >> 48) & 0xFFFF);
        return (float)(s4 - 131070) * 0x1.3c1a2ep-22f;
    }
    __device__ __forceinline__ void scalar(size_t i) const { out[i] = gen(i); }
    __device__ __forceinline__ R load(size_t) const { return 0; }
    __device__ __forceinline__ void store(size_t i, R) const {
        st_nt((f4 *)(out + i), f4{gen(i), gen(i + 1), gen(i + 2), gen(i + 3)});
    }
};

// --------------------------------------------------------- optimizers ----
// BlockingShard::update_params (shard.rs:74-92) fused with the optimizer
// (gradient_descent.rs:44-47, gradient_descent_with_momentum.rs:56-62, adam.rs:76-91).
template <int KIND, int M, bool ZERO, bool PZ> struct OptOp {
    float *g, *w, *v, *s;
    float *w2;  // optional copy of the updated parameters (all_reduce.rs:132), may be NULL
    float lr, mu, b1, omb1, b2, omb2, eps, step, nw;
    int fence;  // w2 is read by other ranks after the next flag barrier (xGMI PS)
    struct R { f4 g, w, v, s; };
    __host__ int occ() const { return KIND == ONO_OPT_GD ? 16 : KIND == ONO_OPT_MOMENTUM || KIND == ONO_OPT_ADAM ? 10 : 0; }
    __device__ __forceinline__ void finish() const {
        if (fence) peer_stores_done();
    }
    // one element in two halves, the scaled gradient and the moments, then the
    // parameter (the vector path stores the first half's results before it
    // runs the second's square root and division)
    __device__ __forceinline__ float moments(float gi, float &vi, float &si) const {
        const float gg = scl<M>(PZ ? gi + 0.0f : gi, nw);
        if constexpr (KIND == ONO_OPT_MOMENTUM) {
            vi = (mu * vi) + gg;
        } else if constexpr (KIND == ONO_OPT_ADAM) {
            vi = b1 * vi + omb1 * gg;
            si = b2 * si + omb2 * (gg * gg);
        }
        return gg;
    }
    __device__ __forceinline__ void param(float gg, float &wi, float vi, float si) const {
        if constexpr (KIND == ONO_OPT_GD) {
            wi -= lr * gg;
        } else if constexpr (KIND == ONO_OPT_MOMENTUM) {
            wi -= lr * vi;
        } else if constexpr (KIND == ONO_OPT_ADAM) {
            wi -= step * vi / (__builtin_sqrtf(si) + eps);
        } else {
            wi += gg;
        }
    }
    __device__ __forceinline__ void one(float &gi, float &wi, float &vi, float &si) const {
        const float gg = moments(gi, vi, si);
        param(gg, wi, vi, si);
        gi = ZERO ? 0.0f : gg;
    }
    __device__ __forceinline__ void scalar(size_t i) const {
        float gi = g[i], wi = w[i], vi = 0.0f, si = 0.0f;
        if constexpr (KIND == ONO_OPT_MOMENTUM || KIND == ONO_OPT_ADAM) vi = v[i];
        if constexpr (KIND == ONO_OPT_ADAM) si = s[i];
        one(gi, wi, vi, si);
        g[i] = gi;
        w[i] = wi;
        if (w2) {
            if (fence) st_sys(w2 + i, wi);
            else w2[i] = wi;
        }
        if constexpr (KIND == ONO_OPT_MOMENTUM || KIND == ONO_OPT_ADAM) v[i] = vi;
        if constexpr (KIND == ONO_OPT_ADAM) s[i] = si;
    }
    // every operand is read once and rewritten: nt loads (+3-5 % over plain
    // loads on fresh buffers for GD / momentum / Adam, profiles/r02_opt_variants.txt)
    __device__ __forceinline__ R load(size_t i) const {
        R r{};
        r.g = ldn((const f4 *)(g + i));
        r.w = ldn((const f4 *)(w + i));
        if constexpr (KIND == ONO_OPT_MOMENTUM || KIND == ONO_OPT_ADAM) r.v = ldn((const f4 *)(v + i));
        if constexpr (KIND == ONO_OPT_ADAM) r.s = ldn((const f4 *)(s + i));
        return r;
    }
    __device__ __forceinline__ void store(size_t i, R r) const {
        float gg[4] = {r.g.x, r.g.y, r.g.z, r.g.w}, ww[4] = {r.w.x, r.w.y, r.w.z, r.w.w};
        float vv[4] = {r.v.x, r.v.y, r.v.z, r.v.w}, ss[4] = {r.s.x, r.s.y, r.s.z, r.s.w};
#pragma unroll
        for (int j = 0; j < 4; j++) gg[j] = moments(gg[j], vv[j], ss[j]);
        // Adam: the moments and the gradient leave before the square roots and
        // divisions (112.6 -> 100 us per 64 MiB launch, 67 -> 75 % of HBM);
        // GD / momentum keep gradient, parameters, copy, moment (measured no
        // better reordered)
        if constexpr (KIND == ONO_OPT_ADAM) {
            st_nt((f4 *)(v + i), f4{vv[0], vv[1], vv[2], vv[3]});
            st_nt((f4 *)(s + i), f4{ss[0], ss[1], ss[2], ss[3]});
            st_nt((f4 *)(g + i), ZERO ? f4{0.0f, 0.0f, 0.0f, 0.0f} : f4{gg[0], gg[1], gg[2], gg[3]});
        }
#pragma unroll
        for (int j = 0; j < 4; j++) param(gg[j], ww[j], vv[j], ss[j]);
        if constexpr (KIND != ONO_OPT_ADAM)
            st_nt((f4 *)(g + i), ZERO ? f4{0.0f, 0.0f, 0.0f, 0.0f} : f4{gg[0], gg[1], gg[2], gg[3]});
        st_nt((f4 *)(w + i), f4{ww[0], ww[1], ww[2], ww[3]});
        if (w2) {  // fence: peers read the copy after the next flag barrier (system-coherent stores)
            if (fence) st_sys((f4 *)(w2 + i), f4{ww[0], ww[1], ww[2], ww[3]});
            else st_nt((f4 *)(w2 + i), f4{ww[0], ww[1], ww[2], ww[3]});
        }
        if constexpr (KIND == ONO_OPT_MOMENTUM) st_nt((f4 *)(v + i), f4{vv[0], vv[1], vv[2], vv[3]});
    }
};

template <int K>
hipError_t sum_scale_k(float *out, const Ptrs &p, size_t n, const Scale &sc, hipStream_t s) {
    auto ph = {phase_of(out, 4), phase_of(p.p[0], 4), phase_of(p.p[K > 1 ? 1 : 0], 4),
               phase_of(p.p[K > 2 ? 2 : 0], 4), phase_of(p.p[K > 3 ? 3 : 0], 4),
               phase_of(p.p[K > 4 ? 4 : 0], 4), phase_of(p.p[K > 5 ? 5 : 0], 4),
               phase_of(p.p[K > 6 ? 6 : 0], 4), phase_of(p.p[K > 7 ? 7 : 0], 4),
               phase_of(p.p[K > 8 ? 8 : 0], 4), phase_of(p.p[K > 9 ? 9 : 0], 4),
               phase_of(p.p[K > 10 ? 10 : 0], 4), phase_of(p.p[K > 11 ? 11 : 0], 4),
               phase_of(p.p[K > 12 ? 12 : 0], 4), phase_of(p.p[K > 13 ? 13 : 0], 4),
               phase_of(p.p[K > 14 ? 14 : 0], 4), phase_of(p.p[K > 15 ? 15 : 0], 4)};
    bool alias = false;  // in-place (out == some input): plain loads
    for (int j = 0; j < K; j++) alias |= (p.p[j] == out);
    if (alias) {
        switch (sc.mode) {
        case SCALE_NONE: return launch_ew(SumScaleOp<K, SCALE_NONE, false>{p, out, sc.v}, n, ph, s);
        case SCALE_RECIP: return launch_ew(SumScaleOp<K, SCALE_RECIP, false>{p, out, sc.v}, n, ph, s);
        default: return launch_ew(SumScaleOp<K, SCALE_DIV, false>{p, out, sc.v}, n, ph, s);
        }
    }
    if constexpr (K >= 4) {
        if (n >= kSerialElems) {
            switch (sc.mode) {
            case SCALE_NONE: return launch_ew(SumScaleOp<K, SCALE_NONE, true, true>{p, out, sc.v}, n, ph, s);
            case SCALE_RECIP: return launch_ew(SumScaleOp<K, SCALE_RECIP, true, true>{p, out, sc.v}, n, ph, s);
            default: return launch_ew(SumScaleOp<K, SCALE_DIV, true, true>{p, out, sc.v}, n, ph, s);
            }
        }
    }
    switch (sc.mode) {
    case SCALE_NONE: return launch_ew(SumScaleOp<K, SCALE_NONE, true>{p, out, sc.v}, n, ph, s);
    case SCALE_RECIP: return launch_ew(SumScaleOp<K, SCALE_RECIP, true>{p, out, sc.v}, n, ph, s);
    default: return launch_ew(SumScaleOp<K, SCALE_DIV, true>{p, out, sc.v}, n, ph, s);
    }
}

template <int K>
hipError_t sum_scale_dispatch(int k, float *out, const Ptrs &p, size_t n, const Scale &sc,
                              hipStream_t s) {
    if constexpr (K > ONO_MAX_INPUTS) {
        return hipErrorInvalidValue;
    } else {
        if (k == K) return sum_scale_k<K>(out, p, n, sc, s);
        return sum_scale_dispatch<K + 1>(k, out, p, n, sc, s);
    }
}

template <int KIND, bool ZERO>
hipError_t opt_kind(const OptLaunch &o, float *g, float *w, float *v, float *s_, float *w2, size_t n,
                    hipStream_t st, bool fence) {
    Scale sc = make_scale(o.nworkers);
    float omb1 = 1.0f - o.beta1, omb2 = 1.0f - o.beta2;
    auto ph = {phase_of(g, 4), phase_of(w, 4), v ? phase_of(v, 4) : phase_of(g, 4),
               s_ ? phase_of(s_, 4) : phase_of(g, 4), w2 ? phase_of(w2, 4) : phase_of(g, 4)};
#define ONO_OPT_OP(MODE, PZ) \
    OptOp<KIND, MODE, ZERO, PZ>{g,        w,       v,    s_,         w2,    o.lr, o.momentum, o.beta1, omb1, o.beta2, \
                                omb2,     o.eps,   o.step_size, sc.v, fence ? 1 : 0}
    if (o.plus_zero) {
        switch (sc.mode) {
        case SCALE_NONE: return launch_ew(ONO_OPT_OP(SCALE_NONE, true), n, ph, st);
        case SCALE_RECIP: return launch_ew(ONO_OPT_OP(SCALE_RECIP, true), n, ph, st);
        default: return launch_ew(ONO_OPT_OP(SCALE_DIV, true), n, ph, st);
        }
    }
    switch (sc.mode) {
    case SCALE_NONE: return launch_ew(ONO_OPT_OP(SCALE_NONE, false), n, ph, st);
    case SCALE_RECIP: return launch_ew(ONO_OPT_OP(SCALE_RECIP, false), n, ph, st);
    default: return launch_ew(ONO_OPT_OP(SCALE_DIV, false), n, ph, st);
    }
#undef ONO_OPT_OP
}

template <class W> unsigned wph(const W *p) { return phase_of(p, sizeof(W)); }

template <int K, class W>
hipError_t direct_k(float *grad, const Outs &out, int nout, bool sys_out, const Ptrs &p, size_t n, const Scale &sc,
                    bool zall, hipStream_t s) {
    unsigned ph[2 * ONO_MAX_INPUTS + 1];
    int c = 0;
    ph[c++] = phase_of(grad, 4);
    for (int j = 0; j < nout; j++) ph[c++] = wph(static_cast<const W *>(out.p[j]));
    for (int k = 0; k < K; k++) ph[c++] = phase_of(p.p[k], 4);
    // SCALE_NONE (d == 1) runs as a multiply by 1: the identity, -0 and NaN payloads included
    const int mode = sc.mode == SCALE_DIV ? SCALE_DIV : SCALE_RECIP;
    const float v = sc.mode == SCALE_NONE ? 1.0f : sc.v;
    if (zall) return launch_ew_arr(DirectOp<K, W, true>{p, grad, out, nout, sys_out ? 1 : 0, v, mode}, n, ph, c, s);
    return launch_ew_arr(DirectOp<K, W, false>{p, grad, out, nout, sys_out ? 1 : 0, v, mode}, n, ph, c, s);
}

template <int K, class W>
hipError_t direct_dispatch(int k, float *grad, const Outs &out, int nout, bool sys_out, const Ptrs &p, size_t n,
                           const Scale &sc, bool zall, hipStream_t s) {
    if constexpr (K > ONO_MAX_INPUTS) {
        return hipErrorInvalidValue;
    } else {
        if (k == K) return direct_k<K, W>(grad, out, nout, sys_out, p, n, sc, zall, s);
        return direct_dispatch<K + 1, W>(k, grad, out, nout, sys_out, p, n, sc, zall, s);
    }
}

}  // namespace

// ================================================================ API ======
Scale make_scale(float d) {
    if (d == 1.0f) return Scale{SCALE_NONE, 1.0f};
    uint32_t u;
    memcpy(&u, &d, 4);
    uint32_t e = (u >> 23) & 0xFF, m = u & 0x7FFFFF;
    // power of two with an exactly representable normal reciprocal
    if (m == 0 && e >= 2 && e <= 252) return Scale{SCALE_RECIP, 1.0f / d};
    return Scale{SCALE_DIV, d};
}

std::vector<size_t> split_chunks(size_t len, size_t n) {
    std::vector<size_t> off{0};
    if (n == 0) return off;
    size_t base = len / n, rem = len % n, pos = 0;
    while (pos < len && off.size() < n + 1) {
        size_t l = base + (rem > 0 ? 1 : 0);
        if (rem > 0) rem--;
        pos += l;
        off.push_back(pos);
    }
    return off;
}

hipError_t launch_sum_scale(float *out, const float *const *ins, int k, size_t n, float divisor,
                            hipStream_t s) {
    if (k < 1 || k > ONO_MAX_INPUTS) return hipErrorInvalidValue;
    Ptrs p{};
    for (int j = 0; j < k; j++) p.p[j] = ins[j];
    return sum_scale_dispatch<1>(k, out, p, n, make_scale(divisor), s);
}

template <class W>
hipError_t launch_direct_multi(float *grad, W *const *outs, int nout, bool sys_out, const float *const *ins, int k,
                               size_t n, float divisor, bool zero_all, hipStream_t s) {
    if (k < 1 || k > ONO_MAX_INPUTS || nout < 0 || nout > ONO_MAX_INPUTS) return hipErrorInvalidValue;
    Ptrs p{};
    for (int j = 0; j < k; j++) p.p[j] = ins[j];
    Outs o{};
    for (int j = 0; j < nout; j++) o.p[j] = outs[j];
    return direct_dispatch<1, W>(k, grad, o, nout, sys_out, p, n, make_scale(divisor), zero_all, s);
}
template <class W>
hipError_t launch_direct(float *grad, W *out, const float *const *ins, int k, size_t n, float divisor,
                         bool zero_all, hipStream_t s) {
    return launch_direct_multi<W>(grad, &out, out ? 1 : 0, false, ins, k, n, divisor, zero_all, s);
}
template hipError_t launch_direct<uint16_t>(float *, uint16_t *, const float *const *, int, size_t, float, bool,
                                            hipStream_t);
template hipError_t launch_direct<float>(float *, float *, const float *const *, int, size_t, float, bool,
                                         hipStream_t);
template hipError_t launch_direct_multi<uint16_t>(float *, uint16_t *const *, int, bool, const float *const *, int,
                                                  size_t, float, bool, hipStream_t);
template hipError_t launch_direct_multi<float>(float *, float *const *, int, bool, const float *const *, int, size_t,
                                               float, bool, hipStream_t);

hipError_t launch_acc(float *acc, const float *in, size_t n, hipStream_t s, bool keep) {
    if (keep) return launch_ew(AccOp<true>{acc, in}, n, {phase_of(acc, 4), phase_of(in, 4)}, s);
    return launch_ew(AccOp<false>{acc, in}, n, {phase_of(acc, 4), phase_of(in, 4)}, s);
}

hipError_t launch_scale_zero(float *dst, const float *src, size_t n, float divisor, float *zero,
                             hipStream_t s) {
    Scale sc = make_scale(divisor);
    auto ph = {phase_of(dst, 4), phase_of(src, 4), zero ? phase_of(zero, 4) : phase_of(dst, 4)};
    switch (sc.mode) {
    case SCALE_NONE: return launch_ew(ScaleZeroOp<SCALE_NONE>{dst, src, zero, sc.v}, n, ph, s);
    case SCALE_RECIP: return launch_ew(ScaleZeroOp<SCALE_RECIP>{dst, src, zero, sc.v}, n, ph, s);
    default: return launch_ew(ScaleZeroOp<SCALE_DIV>{dst, src, zero, sc.v}, n, ph, s);
    }
}

template <class T> hipError_t launch_copy(T *dst, const T *src, size_t n, hipStream_t s) {
    return launch_ew(CopyOp<T>{dst, src}, n, {wph(dst), wph(src)}, s);
}
template <class T> hipError_t launch_fill(T *dst, T value, size_t n, hipStream_t s) {
    return launch_ew(FillOp<T>{dst, value}, n, {wph(dst)}, s);
}
template hipError_t launch_copy<float>(float *, const float *, size_t, hipStream_t);
template hipError_t launch_copy<uint16_t>(uint16_t *, const uint16_t *, size_t, hipStream_t);
template hipError_t launch_fill<float>(float *, float, size_t, hipStream_t);
template hipError_t launch_fill<uint16_t>(uint16_t *, uint16_t, size_t, hipStream_t);

hipError_t launch_synth(float *out, size_t n, uint64_t seed, uint64_t rank, size_t offset,
                        hipStream_t s) {
    auto mix = [](uint64_t z) {
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        return z ^ (z >> 31);
    };
    uint64_t key = mix(seed + 0x9E3779B97F4A7C15ULL * (rank + 1));
    return launch_ew(SynthOp{out, key, offset}, n, {phase_of(out, 4)}, s);
}

template <class W> hipError_t launch_encode(W *out, const float *in, size_t n, hipStream_t s) {
    return launch_ew(EncodeOp<W>{out, in}, n, {wph(out), phase_of(in, 4)}, s);
}
template <class W>
hipError_t launch_decode_scale(float *out, const W *in, size_t n, float divisor, hipStream_t s, KernelDone *done) {
    Scale sc = make_scale(divisor);
    auto ph = {phase_of(out, 4), wph(in)};
    switch (sc.mode) {
    case SCALE_NONE: return launch_ew(DecodeScaleOp<W, SCALE_NONE>{out, in, sc.v}, n, ph, s, done);
    case SCALE_RECIP: return launch_ew(DecodeScaleOp<W, SCALE_RECIP>{out, in, sc.v}, n, ph, s, done);
    default: return launch_ew(DecodeScaleOp<W, SCALE_DIV>{out, in, sc.v}, n, ph, s, done);
    }
}
template <class W> hipError_t launch_encode_zero(W *out, float *chunk, size_t n, hipStream_t s, KernelDone *done) {
    return launch_ew(EncodeZeroOp<W>{out, chunk}, n, {wph(out), phase_of(chunk, 4)}, s, done);
}
template <class W> hipError_t launch_decode_add(float *acc, const W *in, size_t n, hipStream_t s) {
    return launch_ew(DecodeAddOp<W>{acc, in}, n, {phase_of(acc, 4), wph(in)}, s);
}
template <class W>
hipError_t launch_add_encode_zero(W *out, float *acc, const W *in, size_t n, hipStream_t s, KernelDone *done) {
    return launch_ew(AddEncodeZeroOp<W>{out, acc, in}, n, {wph(out), phase_of(acc, 4), wph(in)}, s, done);
}
template <class W>
hipError_t launch_add_finish(float *grad, W *out, float *acc, const W *in, size_t n, float divisor,
                             hipStream_t s, KernelDone *done) {
    Scale sc = make_scale(divisor);
    auto ph = {phase_of(grad, 4), wph(out), phase_of(acc, 4), wph(in)};
    switch (sc.mode) {
    case SCALE_NONE: return launch_ew(AddFinishOp<W, SCALE_NONE>{grad, out, acc, in, sc.v}, n, ph, s, done);
    case SCALE_RECIP: return launch_ew(AddFinishOp<W, SCALE_RECIP>{grad, out, acc, in, sc.v}, n, ph, s, done);
    default: return launch_ew(AddFinishOp<W, SCALE_DIV>{grad, out, acc, in, sc.v}, n, ph, s, done);
    }
}

#define ONO_INST(W)                                                                            \
    template hipError_t launch_encode<W>(W *, const float *, size_t, hipStream_t);            \
    template hipError_t launch_decode_scale<W>(float *, const W *, size_t, float, hipStream_t, KernelDone *); \
    template hipError_t launch_encode_zero<W>(W *, float *, size_t, hipStream_t, KernelDone *);             \
    template hipError_t launch_decode_add<W>(float *, const W *, size_t, hipStream_t);        \
    template hipError_t launch_add_encode_zero<W>(W *, float *, const W *, size_t, hipStream_t, KernelDone *); \
    template hipError_t launch_add_finish<W>(float *, W *, float *, const W *, size_t, float, hipStream_t, KernelDone *);
ONO_INST(uint16_t)
ONO_INST(float)
#undef ONO_INST

hipError_t launch_opt_update(const OptLaunch &o, float *g, float *w, float *v, float *s_, size_t n,
                             bool zero_grad, hipStream_t st, float *w_copy, bool copy_for_peers) {
#define ONO_OPT_CASE(KIND)                                                                     \
    case KIND:                                                                                 \
        return zero_grad ? opt_kind<KIND, true>(o, g, w, v, s_, w_copy, n, st, copy_for_peers) \
                         : opt_kind<KIND, false>(o, g, w, v, s_, w_copy, n, st, copy_for_peers);
    switch (o.kind) {
        ONO_OPT_CASE(ONO_OPT_GD)
        ONO_OPT_CASE(ONO_OPT_MOMENTUM)
        ONO_OPT_CASE(ONO_OPT_ADAM)
        ONO_OPT_CASE(ONO_OPT_ADD)
    default: return hipErrorInvalidValue;
    }
#undef ONO_OPT_CASE
}

}  // namespace ono
