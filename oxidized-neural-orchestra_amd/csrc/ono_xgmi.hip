// ono_xgmi.hip — gfx950 kernels of the xGMI peer-access schedule (ONO_ALGO_XGMI).
//
// The ranks of one node map each other's exchange region (IPC, uncached HBM)
// and move chunk slices with plain vector loads and stores over xGMI — no
// RCCL, no staging copies.  One launch drives every peer link at once: the
// workgroups of a launch are dealt round-robin over the peers' segments
// (blockIdx % nseg), so all n-1 links carry traffic from the first wave on.
//
//   push  (scatter)  x = residual slice; peer.rbuf[k] = x; residual slice = 0
//                    (worker_ring.rs:122, :133 — the slice leaves and is zeroed)
//   pull  (gather)   grad[chunk of q] = dec(peer_q.obuf) / d
//                    (worker_ring.rs:200 + the ÷n of param_manager.rs:183-188)
//   barrier          every rank stores the round's epoch into every peer's flag
//                    slot, then waits for all n-1 flags of its own (bounded:
//                    a rank that never arrives sets the ring's error word
//                    after ~timeout instead of hanging the grid)
//
// The owner's chain between the two (DirectOp in ono_kernels.hip) is the
// reference arithmetic; these kernels only move bytes, HBM- and link-bound.
#include <hip/hip_runtime.h>

#include "ono_device.h"
#include "ono_internal.h"

namespace ono {
namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef uint16_t h4 __attribute__((ext_vector_type(4)));

constexpr int kXBlock = 64;  // one wave per workgroup, one 16-B vector per lane (as ew_kernel)

// half 2.7.1 f16_to_f32 = v_cvt_f32_f16, NaN payloads included (ono_kernels.hip from_f16)
__device__ __forceinline__ float x_from_f16(uint16_t b) { return (float)__builtin_bit_cast(_Float16, b); }

template <int M> __device__ __forceinline__ float xs(float x, float v) {
    if constexpr (M == SCALE_NONE) return x;
    else if constexpr (M == SCALE_RECIP) return x * v;
    else return x / v;
}

// Element geometry of one segment: [0, head) scalar, [head, head + 4 nvec)
// 4-wide, tail scalar; head == kScalarOnly: the operands' 4-element phases
// differ, every element goes through the scalar path.
__device__ __forceinline__ void seg_geometry(const XSeg &s, uint32_t t, int lane, bool &vec_ok, size_t &v,
                                             size_t &nvec) {
    nvec = (s.n - s.head) / 4;
    v = (size_t)t * kXBlock + lane;
    vec_ok = v < nvec;
}

// f32 slice -> peer receive slot; ZERO: then zero the slice (the ring's
// residual); without: a plain copy (the PS mode's gradient stays the caller's)
template <bool ZERO> struct PushOp {
    static constexpr bool kPeerStores = true;
    __device__ __forceinline__ static void scalar(const XSeg &s, size_t i) {
        float *src = (float *)s.src;
        st_sys((float *)s.dst + i, src[i]);
        if constexpr (ZERO) src[i] = 0.0f;
    }
    __device__ __forceinline__ static void vec(const XSeg &s, size_t i) {
        f4 *src = (f4 *)((float *)s.src + i);
        if constexpr (ZERO) {
            f4 x = *src;  // plain load: the same lines are rewritten (zeroed) below
            st_sys_async((f4 *)((float *)s.dst + i), x);
            __builtin_nontemporal_store(f4{0.0f, 0.0f, 0.0f, 0.0f}, src);
        } else {
            st_sys_async((f4 *)((float *)s.dst + i), __builtin_nontemporal_load(src));
        }
    }
};

// host-fed input: the caller's bucket (registered) or a pinned staging slot -> the residual; the host
// memory is read system-coherent (sc0 sc1: no cache keeps an earlier call's lines of it)
template <bool SYS> struct HostInOp {  // SYS = false: nontemporal loads (measurement, ONO_XGMI_HOST_IN=plain)
    static constexpr bool kPeerStores = false;
    __device__ __forceinline__ static void scalar(const XSeg &s, size_t i) {
        const float *p = (const float *)s.src + i;
        ((float *)s.dst)[i] = SYS ? ld_sys(p) : __builtin_nontemporal_load(p);
    }
    __device__ __forceinline__ static void vec(const XSeg &s, size_t i) {
        const f4 *p = (const f4 *)((const float *)s.src + i);
        *(f4 *)((float *)s.dst + i) = SYS ? ld_sys(p) : __builtin_nontemporal_load(p);
    }
};

template <int M> struct PullF32Op {  // owner's f32 result (already ÷n) -> grad
    static constexpr bool kPeerStores = false;
    float v;
    __device__ __forceinline__ void scalar(const XSeg &s, size_t i) const {
        ((float *)s.dst)[i] = xs<M>(ld_sys((const float *)s.src + i), v);
    }
    __device__ __forceinline__ void vec(const XSeg &s, size_t i) const {
        f4 x = ld_sys((const f4 *)((const float *)s.src + i));
        if constexpr (M == SCALE_RECIP) x = x * v;
        else if constexpr (M == SCALE_DIV) x = x / v;
        __builtin_nontemporal_store(x, (f4 *)((float *)s.dst + i));
    }
};

template <int M> struct PullF16Op {  // owner's f16 message -> grad = f32(h) / d
    static constexpr bool kPeerStores = false;
    float v;
    __device__ __forceinline__ void scalar(const XSeg &s, size_t i) const {
        ((float *)s.dst)[i] = xs<M>(x_from_f16(ld_sys((const uint16_t *)s.src + i)), v);
    }
    __device__ __forceinline__ void vec(const XSeg &s, size_t i) const {
        h4 h = ld_sys((const h4 *)((const uint16_t *)s.src + i));
        f4 x = {xs<M>(x_from_f16(h.x), v), xs<M>(x_from_f16(h.y), v), xs<M>(x_from_f16(h.z), v),
                xs<M>(x_from_f16(h.w), v)};
        __builtin_nontemporal_store(x, (f4 *)((float *)s.dst + i));
    }
};

template <class Op>
__global__ __launch_bounds__(kXBlock) void xseg_kernel(Op op, XSegs g) {
    const int j = (int)(blockIdx.x % (unsigned)g.nseg);
    const uint32_t t = blockIdx.x / (unsigned)g.nseg;
    const XSeg s = g.s[j];
    if (t >= s.tiles) return;
    const int lane = threadIdx.x;
    if (s.head == kScalarOnly) {  // 256 elements per tile, 4 per lane
#pragma unroll
        for (int u = 0; u < 4; u++) {
            size_t i = (size_t)t * (4 * kXBlock) + (size_t)u * kXBlock + lane;
            if (i < s.n) op.scalar(s, i);
        }
        if constexpr (Op::kPeerStores) peer_stores_done();
        return;
    }
    bool vec_ok;
    size_t v, nvec;
    seg_geometry(s, t, lane, vec_ok, v, nvec);
    if (t == 0) {
        const size_t tail0 = s.head + 4 * nvec;
        if ((size_t)lane < s.head) op.scalar(s, lane);
        if ((size_t)lane < s.n - tail0) op.scalar(s, tail0 + lane);
    }
    if (vec_ok) op.vec(s, s.head + 4 * v);
    if constexpr (Op::kPeerStores) peer_stores_done();
}

// One workgroup; lane q < n signals peer q and waits for q's signal.
__global__ __launch_bounds__(64) void xbarrier_kernel(XBarrier b) {
    const int q = threadIdx.x;
    __atomic_thread_fence(__ATOMIC_SEQ_CST);  // (system scope) earlier launches' stores first
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the fence's own wait can be dropped (guide §6 G16 P12)
    if (q < b.n && q != b.pos)
        __hip_atomic_store(b.peer_flags[q] + b.pos, b.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (q < b.n && q != b.pos) {
        const uint64_t t0 = wall_clock64();
        uint32_t spins = 0;
        for (;;) {
            const uint64_t f = __hip_atomic_load(b.my_flags + q, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
            // a peer is at most one barrier ahead (it cannot pass barrier e+1 without this rank's e+1);
            // anything larger was not written by this ring's peer for this ring: fail the round loudly
            if (f > b.epoch + 1) {
                __hip_atomic_store(b.err, 3u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                break;
            }
            if (f >= b.epoch) break;
            if (wall_clock64() - t0 > b.timeout_ticks) {
                __hip_atomic_store(b.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                break;
            }
            if ((++spins & 63u) == 0 && __hip_atomic_load(b.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM))
                break;  // timed out elsewhere, or ono_ring_abort()
            __builtin_amdgcn_s_sleep(2);
        }
    }
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
}

// Ring-id stamps of a fresh exchange region, lane p -> page p (page 0: the id
// slot of the flag page); verification reads them back through an import.
constexpr size_t kXPage = 4096;
__global__ __launch_bounds__(64) void xstamp_kernel(uint8_t *region, uint64_t npages, uint64_t id_off, uint64_t id) {
    const uint64_t p = (uint64_t)blockIdx.x * 64 + threadIdx.x;
    if (p < npages) st_sys(reinterpret_cast<uint64_t *>(region + (p ? p * kXPage : id_off)), id);
    peer_stores_done();
}
__global__ __launch_bounds__(64) void xverify_kernel(const uint8_t *region, uint64_t npages, uint64_t id_off,
                                                     uint64_t id, uint8_t *bad) {
    const uint64_t p = (uint64_t)blockIdx.x * 64 + threadIdx.x;
    if (p < npages) bad[p] = ld_sys(reinterpret_cast<const uint64_t *>(region + (p ? p * kXPage : id_off))) != id;
}
// Teardown: lane q tells peer q that this rank is done with its region.
__global__ __launch_bounds__(64) void xsignal_kernel(XSignal sg) {
    const int q = threadIdx.x;
    if (q < sg.n && q != sg.pos) st_sys(sg.peer_done[q] + sg.pos, sg.peer_id[q]);
    peer_stores_done();
}

// Release bookkeeping: an importer counts itself in (at import) and out (at
// close) of the exporter's region; the exporter frees only when they match.
__global__ __launch_bounds__(64) void xbump_kernel(uint64_t *counter) {
    if (threadIdx.x == 0) __hip_atomic_fetch_add(counter, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    peer_stores_done();
}

// Host-fed rounds: a system-scope fence (L2 write-back + invalidate) on every
// XCD between the copy engine's writes and the round's first read of them,
// and between the round's last writes and the copy engine's read.  The
// workgroups are dealt round-robin over the XCDs, so 256 of them reach each
// XCD's L2 several times over.
constexpr unsigned kXFenceBlocks = 256;
template <bool ACQUIRE> __global__ __launch_bounds__(64) void xfence_kernel() {
    if (threadIdx.x == 0) {  // the compiler leaves the write-back's wait out of a bare fence; the waits are explicit
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // (system scope) L2 write-back
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if constexpr (ACQUIRE) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // L2 invalidate
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
}

template <class Op>
hipError_t launch_segs(const Op &op, XSegs g, hipStream_t s) {
    uint32_t tiles = 0;
    for (int j = 0; j < g.nseg; j++) {
        XSeg &x = g.s[j];
        if (x.head != kScalarOnly) {
            if (x.head > x.n) x.head = (uint32_t)x.n;
            size_t nvec = (x.n - x.head) / 4;
            x.tiles = (uint32_t)std::max<size_t>(1, (nvec + kXBlock - 1) / kXBlock);
        } else {
            x.tiles = (uint32_t)((x.n + 4 * kXBlock - 1) / (4 * kXBlock));
        }
        if (x.n == 0) x.tiles = 0;
        tiles = std::max(tiles, x.tiles);
    }
    if (g.nseg == 0 || tiles == 0) return hipSuccess;
    const size_t blocks = (size_t)tiles * (size_t)g.nseg;
    if (blocks > 0x7FFFFFFFu) return hipErrorInvalidValue;
    hipLaunchKernelGGL(xseg_kernel<Op>, dim3((unsigned)blocks), dim3(kXBlock), 0, s, op, g);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_xgmi_push(const XSegs &g, bool zero_src, hipStream_t s) {
    return zero_src ? launch_segs(PushOp<true>{}, g, s) : launch_segs(PushOp<false>{}, g, s);
}

hipError_t launch_xgmi_host_in(const XSegs &g, hipStream_t s, bool sys) {
    return sys ? launch_segs(HostInOp<true>{}, g, s) : launch_segs(HostInOp<false>{}, g, s);
}

hipError_t launch_xgmi_pull(const XSegs &g, bool f16, float divisor, hipStream_t s) {
    Scale sc = make_scale(divisor);
    if (f16) {
        switch (sc.mode) {
        case SCALE_NONE: return launch_segs(PullF16Op<SCALE_NONE>{sc.v}, g, s);
        case SCALE_RECIP: return launch_segs(PullF16Op<SCALE_RECIP>{sc.v}, g, s);
        default: return launch_segs(PullF16Op<SCALE_DIV>{sc.v}, g, s);
        }
    }
    switch (sc.mode) {
    case SCALE_NONE: return launch_segs(PullF32Op<SCALE_NONE>{sc.v}, g, s);
    case SCALE_RECIP: return launch_segs(PullF32Op<SCALE_RECIP>{sc.v}, g, s);
    default: return launch_segs(PullF32Op<SCALE_DIV>{sc.v}, g, s);
    }
}

hipError_t launch_xgmi_stamp(uint8_t *region, size_t npages, size_t id_off, uint64_t id, hipStream_t s) {
    if (npages == 0) return hipSuccess;
    hipLaunchKernelGGL(xstamp_kernel, dim3((unsigned)((npages + 63) / 64)), dim3(64), 0, s, region, (uint64_t)npages,
                       (uint64_t)id_off, id);
    return hipGetLastError();
}

hipError_t launch_xgmi_verify(const uint8_t *region, size_t npages, size_t id_off, uint64_t id, uint8_t *bad,
                              hipStream_t s) {
    if (npages == 0) return hipSuccess;
    hipLaunchKernelGGL(xverify_kernel, dim3((unsigned)((npages + 63) / 64)), dim3(64), 0, s, region,
                       (uint64_t)npages, (uint64_t)id_off, id, bad);
    return hipGetLastError();
}

hipError_t launch_xgmi_signal(const XSignal &sig, hipStream_t s) {
    if (sig.n < 1 || sig.n > ONO_MAX_INPUTS) return hipErrorInvalidValue;
    hipLaunchKernelGGL(xsignal_kernel, dim3(1), dim3(64), 0, s, sig);
    return hipGetLastError();
}

hipError_t launch_xgmi_bump(uint64_t *counter, hipStream_t s) {
    hipLaunchKernelGGL(xbump_kernel, dim3(1), dim3(64), 0, s, counter);
    return hipGetLastError();
}

hipError_t launch_xgmi_fence_all(hipStream_t s, bool acquire) {
    if (acquire) hipLaunchKernelGGL(xfence_kernel<true>, dim3(kXFenceBlocks), dim3(64), 0, s);
    else hipLaunchKernelGGL(xfence_kernel<false>, dim3(kXFenceBlocks), dim3(64), 0, s);
    return hipGetLastError();
}

hipError_t launch_xgmi_barrier(const XBarrier &b, hipStream_t s) {
    if (b.n < 1 || b.n > ONO_MAX_INPUTS) return hipErrorInvalidValue;
    hipLaunchKernelGGL(xbarrier_kernel, dim3(1), dim3(64), 0, s, b);
    return hipGetLastError();
}

}  // namespace ono
