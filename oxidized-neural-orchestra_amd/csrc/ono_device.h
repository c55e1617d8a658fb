// ono_device.h — device-side helpers shared by the kernel files (not part of
// the ABI): the accesses to memory that other ranks read or write.
#pragma once

#include <hip/hip_runtime.h>

namespace ono {

// Peer HBM (and the exchange slots peers write) is accessed system-coherent:
// volatile accesses compile to sc0 sc1 loads/stores on gfx950, which no cache
// on either GPU keeps, whatever cache policy the IPC import maps the peer's
// region with.  Streaming data gains nothing from caching anyway.
template <class T> __device__ __forceinline__ T ld_sys(const T *p) {
    return *(const volatile __attribute__((address_space(1))) T *)p;  // global_load ... sc0 sc1
}
template <class T> __device__ __forceinline__ void st_sys(T *p, T v) {
    *(volatile __attribute__((address_space(1))) T *)p = v;  // global_store ... sc0 sc1
}

// The same system-coherent 16-byte store without the volatile semantics: the
// compiler waits for every volatile store to complete before the next memory
// operation (`s_waitcnt vmcnt(0)` after each), which keeps a remote round
// trip per store on the wave's critical path; this one is waited for once, by
// peer_stores_done() at the end of the wave.  Vector store (no scalar-cache
// write); `s_nop 1` covers the gfx940+ store-data hazard the compiler cannot
// see through the asm (as st_sc1 in ono_kernels.hip).
typedef float f4_dev __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_sys_async(f4_dev *p, f4_dev v) {
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" : : "v"(p), "v"(v) : "memory");
}

// Publication of stores other ranks read after a flag barrier.
//
// The barrier is a later launch on the same stream: its first lane runs a
// system-scope release fence, then stores the round's epoch into every peer's
// flag slot (system-scope release store); a peer spins on its own slot with
// system-scope acquire loads and only then launches the kernel that reads
// what we wrote.  That release orders memory operations the *barrier* wave
// issued or that are already complete — it cannot wait for stores a retired
// wave of an earlier launch left in flight: on gfx950 a wave may reach
// s_endpgm with vector stores outstanding (vmcnt > 0), and the end-of-kernel
// release only covers the agent scope, not stores bound over xGMI to another
// device's (or process's) memory.  So every wave that writes such memory
// waits for its own stores to be acknowledged before it ends.  The stores are
// sc0 sc1 (system scope, write-through to the memory side: uncached exchange
// regions, peer HBM), so their acknowledgement means they have reached the
// point of system coherence; the chain is then
//   writer wave: st_sys ...; s_waitcnt vmcnt(0); s_endpgm
//   -> stream order -> barrier: fence(release, system); flag store (release, system)
//   -> reader barrier: flag load (acquire, system) -> stream order -> reader kernel loads.
// Without the wait the pipelined host-fed xGMI test failed about one run in
// two (an owner chain read a receive slot before the pushed slice landed).
// A system-scope release fence per wave instead (an L2 writeback each) was
// also correct but made rounds 25x slower.  tests/test_isa.py checks in the
// built code object that every kernel with sc0 sc1 stores waits with
// vmcnt(0) after its last such store.
__device__ __forceinline__ void peer_stores_done() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores acknowledged
}

}  // namespace ono
