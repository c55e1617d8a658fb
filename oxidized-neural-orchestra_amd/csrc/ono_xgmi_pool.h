// ono_xgmi_pool.h — the process's exchange regions and peer imports (host
// bookkeeping of the xGMI schedule; no HIP here, so the CPU suite can drive it
// with simulated processes: tests/native/xgmi_pool_test.cpp).
//
// What it enforces (DESIGN.md §4 "Retention" and §8):
//   * regions are pooled: a destroyed ring's region serves the next ring that
//     fits; a new one is allocated only when none does;
//   * no IPC handle is handed out twice: a fresh allocation whose handle bytes
//     repeat any handle this process obtained before is parked (kept
//     allocated for the life of the process, never exported — freeing it would
//     hand the allocator the same block back, so every release cycle would need
//     one more discarded allocation than the last) and another is allocated —
//     round 3 traced a wrong result to a re-import whose handle repeated an
//     earlier one;
//   * an importer never opens a handle whose bytes it opened before (the same
//     hazard from the other side: ONO_E_IO instead of a stale mapping);
//   * release is two-phase.  close_imports (every rank) marks each peer region
//     it maps as closed — a system-scope add to that region's close counter —
//     and closes the import; then, after a collective step, free_exports
//     (every rank) frees a region only once its close counter has caught up
//     with its open counter (every importer bumped the open counter when it
//     mapped the region), waiting a bounded time without holding the pool's
//     lock; a region some peer still maps is kept — never freed under it,
//     never handed to a later ring (its peers may have closed it), retried by
//     the next free_exports;
//   * a ring's liveness count moves only for rings that obtained a region, so
//     an allocation that failed cannot let a release free a region in use.
#pragma once

#include <array>
#include <cstddef>
#include <cstdint>
#include <functional>
#include <mutex>
#include <set>
#include <string>
#include <vector>

namespace ono {

using IpcBytes = std::array<uint8_t, 64>;

// The device operations the bookkeeping drives.  Each returns 0 or an ONO_E_*
// code and may fill msg.
struct XgmiPoolOps {
    // allocate `bytes` of exchange memory (uncached HBM) on `device` and get its IPC handle
    std::function<int(int device, size_t bytes, uint8_t **ptr, IpcBytes *handle, std::string &msg)> alloc;
    std::function<int(int device, uint8_t *ptr, std::string &msg)> free;
    std::function<int(int device, const IpcBytes &handle, uint8_t **ptr, std::string &msg)> open;
    std::function<int(int device, uint8_t *ptr, std::string &msg)> close;
    // system-scope atomic add of 1 to the u64 at p (p inside a peer region as mapped here), completed on return
    std::function<int(int device, uint64_t *p, std::string &msg)> bump;
    // the two u64 words at p (inside a region this process owns), as they have landed in memory
    std::function<int(int device, const uint64_t *p, uint64_t out[2], std::string &msg)> read2;
    std::function<void()> pause;  // between polls
    std::function<double()> now;  // seconds, monotonic
};

class XgmiPool {
public:
    struct Region {
        int device;
        uint8_t *ptr;
        size_t bytes;
        uint64_t uid;
        IpcBytes handle;
        bool busy;         // a ring uses it
        bool quarantined;  // a ring's teardown ended without every peer's marker: never reused, never freed
        bool retired;      // a free_exports found it still imported: never reused, freed by a later free_exports
    };
    struct Import {
        int device;
        uint64_t uid;
        size_t bytes;
        uint8_t *ptr;
        IpcBytes handle;
    };
    struct Stats {
        size_t regions, region_bytes, quarantined, imports, parked;
    };

    // count_off: byte offset, inside every region, of its two u64 counters {opens, closes}
    XgmiPool(XgmiPoolOps ops, size_t count_off) : ops_(std::move(ops)), count_off_(count_off) {}

    // A region of >= bytes for a ring on `device`: the smallest idle pooled one, else a fresh allocation of
    // alloc_bytes with an IPC handle this process never obtained before (uid = new_uid).  *fresh tells
    // which.  Counts the ring as alive on success only.
    int acquire(int device, size_t bytes, size_t alloc_bytes, uint64_t new_uid, Region *out, bool *fresh,
                std::string &msg);
    // The ring that held `ptr` is gone: the region back to the pool (released) or into quarantine.
    void release_ring(uint8_t *ptr, bool released);
    // Peer region `uid` as mapped here: the mapping made for an earlier ring, else a new import (its
    // open counter bumped).  A new import whose handle bytes this process opened before is refused.
    int map(int device, const IpcBytes &handle, uint64_t uid, size_t bytes, uint8_t **out, std::string &msg);
    // Release, phase 1: every import marked closed in its region, then closed.  Refused while a ring lives.
    int close_imports(size_t *closed, std::string &msg);
    // Release, phase 2: every idle region freed once its importers have all closed it (polls up to
    // wait_s, the lock released in between).  Regions still imported after the wait are kept and
    // retired (ONO_E_IO, *kept).  Parked allocations stay.  Refused while a ring lives.
    int free_exports(double wait_s, size_t *freed_bytes, size_t *kept, std::string &msg);
    Stats stats();
    int live();

private:
    XgmiPoolOps ops_;
    size_t count_off_;
    std::mutex mu_;
    std::vector<Region> regions_;
    std::vector<Region> parked_;  // fresh allocations whose handle repeated an earlier one
    std::vector<Import> imports_;
    std::set<IpcBytes> obtained_;  // every IPC handle this process's allocations got
    std::set<IpcBytes> opened_;    // every IPC handle this process imported
    int live_ = 0;
};

}  // namespace ono
