// ono_xgmi_pool.cpp — see ono_xgmi_pool.h.  Host-only bookkeeping: every
// device operation goes through XgmiPoolOps (HIP in ono_xgmi.cpp, simulated
// processes in tests/native/xgmi_pool_test.cpp).
#include "ono_xgmi_pool.h"

#include <algorithm>
#include <cstdio>

#include "ono_reduce.h"

namespace ono {

namespace {
std::string hex8(const IpcBytes &h) {
    char b[20];
    snprintf(b, sizeof b, "%02x%02x%02x%02x..", h[0], h[1], h[2], h[3]);
    return b;
}
constexpr int kMaxParkTries = 8;
}  // namespace

int XgmiPool::acquire(int device, size_t bytes, size_t alloc_bytes, uint64_t new_uid, Region *out, bool *fresh,
                      std::string &msg) {
    std::lock_guard<std::mutex> lk(mu_);
    Region *best = nullptr;
    for (auto &r : regions_)
        if (!r.busy && !r.retired && r.device == device && r.bytes >= bytes && (!best || r.bytes < best->bytes))
            best = &r;
    *fresh = best == nullptr;
    if (!best) {
        Region r{};
        r.device = device;
        r.bytes = std::max(alloc_bytes, bytes);
        r.uid = new_uid;
        for (int tries = 0;; tries++) {
            int rc = ops_.alloc(device, r.bytes, &r.ptr, &r.handle, msg);
            if (rc) return rc;
            if (!obtained_.count(r.handle)) break;
            // this handle's bytes were handed out before (the allocator reused an earlier region's memory
            // and the IPC layer named it the same way): a peer importing it could be given its old mapping
            parked_.push_back(r);
            if (tries + 1 >= kMaxParkTries) {
                msg = "xGMI exchange region: " + std::to_string(kMaxParkTries) +
                      " fresh allocations in a row repeated IPC handles handed out before (last " + hex8(r.handle) + ")";
                return ONO_E_HIP;
            }
        }
        obtained_.insert(r.handle);
        regions_.push_back(r);
        best = &regions_.back();
    }
    best->busy = true;
    live_++;
    *out = *best;
    return ONO_OK;
}

void XgmiPool::release_ring(uint8_t *ptr, bool released) {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto &r : regions_)
        if (r.ptr == ptr) {
            if (released) r.busy = false;
            else r.quarantined = true;  // stays busy: never handed to another ring
        }
    live_--;
}

int XgmiPool::map(int device, const IpcBytes &handle, uint64_t uid, size_t bytes, uint8_t **out, std::string &msg) {
    std::lock_guard<std::mutex> lk(mu_);
    for (const auto &m : imports_)
        if (m.device == device && m.uid == uid && m.bytes == bytes) {
            *out = m.ptr;
            return ONO_OK;
        }
    if (opened_.count(handle)) {
        msg = "xGMI connect: a peer's exchange region comes with an IPC handle (" + hex8(handle) +
              ") this process imported before; refusing a possibly stale import";
        return ONO_E_IO;
    }
    uint8_t *p = nullptr;
    int rc = ops_.open(device, handle, &p, msg);
    if (rc) return rc;
    opened_.insert(handle);
    // counted before it is used: the exporter frees the region only once the closes match the opens
    if ((rc = ops_.bump(device, reinterpret_cast<uint64_t *>(p + count_off_), msg))) {
        std::string m2;
        (void)ops_.close(device, p, m2);
        return rc;
    }
    imports_.push_back({device, uid, bytes, p, handle});
    *out = p;
    return ONO_OK;
}

int XgmiPool::close_imports(size_t *closed, std::string &msg) {
    std::lock_guard<std::mutex> lk(mu_);
    if (closed) *closed = 0;
    if (live_ > 0) {
        msg = std::to_string(live_) + " xGMI ring(s) of this process are alive";
        return ONO_E_ARG;
    }
    int rc = ONO_OK;
    size_t n = 0;
    for (auto &m : imports_) {
        std::string m1, m2;
        // the close mark first, through the mapping that is about to go; then the import itself
        int r1 = ops_.bump(m.device, reinterpret_cast<uint64_t *>(m.ptr + count_off_ + 8), m1);
        int r2 = ops_.close(m.device, m.ptr, m2);
        if (rc == ONO_OK && (r1 || r2)) {
            rc = r1 ? r1 : r2;
            msg = r1 ? m1 : m2;
        }
        n++;
    }
    imports_.clear();
    if (closed) *closed = n;
    return rc;
}

int XgmiPool::free_exports(double wait_s, size_t *freed_bytes, size_t *kept, std::string &msg) {
    if (freed_bytes) *freed_bytes = 0;
    if (kept) *kept = 0;
    std::vector<Region> pending;
    {
        std::lock_guard<std::mutex> lk(mu_);
        if (live_ > 0) {
            msg = std::to_string(live_) + " xGMI ring(s) of this process are alive";
            return ONO_E_ARG;
        }
        // the idle regions leave the pool while they are polled (no ring can be handed one); the busy ones
        // here are the quarantined.  Parked allocations stay allocated: freed, the allocator would hand the
        // same blocks (and handles) back to the next fresh allocation.
        std::vector<Region> keep;
        for (auto &r : regions_) (r.busy ? keep : pending).push_back(r);
        regions_.swap(keep);
    }
    // polled without the lock: a peer that never closes costs this caller the wait, not every other call
    int rc = ONO_OK;
    size_t freed = 0;
    std::vector<Region> kept_regions;
    const double t0 = ops_.now();
    for (;;) {
        std::vector<Region> later;
        for (auto &r : pending) {
            uint64_t c[2] = {0, 0};
            std::string m;
            int e = ops_.read2(r.device, reinterpret_cast<const uint64_t *>(r.ptr + count_off_), c, m);
            if (e) {  // cannot tell whether a peer still maps it: keep it
                if (rc == ONO_OK) rc = e, msg = m;
                kept_regions.push_back(r);
            } else if (c[1] >= c[0]) {
                if ((e = ops_.free(r.device, r.ptr, m)) && rc == ONO_OK) rc = e, msg = m;
                freed += r.bytes;
            } else {
                later.push_back(r);
            }
        }
        pending.swap(later);
        if (pending.empty() || ops_.now() - t0 > wait_s) break;
        ops_.pause();
    }
    const size_t still = pending.size();
    for (auto &r : pending) kept_regions.push_back(r);
    {
        std::lock_guard<std::mutex> lk(mu_);
        for (auto &r : kept_regions) {
            r.retired = true;  // its peers may have closed it: never exported to another ring
            regions_.push_back(r);
        }
    }
    if (still && rc == ONO_OK) {
        msg = std::to_string(still) + " exchange region(s) still imported by a peer after " + std::to_string(wait_s) +
              " s: kept (call ono_xgmi_pool_close_imports on every rank first)";
        rc = ONO_E_IO;
    }
    if (freed_bytes) *freed_bytes = freed;
    if (kept) *kept = still;
    return rc;
}

XgmiPool::Stats XgmiPool::stats() {
    std::lock_guard<std::mutex> lk(mu_);
    Stats s{};
    for (const auto &r : regions_) {
        s.regions++;
        s.region_bytes += r.bytes;
        s.quarantined += r.quarantined ? 1 : 0;
    }
    s.imports = imports_.size();
    s.parked = parked_.size();
    return s;
}

int XgmiPool::live() {
    std::lock_guard<std::mutex> lk(mu_);
    return live_;
}

}  // namespace ono
