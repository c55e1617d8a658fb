// xgmi_pool_test.cpp (TEST INFRASTRUCTURE, CPU only) — the xGMI exchange-region
// pool's bookkeeping (csrc/ono_xgmi_pool.{h,cpp}) driven by simulated
// processes over one simulated device, no HIP:
//   * a fresh allocation whose IPC handle repeats one obtained before is parked
//     and another is allocated; an import of a handle opened before is refused;
//   * the release order: no region is ever freed while an import of it is open
//     (the simulated device counts open imports per region and records every
//     free that happens under one), the two phases free everything, a phase 2
//     that runs before a peer's phase 1 keeps the region (ONO_E_IO) and frees
//     it on the next call;
//   * liveness: a failed allocation does not count as a live ring (round 4's
//     g_live underflow), release is refused while a ring lives.
// Prints "ok <checks>" and exits 0, or the first failures and exits 1.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "ono_reduce.h"
#include "ono_xgmi_pool.h"

using namespace ono;

namespace {

int g_checks = 0, g_fail = 0;
#define CHECK(cond, ...)                                              \
    do {                                                              \
        g_checks++;                                                   \
        if (!(cond)) {                                                \
            g_fail++;                                                 \
            fprintf(stderr, "FAIL %s:%d %s: ", __FILE__, __LINE__, #cond); \
            fprintf(stderr, __VA_ARGS__);                             \
            fprintf(stderr, "\n");                                    \
        }                                                             \
    } while (0)

constexpr size_t kCountOff = 3072;

// One device shared by every simulated process: allocations are host memory,
// an import maps the same bytes (as an IPC import of one device does).
struct Device {
    struct Alloc {
        std::unique_ptr<uint8_t[]> mem;
        size_t bytes;
        IpcBytes handle;
        int open_imports = 0;
        bool freed = false;
        int owner = 0;  // the simulated process that allocated it (each process has its own allocator)
    };
    std::vector<std::unique_ptr<Alloc>> allocs;
    std::vector<IpcBytes> next_handles;  // handles the next allocations get (then fresh ones)
    uint8_t fresh_counter = 1;
    int fail_next_alloc = 0;
    int frees_under_import = 0;
    double clock = 0;
    // lifo: an allocation takes the most recently freed block that fits, with the handle it had (the
    // deterministic reuse ADVICE r5 describes: every freed block comes back, named as before)
    bool lifo = false;
    int procs = 0;
    std::vector<Alloc *> free_list;
    std::function<void()> on_pause;  // (called between free_exports' polls)

    Alloc *by_ptr(const uint8_t *p) {
        for (auto &a : allocs)
            if (p >= a->mem.get() && p < a->mem.get() + a->bytes) return a.get();
        return nullptr;
    }
    Alloc *by_handle(const IpcBytes &h) {
        Alloc *last = nullptr;  // the newest allocation named so (a repeated handle names the newest)
        for (auto &a : allocs)
            if (!a->freed && a->handle == h) last = a.get();
        return last;
    }
};

IpcBytes handle_of(uint8_t tag) {
    IpcBytes h{};
    h[0] = 0xAB;
    h[1] = tag;
    return h;
}

XgmiPoolOps ops_for(Device &d, int owner) {
    XgmiPoolOps o;
    o.alloc = [&d, owner](int, size_t bytes, uint8_t **ptr, IpcBytes *h, std::string &msg) -> int {
        if (d.fail_next_alloc > 0) {
            d.fail_next_alloc--;
            msg = "simulated allocation failure";
            return ONO_E_HIP;
        }
        if (d.lifo)
            for (size_t k = d.free_list.size(); k-- > 0;)
                if (d.free_list[k]->owner == owner && d.free_list[k]->bytes >= bytes) {
                    Device::Alloc *b = d.free_list[k];
                    d.free_list.erase(d.free_list.begin() + (long)k);
                    b->freed = false;
                    std::memset(b->mem.get(), 0, b->bytes);
                    *ptr = b->mem.get();
                    *h = b->handle;
                    return ONO_OK;
                }
        auto a = std::make_unique<Device::Alloc>();
        a->mem.reset(new uint8_t[bytes]());
        a->bytes = bytes;
        a->owner = owner;
        if (!d.next_handles.empty()) {
            a->handle = d.next_handles.front();
            d.next_handles.erase(d.next_handles.begin());
        } else {
            a->handle = handle_of((uint8_t)(0x80 + d.fresh_counter++));
        }
        *ptr = a->mem.get();
        *h = a->handle;
        d.allocs.push_back(std::move(a));
        return ONO_OK;
    };
    o.free = [&d](int, uint8_t *ptr, std::string &msg) -> int {
        Device::Alloc *a = d.by_ptr(ptr);
        if (!a || a->freed) {
            msg = "free of an unknown region";
            return ONO_E_HIP;
        }
        if (a->open_imports > 0) d.frees_under_import++;
        a->freed = true;
        d.free_list.push_back(a);
        return ONO_OK;
    };
    o.open = [&d](int, const IpcBytes &h, uint8_t **ptr, std::string &msg) -> int {
        Device::Alloc *a = d.by_handle(h);
        if (!a) {
            msg = "open of an unknown handle";
            return ONO_E_HIP;
        }
        a->open_imports++;
        *ptr = a->mem.get();
        return ONO_OK;
    };
    o.close = [&d](int, uint8_t *ptr, std::string &msg) -> int {
        Device::Alloc *a = d.by_ptr(ptr);
        if (!a || a->open_imports <= 0) {
            msg = "close of an import that is not open";
            return ONO_E_HIP;
        }
        a->open_imports--;
        return ONO_OK;
    };
    o.bump = [](int, uint64_t *p, std::string &) -> int {
        (*p)++;
        return ONO_OK;
    };
    o.read2 = [](int, const uint64_t *p, uint64_t out[2], std::string &) -> int {
        out[0] = p[0];
        out[1] = p[1];
        return ONO_OK;
    };
    o.pause = [&d] {
        d.clock += 0.001;
        if (d.on_pause) d.on_pause();
    };
    o.now = [&d] { return d.clock; };
    return o;
}

struct Proc {
    XgmiPool pool;
    XgmiPool::Region reg{};
    explicit Proc(Device &d) : pool(ops_for(d, ++d.procs), kCountOff) {}
};

// n processes each create one ring region and map every peer's (connect); then all rings are destroyed
void rings(std::vector<std::unique_ptr<Proc>> &ps, size_t bytes, uint64_t uid0) {
    std::string msg;
    for (size_t i = 0; i < ps.size(); i++) {
        bool fresh = false;
        int rc = ps[i]->pool.acquire(0, bytes, bytes, uid0 + i, &ps[i]->reg, &fresh, msg);
        CHECK(rc == ONO_OK, "acquire: %s", msg.c_str());
    }
    for (size_t i = 0; i < ps.size(); i++)
        for (size_t j = 0; j < ps.size(); j++) {
            if (i == j) continue;
            uint8_t *p = nullptr;
            int rc = ps[i]->pool.map(0, ps[j]->reg.handle, ps[j]->reg.uid, ps[j]->reg.bytes, &p, msg);
            CHECK(rc == ONO_OK && p == ps[j]->reg.ptr, "map: %s", msg.c_str());
        }
    for (auto &p : ps) p->pool.release_ring(p->reg.ptr, true);
}

void test_two_phase_release() {
    Device d;
    std::vector<std::unique_ptr<Proc>> ps;
    for (int i = 0; i < 3; i++) ps.push_back(std::make_unique<Proc>(d));
    rings(ps, 8192, 100);
    rings(ps, 8192, 200);  // pooled regions and imports reused: no new import, no new allocation
    CHECK(d.allocs.size() == 3, "%zu allocations for two rings of three processes", d.allocs.size());
    for (auto &p : ps) {
        const uint64_t *c = reinterpret_cast<const uint64_t *>(p->reg.ptr + kCountOff);
        CHECK(c[0] == 2 && c[1] == 0, "opens %llu closes %llu (2 peers mapped it once each)",
              (unsigned long long)c[0], (unsigned long long)c[1]);
    }
    std::string msg;
    for (auto &p : ps) {  // phase 1 everywhere
        size_t closed = 0;
        CHECK(p->pool.close_imports(&closed, msg) == ONO_OK && closed == 2, "close_imports: %s", msg.c_str());
    }
    for (auto &p : ps) {  // (collective step) then phase 2 everywhere
        size_t freed = 0, kept = 9;
        CHECK(p->pool.free_exports(0.0, &freed, &kept, msg) == ONO_OK && freed == 8192 && kept == 0,
              "free_exports: %s", msg.c_str());
        XgmiPool::Stats st = p->pool.stats();
        CHECK(st.regions == 0 && st.imports == 0, "after release: %zu regions %zu imports", st.regions, st.imports);
    }
    CHECK(d.frees_under_import == 0, "%d regions freed while imported", d.frees_under_import);
}

void test_free_before_peer_closes_is_kept() {
    Device d;
    std::vector<std::unique_ptr<Proc>> ps;
    for (int i = 0; i < 2; i++) ps.push_back(std::make_unique<Proc>(d));
    rings(ps, 4096, 300);
    std::string msg;
    size_t closed = 0, freed = 0, kept = 0;
    CHECK(ps[0]->pool.close_imports(&closed, msg) == ONO_OK, "%s", msg.c_str());
    // rank 0 frees before rank 1 has closed its import of rank 0's region: refused, kept, nothing freed
    const double t0 = d.clock;
    int rc = ps[0]->pool.free_exports(0.05, &freed, &kept, msg);
    CHECK(rc == ONO_E_IO && kept == 1 && freed == 0, "rc %d kept %zu freed %zu", rc, kept, freed);
    CHECK(d.clock - t0 >= 0.05, "free_exports did not wait (%.3f s)", d.clock - t0);
    CHECK(ps[0]->pool.stats().regions == 1, "the kept region left the pool");
    CHECK(ps[1]->pool.close_imports(&closed, msg) == ONO_OK, "%s", msg.c_str());
    CHECK(ps[0]->pool.free_exports(0.0, &freed, &kept, msg) == ONO_OK && freed == 4096 && kept == 0,
          "second free_exports: %s", msg.c_str());
    CHECK(ps[1]->pool.free_exports(0.0, &freed, &kept, msg) == ONO_OK && freed == 4096, "%s", msg.c_str());
    CHECK(d.frees_under_import == 0, "%d regions freed while imported", d.frees_under_import);
}

void test_repeated_handles() {
    Device d;
    std::vector<std::unique_ptr<Proc>> ps;
    for (int i = 0; i < 2; i++) ps.push_back(std::make_unique<Proc>(d));
    d.next_handles = {handle_of(1), handle_of(2)};
    rings(ps, 4096, 400);
    std::string msg;
    size_t closed, freed, kept;
    for (auto &p : ps) p->pool.close_imports(&closed, msg);
    for (auto &p : ps) p->pool.free_exports(0.0, &freed, &kept, msg);
    // the allocator now hands rank 0 its old handle again, then a fresh one
    d.next_handles = {handle_of(1), handle_of(3), handle_of(4)};
    bool fresh = false;
    XgmiPool::Region r0{}, r1{};
    CHECK(ps[0]->pool.acquire(0, 4096, 4096, 500, &r0, &fresh, msg) == ONO_OK, "%s", msg.c_str());
    CHECK(r0.handle == handle_of(3), "rank 0 got handle %02x, not the fresh 03", r0.handle[1]);
    CHECK(ps[0]->pool.stats().parked == 1, "the repeated allocation was not parked");
    CHECK(ps[1]->pool.acquire(0, 4096, 4096, 501, &r1, &fresh, msg) == ONO_OK && r1.handle == handle_of(4), "%s",
          msg.c_str());
    uint8_t *p = nullptr;
    CHECK(ps[1]->pool.map(0, r0.handle, r0.uid, r0.bytes, &p, msg) == ONO_OK, "%s", msg.c_str());
    // an importer never re-opens a handle it opened before (here: rank 0's first handle, seen by rank 1)
    int rc = ps[1]->pool.map(0, handle_of(1), 999, 4096, &p, msg);
    CHECK(rc == ONO_E_IO, "re-import of a handle opened before: rc %d", rc);
    // eight repeats in a row: refused (ONO_E_HIP), every repeated allocation parked
    d.next_handles.assign(8, handle_of(3));
    rc = ps[0]->pool.acquire(0, 1 << 20, 1 << 20, 502, &r0, &fresh, msg);
    CHECK(rc == ONO_E_HIP && ps[0]->pool.stats().parked == 9, "rc %d parked %zu", rc, ps[0]->pool.stats().parked);
    ps[0]->pool.release_ring(r0.ptr, true);  // (the first acquire's ring)
    ps[1]->pool.release_ring(r1.ptr, true);
    for (auto &q : ps) q->pool.close_imports(&closed, msg);
    // parked allocations stay allocated (freed, the allocator would hand the same blocks back)
    CHECK(ps[0]->pool.free_exports(0.0, &freed, &kept, msg) == ONO_OK && ps[0]->pool.stats().parked == 9,
          "parked allocations freed: %s (%zu parked)", msg.c_str(), ps[0]->pool.stats().parked);
}

// an allocator that reuses every freed block in LIFO order, handle and all.  Over 12 release
// cycles every ring still gets a region whose handle was never handed out before (at most one repeat per
// cycle: the parked blocks stay out of the allocator), no region is freed while imported, and the pool
// holds at most one parked block per cycle.
void test_release_cycles_lifo() {
    Device d;
    d.lifo = true;
    std::vector<std::unique_ptr<Proc>> ps;
    for (int i = 0; i < 3; i++) ps.push_back(std::make_unique<Proc>(d));
    std::string msg;
    std::set<IpcBytes> seen;
    for (int cycle = 0; cycle < 12; cycle++) {
        std::vector<IpcBytes> got;
        for (size_t i = 0; i < ps.size(); i++) {
            bool fresh = false;
            int rc = ps[i]->pool.acquire(0, 8192, 8192, 1000 + 10 * (uint64_t)cycle + i, &ps[i]->reg, &fresh, msg);
            CHECK(rc == ONO_OK && fresh, "cycle %d rank %zu acquire: rc %d %s", cycle, i, rc, msg.c_str());
            if (rc) return;
            CHECK(!seen.count(ps[i]->reg.handle), "cycle %d rank %zu: a handle handed out before", cycle, i);
            got.push_back(ps[i]->reg.handle);
        }
        for (auto &h : got) seen.insert(h);
        for (size_t i = 0; i < ps.size(); i++)
            for (size_t j = 0; j < ps.size(); j++) {
                if (i == j) continue;
                uint8_t *p = nullptr;
                int rc = ps[i]->pool.map(0, ps[j]->reg.handle, ps[j]->reg.uid, ps[j]->reg.bytes, &p, msg);
                CHECK(rc == ONO_OK && p == ps[j]->reg.ptr, "cycle %d map: %s", cycle, msg.c_str());
            }
        for (auto &p : ps) p->pool.release_ring(p->reg.ptr, true);
        size_t closed, freed, kept;
        for (auto &p : ps) CHECK(p->pool.close_imports(&closed, msg) == ONO_OK, "%s", msg.c_str());
        for (auto &p : ps)
            CHECK(p->pool.free_exports(0.0, &freed, &kept, msg) == ONO_OK && freed == 8192, "cycle %d free: %s",
                  cycle, msg.c_str());
    }
    size_t parked = 0;
    for (auto &p : ps) parked += p->pool.stats().parked;
    // every cycle after the first: the freed block came back first (one repeat, parked) — the case exercised
    CHECK(parked == 11 * ps.size(), "%zu parked blocks after 12 cycles of 3 processes", parked);
    CHECK(d.frees_under_import == 0, "%d regions freed while imported", d.frees_under_import);
}

// free_exports waits for a peer without holding the pool's lock: during its polls the same pool
// answers stats() and hands a new ring a region; the region it gave up on is kept, retired (not handed out),
// and freed by the next free_exports once the peer has closed.
void test_free_exports_polls_unlocked() {
    Device d;
    std::vector<std::unique_ptr<Proc>> ps;
    for (int i = 0; i < 2; i++) ps.push_back(std::make_unique<Proc>(d));
    rings(ps, 4096, 700);
    std::string msg;
    size_t closed = 0, freed = 0, kept = 0;
    CHECK(ps[0]->pool.close_imports(&closed, msg) == ONO_OK, "%s", msg.c_str());
    int polls = 0, acquired = 0;
    XgmiPool::Region other{};
    d.on_pause = [&] {
        polls++;
        (void)ps[0]->pool.stats();  // would deadlock if free_exports held the lock
        if (polls == 3) {
            bool fresh = false;
            std::string m;
            if (ps[0]->pool.acquire(0, 4096, 4096, 777, &other, &fresh, m) == ONO_OK) acquired = fresh ? 1 : -1;
        }
    };
    int rc = ps[0]->pool.free_exports(0.01, &freed, &kept, msg);
    d.on_pause = nullptr;
    CHECK(rc == ONO_E_IO && kept == 1 && polls >= 3, "rc %d kept %zu polls %d", rc, kept, polls);
    CHECK(acquired == 1 && other.ptr != ps[0]->reg.ptr, "acquire during the polls: %d", acquired);
    ps[0]->pool.release_ring(other.ptr, true);
    XgmiPool::Region again{};
    bool fresh = false;
    CHECK(ps[0]->pool.acquire(0, 4096, 4096, 778, &again, &fresh, msg) == ONO_OK && again.ptr != ps[0]->reg.ptr,
          "the kept region was handed to another ring");
    ps[0]->pool.release_ring(again.ptr, true);
    CHECK(ps[1]->pool.close_imports(&closed, msg) == ONO_OK, "%s", msg.c_str());
    CHECK(ps[0]->pool.free_exports(0.0, &freed, &kept, msg) == ONO_OK && kept == 0 && freed >= 4096,
          "the retired region was not freed once closed: %s", msg.c_str());
    CHECK(d.frees_under_import == 0, "%d regions freed while imported", d.frees_under_import);
}

void test_liveness() {
    Device d;
    Proc p(d);
    std::string msg;
    d.fail_next_alloc = 1;
    XgmiPool::Region r{};
    bool fresh = false;
    CHECK(p.pool.acquire(0, 4096, 4096, 1, &r, &fresh, msg) == ONO_E_HIP, "failed allocation reported");
    CHECK(p.pool.live() == 0, "a failed allocation counts as a live ring (%d)", p.pool.live());
    CHECK(p.pool.acquire(0, 4096, 4096, 2, &r, &fresh, msg) == ONO_OK && p.pool.live() == 1, "%s", msg.c_str());
    size_t closed, freed, kept;
    CHECK(p.pool.close_imports(&closed, msg) == ONO_E_ARG, "close_imports while a ring lives");
    CHECK(p.pool.free_exports(0.0, &freed, &kept, msg) == ONO_E_ARG, "free_exports while a ring lives");
    p.pool.release_ring(r.ptr, false);  // teardown without every peer's marker: quarantined
    CHECK(p.pool.live() == 0 && p.pool.stats().quarantined == 1, "quarantine");
    CHECK(p.pool.free_exports(0.0, &freed, &kept, msg) == ONO_OK && freed == 0 && p.pool.stats().regions == 1,
          "a quarantined region was freed");
    XgmiPool::Region r2{};
    CHECK(p.pool.acquire(0, 4096, 4096, 3, &r2, &fresh, msg) == ONO_OK && fresh && r2.ptr != r.ptr,
          "a quarantined region was handed out again");
    p.pool.release_ring(r2.ptr, true);
}

}  // namespace

int main() {
    test_two_phase_release();
    test_free_before_peer_closes_is_kept();
    test_repeated_handles();
    test_liveness();
    test_release_cycles_lifo();
    test_free_exports_polls_unlocked();
    if (g_fail) {
        fprintf(stderr, "%d of %d checks failed\n", g_fail, g_checks);
        return 1;
    }
    printf("ok %d\n", g_checks);
    return 0;
}
