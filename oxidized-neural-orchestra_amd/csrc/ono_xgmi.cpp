// ono_xgmi.cpp — the xGMI peer-access schedule of the ring (ONO_ALGO_XGMI).
//
// The same round as the direct schedule (worker_ring.rs:112-204 restated as
// "every slice of chunk c reaches its owner, the owner replays the hop chain
// c, c+1, ..., c+n-1, the result goes back to everyone"), but with no
// collective library in the data path: every rank exports one exchange region
// of uncached HBM (IPC), maps its peers' regions, and the kernels move the
// bytes with vector loads and stores over the node's xGMI links:
//
//   1. push     for every peer q: my slice of q's chunk -> q.rbuf[k], my slice
//               zeroed in the same pass (k = my place in that chunk's chain)
//   2. barrier  all slices have landed
//   3. owner    DirectOp: grad[c] = chain(rbuf[0..n-2], own slice) / n, own
//               slice zeroed, the result (f32 wire: grad[c]; f16 wire: the
//               f16 message the reference forwards) into my obuf
//   4. barrier  all owners' results are ready
//   5. pull     for every peer q: grad[chunk of q] = dec(q.obuf) (/ n for f16)
//
// Gather variant (env ONO_XGMI_GATHER=push, read when the region is made):
// step 3 also stores the owner's result into every peer's gather slot over
// xGMI (remote writes instead of remote reads), and step 5 unpacks the local
// gather slots.  Same bytes on the links, one extra local pass; which one the
// links prefer is measured by bench.py at N > 1.
//
// Bit-exact with the reference hop order for both wires (the chain is the
// direct schedule's, tested against the oracle).  Bytes per rank on the links:
// (n-1)/n 4N out in step 1, (n-1)/n 4N (f32) or 2N (f16) in step 5, all n-1
// links at once.  No stream synchronisation or host round trip per round: the
// barriers are device-side flag exchanges with a timeout.
//
// Connect is verified, teardown is ordered, and no exchange region is freed
// or unmapped while a ring of the process is alive (round 3; round 4 adds the
// explicit ono_xgmi_pool_release for when none is).  Every region carries a
// random 64-bit ring id, stamped at the start of every 4 KiB page before its
// handle leaves the process; the handle blob (ONO_XGMI_HANDLE_BYTES) holds the
// IPC handle, the ring id, the layout's size and a per-region uid.  An
// importer reads every page's stamp through its mapping before the first
// round (a device barrier at the end of connect keeps every rank from writing
// a peer region until all importers have checked): a mapping that shows
// another region's memory is an ONO_E_IO at connect time.  That check is what
// found the cause of round 2's one wrong host-fed result: with regions freed
// at destroy and re-imported by the next ring of the same processes, the HIP
// IPC path on this image handed out mappings with a few pages (9 of 1,026 in
// the recorded case) still backed by an earlier region's memory — after the
// exporter's new IPC handle had repeated the bytes of one it had exported
// before (the test logs the repeats).  So regions are pooled per process: a
// destroyed ring's region (flags reset, re-stamped) serves the next ring that
// fits in it, a new one is allocated only when none fits, and importers keep
// every peer region they mapped (keyed by its uid) for reuse instead of
// closing it — no handle, virtual address or mapping is recycled while rings
// come and go.  A region whose teardown ended without every peer's marker
// (timeout, abort) is quarantined: never reset for another ring, never freed.
// ono_xgmi_pool_release frees the idle regions and closes every import once no
// ring of the process is alive (collectively, on every rank, so that the
// peers' imports stop pinning the freed HBM); a ring created after it exports
// and imports fresh regions, which the page check verifies as always.
// Destroy stays collective: each rank, once its own work is done, stores the
// owner's id into a teardown slot of every peer region it mapped; an owner
// returns its region to the pool only when every peer's marker is there (or
// the timeout passed), so a region is never reset while a peer still uses it.
//
// Reuse safety without a third barrier: a rank writes peer q's rbuf in round
// r+1 only after passing barrier 4 of round r, which q reaches after its step 3
// (the only reader of its rbuf); it overwrites its own obuf (round r+1 step 3)
// only after barrier 2 of round r+1, which every peer reaches after its round-r
// step 5 (the only remote reader of obuf).
#include <hip/hip_runtime.h>

#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <mutex>
#include <cstring>
#include <random>
#include <thread>

#include "ono_internal.h"
#include "ono_ring_impl.h"
#include "ono_xgmi_pool.h"

static_assert(sizeof(hipIpcMemHandle_t) == 64, "IPC handle size");

namespace ono {

constexpr size_t kFlagBytes = 4096;  // flag page: barrier slots (n x u64) at offset 0,
constexpr size_t kDoneOff = 1024;    //   teardown markers (n x u64),
constexpr size_t kIdOff = 2048;      //   the region's ring id,
constexpr size_t kCountOff = 3072;   //   {opens, closes} of the region's peer imports (ono_xgmi_pool.h)
constexpr size_t kPage = 4096;       // every later page starts with the id until the first round
// the handle blob: [hipIpcMemHandle_t (64 B)][u64 ring id][u64 layout bytes][u64 region uid][u64 region
// alloc bytes][zero to ONO_XGMI_HANDLE_BYTES]
constexpr size_t kBlobId = sizeof(hipIpcMemHandle_t), kBlobBytes = kBlobId + 8, kBlobUid = kBlobBytes + 8,
                 kBlobAlloc = kBlobUid + 8;
static_assert(kBlobAlloc + 8 <= ONO_XGMI_HANDLE_BYTES, "handle blob layout");

struct XgmiState {
    uint8_t *xbuf = nullptr;          // this rank's exchange region (uncached HBM, exported)
    size_t slot = 0;                  // elements per receive slot (multiple of 64: 256-B aligned slots)
    size_t obuf_off = 0;              // byte offset of the owner's result buffer
    bool push_gather = false;         // env ONO_XGMI_GATHER=push: owners store results into peers' gather slots
    size_t gat_off = 0;               // byte offset of the n-1 gather slots (push_gather only)
    std::vector<uint8_t *> peer;      // every rank's region as mapped here (peer[pos] = xbuf)
    bool connected = false;
    uint64_t epoch = 0;               // barriers issued so far (the same sequence on every rank)
    uint32_t *err = nullptr;          // host-mapped: set by a barrier that timed out
    uint32_t *err_dev = nullptr;
    uint64_t timeout_ticks = 0;
    double timeout_s = 0;
    std::vector<hipEvent_t> ev;       // host-fed sub-round pipeline: H2D / round / D2H per sub-round
    float *hin = nullptr;             // host-fed input staging (pinned, mapped): two slots of n pieces
    float *hin_dev = nullptr;         // the same as the kernels address it
    size_t hin_elems = 0;
    uint64_t id = 0;                  // this ring's id (stamped into the region, sent in the handle blob)
    size_t bytes = 0;                 // the layout's size (every rank of the ring computes the same)
    size_t alloc = 0;                 // the pooled region's size (>= bytes)
    uint64_t uid = 0;                 // the pooled region's uid
    hipIpcMemHandle_t handle{};       // its IPC handle
    bool exported = false;            // the handle left this process (a peer may have mapped the region)
    bool counted = false;             // holds a pooled region (counted among the process's live rings)
    std::vector<uint64_t> peer_id;    // every peer region's id, from its blob
};

// The process's exchange regions and peer imports (ono_xgmi_pool.h) over the
// HIP runtime.
XgmiPool &pool() {
    static XgmiPool *p = [] {
        XgmiPoolOps o;
        o.alloc = [](int dev, size_t bytes, uint8_t **ptr, IpcBytes *h, std::string &msg) -> int {
            DeviceGuard g(dev);
            hipError_t e = hipExtMallocWithFlags((void **)ptr, bytes, hipDeviceMallocUncached);
            if (e != hipSuccess) {
                msg = std::string("hipExtMallocWithFlags (exchange region): ") + hipGetErrorString(e);
                return ONO_E_HIP;
            }
            hipIpcMemHandle_t ih;
            if ((e = hipIpcGetMemHandle(&ih, *ptr)) != hipSuccess) {
                (void)hipFree(*ptr);
                msg = std::string("hipIpcGetMemHandle (exchange region): ") + hipGetErrorString(e);
                return ONO_E_HIP;
            }
            memcpy(h->data(), &ih, sizeof ih);
            return ONO_OK;
        };
        o.free = [](int dev, uint8_t *ptr, std::string &msg) -> int {
            DeviceGuard g(dev);
            hipError_t e = hipFree(ptr);
            if (e != hipSuccess) msg = std::string("hipFree (pooled exchange region): ") + hipGetErrorString(e);
            return e == hipSuccess ? ONO_OK : ONO_E_HIP;
        };
        o.open = [](int dev, const IpcBytes &h, uint8_t **ptr, std::string &msg) -> int {
            DeviceGuard g(dev);
            hipIpcMemHandle_t ih;
            memcpy(&ih, h.data(), sizeof ih);
            hipError_t e = hipIpcOpenMemHandle((void **)ptr, ih, hipIpcMemLazyEnablePeerAccess);
            if (e != hipSuccess) msg = std::string("hipIpcOpenMemHandle (peer exchange region): ") + hipGetErrorString(e);
            return e == hipSuccess ? ONO_OK : ONO_E_HIP;
        };
        o.close = [](int dev, uint8_t *ptr, std::string &msg) -> int {
            DeviceGuard g(dev);
            hipError_t e = hipIpcCloseMemHandle(ptr);
            if (e != hipSuccess) msg = std::string("hipIpcCloseMemHandle (peer region): ") + hipGetErrorString(e);
            return e == hipSuccess ? ONO_OK : ONO_E_HIP;
        };
        o.bump = [](int dev, uint64_t *c, std::string &msg) -> int {
            DeviceGuard g(dev);
            hipError_t e = launch_xgmi_bump(c, nullptr);
            if (e == hipSuccess) e = hipStreamSynchronize(nullptr);
            if (e != hipSuccess) msg = std::string("exchange region import count: ") + hipGetErrorString(e);
            return e == hipSuccess ? ONO_OK : ONO_E_HIP;
        };
        o.read2 = [](int dev, const uint64_t *c, uint64_t out[2], std::string &msg) -> int {
            DeviceGuard g(dev);  // uncached region: a copy reads what has landed
            hipError_t e = hipMemcpy(out, c, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost);
            if (e != hipSuccess) msg = std::string("exchange region import count: ") + hipGetErrorString(e);
            return e == hipSuccess ? ONO_OK : ONO_E_HIP;
        };
        o.pause = [] { std::this_thread::sleep_for(std::chrono::microseconds(200)); };
        o.now = [] {
            return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
        };
        return new XgmiPool(std::move(o), kCountOff);  // (never destroyed: regions outlive static destructors)
    }();
    return *p;
}

// The error word's values: 1 a barrier timed out, 2 ono_ring_abort, 3 a flag
// ahead of the round (something other than this ring's peer wrote it).
int xgmi_err(uint32_t w) {
    if (w == 3u)
        return set_error(ONO_E_IO, "xGMI ring: a barrier flag was ahead of the round (written by something other "
                                   "than this ring's peer): the round's results are invalid");
    return set_error(ONO_E_IO, "xGMI ring: a peer did not reach a barrier within the timeout");
}

}  // namespace ono

using namespace ono;

namespace {

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

uint64_t fresh_ring_id() {
    static std::atomic<uint64_t> counter{0};
    std::random_device rd;
    uint64_t z = ((uint64_t)rd() << 32) ^ rd() ^ ((uint64_t)getpid() << 20) ^
                 (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count() ^
                 (counter.fetch_add(1) * 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z ^= z >> 31;
    return z ? z : 1;
}

int xgmi_alloc(ono_ring *r) {
    if (r->xgmi) return ONO_OK;
    if (r->n > ONO_MAX_INPUTS) return set_error(ONO_E_ARG, "xGMI schedule supports up to %d ranks", ONO_MAX_INPUTS);
    DeviceGuard g(r->device);
    auto *x = new XgmiState();
    r->xgmi = x;
    x->slot = align_up(r->maxc + 4, 64);
    const size_t rb = (size_t)std::max(r->n - 1, 1) * x->slot * sizeof(float);
    x->obuf_off = align_up(kFlagBytes + rb, 256);
    x->gat_off = align_up(x->obuf_off + x->slot * sizeof(float), 256);
    const char *gm = getenv("ONO_XGMI_GATHER");
    x->push_gather = gm && strcmp(gm, "push") == 0;
    const size_t bytes = x->push_gather ? x->gat_off + rb : x->gat_off;
    x->bytes = bytes;
    x->id = fresh_ring_id();
    {  // the smallest free pooled region that fits, else a new one (never with a handle handed out before)
        XgmiPool::Region reg{};
        bool fresh = false;
        std::string msg;
        int rc = pool().acquire(r->device, bytes, align_up(bytes, kPage), fresh_ring_id(), &reg, &fresh, msg);
        if (rc) return set_error(rc, "%s", msg.c_str());
        x->counted = true;
        x->xbuf = reg.ptr;
        x->alloc = reg.bytes;
        x->uid = reg.uid;
        memcpy(&x->handle, reg.handle.data(), sizeof x->handle);
        // flags start at epoch 0, no teardown markers; the import counters of a pooled region stay (its
        // peers' mappings of it stay open across rings), a fresh region's start at zero
        ONO_HIP(hipMemset(x->xbuf, 0, fresh ? kFlagBytes : kCountOff));
    }
    ONO_HIP(launch_xgmi_stamp(x->xbuf, (bytes + kPage - 1) / kPage, kIdOff, x->id, nullptr));
    ONO_HIP(hipDeviceSynchronize());              // zeroed and stamped before the handle leaves this process
    x->peer.assign(r->n, nullptr);
    x->peer[r->pos] = x->xbuf;
    ONO_HIP(hipHostMalloc((void **)&x->err, sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent));
    *x->err = 0;
    ONO_HIP(hipHostGetDevicePointer((void **)&x->err_dev, x->err, 0));
    xgmi_set_timeout(r);
    return ONO_OK;
}

}  // namespace

namespace ono {

// How long a device barrier waits for a peer before it gives up (ONO_E_IO).
// The reference's TCP ring blocks for as long as a peer is merely slow, so the
// default is long (kDefaultTimeoutS): ranks may drift apart by up to that much
// between rounds (rank-0 evaluation, checkpointing).  The bound exists so that
// a peer that died cannot pin a spinning workgroup forever; ono_ring_abort
// ends a waiting barrier at once.  Per ring: ono_ring_set_xgmi_timeout; else
// env ONO_XGMI_TIMEOUT_S.
constexpr double kDefaultTimeoutS = 600.0;
void xgmi_set_timeout(ono_ring *r) {
    XgmiState *x = r->xgmi;
    if (!x) return;
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, r->device) != hipSuccess || khz <= 0)
        khz = 100000;  // MI300-class constant 100 MHz wall clock
    const char *e = getenv("ONO_XGMI_TIMEOUT_S");
    const double secs = r->xgmi_timeout_s > 0 ? r->xgmi_timeout_s : e && atof(e) > 0 ? atof(e) : kDefaultTimeoutS;
    x->timeout_ticks = (uint64_t)(secs * khz * 1000.0);
    x->timeout_s = secs;
}

}  // namespace ono

namespace {

uint64_t *flags_of(uint8_t *region) { return reinterpret_cast<uint64_t *>(region); }
float *rbuf_of(const XgmiState *x, uint8_t *region, int k) {
    return reinterpret_cast<float *>(region + kFlagBytes) + (size_t)k * x->slot;
}
uint8_t *obuf_of(const XgmiState *x, uint8_t *region) { return region + x->obuf_off; }
// receiver q's gather slot for owner o's result (push_gather), slots in owner order without q
uint8_t *gslot_of(const XgmiState *x, uint8_t *region_q, int o, int q) {
    return region_q + x->gat_off + (size_t)(o < q ? o : o - 1) * x->slot * sizeof(float);
}

int barrier(ono_ring *r, hipStream_t s);

void make_blob(const XgmiState *x, uint8_t *blob) {
    memset(blob, 0, ONO_XGMI_HANDLE_BYTES);
    memcpy(blob, &x->handle, sizeof x->handle);
    memcpy(blob + kBlobId, &x->id, 8);
    const uint64_t b = x->bytes, a = x->alloc;
    memcpy(blob + kBlobBytes, &b, 8);
    memcpy(blob + kBlobUid, &x->uid, 8);
    memcpy(blob + kBlobAlloc, &a, 8);
}

// peer region `uid` as mapped in this process: the mapping made for an
// earlier ring, else a new import (kept until ono_xgmi_pool_close_imports)
int map_peer(ono_ring *r, const hipIpcMemHandle_t &h, uint64_t uid, size_t alloc, uint8_t **out) {
    IpcBytes hb;
    memcpy(hb.data(), &h, sizeof h);
    std::string msg;
    int rc = pool().map(r->device, hb, uid, alloc, out, msg);
    return rc ? set_error(rc, "%s", msg.c_str()) : ONO_OK;
}

// Every page of peer q's region as mapped here must show the id q stamped.
int verify_import(ono_ring *r, int q, uint64_t id, size_t bytes) {
    XgmiState *x = r->xgmi;
    const size_t npages = (bytes + kPage - 1) / kPage;
    uint8_t *bad_dev = nullptr;
    ONO_HIP(hipMalloc((void **)&bad_dev, npages));
    std::vector<uint8_t> bad(npages);
    hipError_t e = launch_xgmi_verify(x->peer[q], npages, kIdOff, id, bad_dev, nullptr);
    if (e == hipSuccess) e = hipMemcpy(bad.data(), bad_dev, npages, hipMemcpyDeviceToHost);
    (void)hipFree(bad_dev);
    if (e != hipSuccess) return hip_error(e, "exchange region verification", __FILE__, __LINE__);
    size_t nbad = 0, first = npages;
    for (size_t p = 0; p < npages; p++)
        if (bad[p]) { nbad++; first = std::min(first, p); }
    if (nbad)
        return set_error(ONO_E_IO,
                         "xGMI connect: rank %d's exchange region as mapped here shows another region's memory "
                         "(%zu of %zu pages lack ring id %016llx, first page %zu): a stale IPC import",
                         q, nbad, npages, (unsigned long long)id, first);
    return ONO_OK;
}

int xgmi_connect(ono_ring *r, const uint8_t *handles) {
    XgmiState *x = r->xgmi;
    if (x->connected) return ONO_OK;
    DeviceGuard g(r->device);
    x->peer_id.assign(r->n, 0);
    x->peer_id[r->pos] = x->id;
    int rc = ONO_OK;
    for (int q = 0; q < r->n && rc == ONO_OK; q++) {
        if (q == r->pos) continue;
        const uint8_t *blob = handles + (size_t)q * ONO_XGMI_HANDLE_BYTES;
        hipIpcMemHandle_t h;
        memcpy(&h, blob, sizeof h);
        uint64_t id = 0, bytes = 0, uid = 0, alloc = 0;
        memcpy(&id, blob + kBlobId, 8);
        memcpy(&bytes, blob + kBlobBytes, 8);
        memcpy(&uid, blob + kBlobUid, 8);
        memcpy(&alloc, blob + kBlobAlloc, 8);
        if (id == 0 || uid == 0 || bytes != x->bytes || alloc < bytes) {
            rc = set_error(ONO_E_ARG, "xGMI connect: rank %d's handle is not an exchange region of this ring "
                           "(id %016llx, %llu bytes; expected %zu)", q, (unsigned long long)id,
                           (unsigned long long)bytes, x->bytes);
            break;
        }
        uint8_t *p = nullptr;
        if ((rc = map_peer(r, h, uid, (size_t)alloc, &p))) break;
        x->peer[q] = p;
        x->peer_id[q] = id;
        rc = verify_import(r, q, id, (size_t)bytes);
    }
    if (rc) {  // the mappings stay in the process's table (never unmapped); this ring is not connected
        for (int q = 0; q < r->n; q++)
            if (q != r->pos) x->peer[q] = nullptr;
        return rc;
    }
    x->connected = true;
    // No rank writes a peer's region before every importer has checked its
    // stamps: a barrier that every rank passes only once all are connected.
    if ((rc = barrier(r, nullptr))) return rc;
    ONO_HIP(hipDeviceSynchronize());
    if (uint32_t w = __atomic_load_n(x->err, __ATOMIC_ACQUIRE))
        return w == 3u ? xgmi_err(w) : set_error(ONO_E_IO, "xGMI connect: a peer did not connect within the timeout");
    return ONO_OK;
}

// An RCCL ring switched to ONO_ALGO_XGMI exchanges the handles over its own
// communicator on first use (every rank is inside pull_grads together).
int xgmi_connect_over_rccl(ono_ring *r, hipStream_t s) {
    int rc = xgmi_alloc(r);
    if (rc) return rc;
    if (!r->comm) return set_error(ONO_E_ARG, "xGMI ring not connected: call ono_ring_xgmi_connect first");
    const size_t H = ONO_XGMI_HANDLE_BYTES;
    std::vector<uint8_t> all((size_t)r->n * H);
    make_blob(r->xgmi, all.data() + (size_t)r->pos * H);
    r->xgmi->exported = true;
    uint8_t *d = nullptr;
    ONO_HIP(hipMalloc((void **)&d, all.size()));
    hipError_t e = hipMemcpyAsync(d + (size_t)r->pos * H, all.data() + (size_t)r->pos * H, H, hipMemcpyHostToDevice, s);
    ncclResult_t nr = e == hipSuccess ? ncclAllGather(d + (size_t)r->pos * H, d, H, ncclUint8, r->comm, s) : ncclSuccess;
    if (e == hipSuccess && nr == ncclSuccess) e = hipMemcpyAsync(all.data(), d, all.size(), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess && nr == ncclSuccess) e = hipStreamSynchronize(s);
    (void)hipFree(d);
    if (nr != ncclSuccess) return set_error(ONO_E_RCCL, "handle all-gather: %s", ncclGetErrorString(nr));
    if (e != hipSuccess) return hip_error(e, "handle exchange", __FILE__, __LINE__);
    return xgmi_connect(r, all.data());
}

int barrier(ono_ring *r, hipStream_t s) {
    XgmiState *x = r->xgmi;
    XBarrier b{};
    for (int q = 0; q < r->n; q++) b.peer_flags[q] = flags_of(x->peer[q]);
    b.my_flags = flags_of(x->xbuf);
    b.err = x->err_dev;
    b.epoch = ++x->epoch;
    b.timeout_ticks = x->timeout_ticks;
    b.n = r->n;
    b.pos = r->pos;
    return timed(r, s, ONO_PHASE_XGMI_BARRIER, [&]() -> int {
        ONO_HIP(launch_xgmi_barrier(b, s));
        return ONO_OK;
    });
}

uint32_t head_of(const void *a, size_t esz_a, const void *b, size_t esz_b) {
    const unsigned pa = (unsigned)(((uintptr_t)a / esz_a) & 3u), pb = (unsigned)(((uintptr_t)b / esz_b) & 3u);
    return pa == pb ? (4u - pa) & 3u : kScalarOnly;
}

// One round over a piece of every chunk: chunk q contributes elements
// [off[q], off[q] + len[q]) of the buckets (a whole round: off = the chunk
// starts, len = the chunk lengths).  Every rank passes the same pieces, whose
// starts keep the chunks' 4-element phases (the slots are phase-matched).
template <class W>
int xgmi_round(ono_ring *r, float *res, float *grad, hipStream_t s, const size_t *off, const size_t *plen) {
    XgmiState *x = r->xgmi;
    const int n = r->n, pos = r->pos, c = (pos + 1) % n;
    auto len = [&](int q) { return plen[q]; };
    constexpr bool f16 = sizeof(W) == 2;
    if (uint32_t w = __atomic_load_n(x->err, __ATOMIC_ACQUIRE)) return xgmi_err(w);

    XSegs push{};  // 1. my slice of every peer's chunk -> that owner's receive slot
    for (int d = 1; d < n; d++) {
        const int q = (pos + d) % n, cq = (q + 1) % n, k = (pos - cq + n) % n;
        XSeg &sg = push.s[push.nseg++];
        sg.src = res + off[cq];
        sg.dst = rbuf_of(x, x->peer[q], k) + ph(off[cq]);
        sg.n = len(cq);
        sg.head = head_of(sg.src, 4, sg.dst, 4);
    }
    int rc = timed(r, s, ONO_PHASE_XGMI_SCATTER, [&]() -> int {
        ONO_HIP(launch_xgmi_push(push, true, s));
        return ONO_OK;
    });
    if (rc || (rc = barrier(r, s))) return rc;  // 2.

    const float *ins[ONO_MAX_INPUTS];  // 3. the chain of my chunk, reference order
    for (int k = 0; k < n - 1; k++) ins[k] = rbuf_of(x, x->xbuf, k) + ph(off[c]);
    ins[n - 1] = res + off[c];
    if (x->push_gather) {  // 3'. owner chain + its result stored straight into every peer's gather slot
        W *outs[ONO_MAX_INPUTS];
        int no = 0;
        for (int d = 1; d < n; d++) {
            const int q = (pos + d) % n;
            outs[no++] = reinterpret_cast<W *>(gslot_of(x, x->peer[q], pos, q)) + ph(off[c]);
        }
        rc = timed(r, s, ONO_PHASE_XGMI_GATHER, [&]() -> int {
            ONO_HIP(launch_direct_multi<W>(grad + off[c], outs, no, true, ins, n, len(c), (float)n, false, s));
            return ONO_OK;
        });
        if (rc || (rc = barrier(r, s))) return rc;
        XSegs unpack{};  // 5'. local: every owner's result from my gather slots -> my grad
        for (int d = 1; d < n; d++) {
            const int q = (pos + d) % n, cq = (q + 1) % n;
            XSeg &sg = unpack.s[unpack.nseg++];
            sg.src = reinterpret_cast<const W *>(gslot_of(x, x->xbuf, q, pos)) + ph(off[cq]);
            sg.dst = grad + off[cq];
            sg.n = len(cq);
            sg.head = head_of(sg.src, sizeof(W), sg.dst, 4);
        }
        ONO_K(r, s, launch_xgmi_pull(unpack, f16, f16 ? (float)n : 1.0f, s));
        return ONO_OK;
    }
    W *out = reinterpret_cast<W *>(obuf_of(x, x->xbuf)) + ph(off[c]);  // peers pull it after the barrier:
    ONO_K(r, s, launch_direct_multi<W>(grad + off[c], &out, 1, true, ins, n, len(c), (float)n, false, s));  // sys
    if ((rc = barrier(r, s))) return rc;  // 4.

    XSegs pull{};  // 5. every owner's result -> my grad
    for (int d = 1; d < n; d++) {
        const int q = (pos + d) % n, cq = (q + 1) % n;
        XSeg &sg = pull.s[pull.nseg++];
        sg.src = reinterpret_cast<const W *>(obuf_of(x, x->peer[q])) + ph(off[cq]);
        sg.dst = grad + off[cq];
        sg.n = len(cq);
        sg.head = head_of(sg.src, sizeof(W), sg.dst, 4);
    }
    return timed(r, s, ONO_PHASE_XGMI_GATHER, [&]() -> int {
        ONO_HIP(launch_xgmi_pull(pull, f16, f16 ? (float)n : 1.0f, s));
        return ONO_OK;
    });
}

int ensure_connected(ono_ring *r, hipStream_t s) {
    if (r->xgmi && r->xgmi->connected) return ONO_OK;
    return xgmi_connect_over_rccl(r, s);
}

}  // namespace

namespace ono {

// Multi-GPU parameter-server step over the same exchange regions (BASELINE
// config 5; the RCCL form is ono_ps_step's reduce-scatter + all-gather).
// Shard q = [q C, min(N, (q+1) C)) lives on rank q (store.rs:84-124 with one
// shard server per GPU):
//   1. push     my gradient slice of every peer's shard -> that owner's slot
//               for my worker index (the gradient itself is left untouched)
//   2. barrier
//   3. owner    acc = g_0 + g_1 + ... + g_{n-1} in worker order (the
//               BlockingStore accumulate order when workers arrive in rank
//               order, store.rs:84-91), then the fused (+0, ÷n, optimizer,
//               zero_grad) shard update (shard.rs:74-92) that also writes the
//               new shard into my result buffer
//   4. barrier
//   5. pull     every shard's parameters -> params (store.rs:110-124)
// Bit-exact with the store oracle fed in worker order.
int xgmi_ps_step(ono_ring *r, const float *grad, float *params, size_t N, size_t C, float *gshard, float *wshard,
                 const OptLaunch &opt, float *v, float *s_, hipStream_t s) {
    int rc = ensure_connected(r, s);
    if (rc) return rc;
    XgmiState *x = r->xgmi;
    if (C + 4 > x->slot)
        return set_error(ONO_E_SIZE, "PS shard of %zu elements exceeds the ring's exchange slot (%zu)", C, x->slot - 4);
    if (uint32_t w = __atomic_load_n(x->err, __ATOMIC_ACQUIRE)) return xgmi_err(w);
    const int n = r->n, pos = r->pos;
    auto lo = [&](int q) { return std::min(N, (size_t)q * C); };
    auto len = [&](int q) { return std::min(N, lo(q) + C) - lo(q); };
    auto slot_of = [&](int w, int owner) { return w < owner ? w : w - 1; };  // worker order, owner excluded

    XSegs push{};
    for (int d = 1; d < n; d++) {
        const int q = (pos + d) % n;
        XSeg &sg = push.s[push.nseg++];
        sg.src = grad + lo(q);
        sg.dst = rbuf_of(x, x->peer[q], slot_of(pos, q)) + ph(lo(q));
        sg.n = len(q);
        sg.head = head_of(sg.src, 4, sg.dst, 4);
    }
    rc = timed(r, s, ONO_PHASE_XGMI_SCATTER, [&]() -> int {
        ONO_HIP(launch_xgmi_push(push, false, s));
        return ONO_OK;
    });
    if (rc || (rc = barrier(r, s))) return rc;

    float *out = reinterpret_cast<float *>(obuf_of(x, x->xbuf)) + ph(lo(pos));
    if (len(pos) > 0) {
        const float *ins[ONO_MAX_INPUTS];
        for (int w = 0; w < n; w++)
            ins[w] = w == pos ? grad + lo(pos) : rbuf_of(x, x->xbuf, slot_of(w, pos)) + ph(lo(pos));
        ONO_K(r, s, launch_sum_scale(gshard, ins, n, len(pos), 1.0f, s));
        ONO_K(r, s, launch_opt_update(opt, gshard, wshard, v, s_, len(pos), true, s, out, true));
    }
    if ((rc = barrier(r, s))) return rc;

    XSegs pull{};
    for (int d = 0; d < n; d++) {
        const int q = (pos + d) % n;
        XSeg &sg = pull.s[pull.nseg++];
        sg.src = reinterpret_cast<const float *>(obuf_of(x, x->peer[q])) + ph(lo(q));
        sg.dst = params + lo(q);
        sg.n = len(q);
        sg.head = head_of(sg.src, 4, sg.dst, 4);
    }
    return timed(r, s, ONO_PHASE_XGMI_GATHER, [&]() -> int {
        ONO_HIP(launch_xgmi_pull(pull, false, 1.0f, s));
        return ONO_OK;
    });
}

int xgmi_pull_grads(ono_ring *r, float *res, float *grad, hipStream_t s) {
    int rc = ensure_connected(r, s);
    if (rc) return rc;
    std::vector<size_t> len(r->n);
    for (int q = 0; q < r->n; q++) len[q] = r->off[q + 1] - r->off[q];
    return r->wire == ONO_WIRE_F16 ? xgmi_round<uint16_t>(r, res, grad, s, r->off.data(), len.data())
                                   : xgmi_round<float>(r, res, grad, s, r->off.data(), len.data());
}

// Host-fed round (the reference's buckets are host memory): the round is cut
// into sub-rounds, sub-round j taking elements [j sub, (j+1) sub) of every
// chunk, so the H2D of sub-round j+1 (hstream), the xGMI round of j (cstream)
// and the D2H of j-1 (dstream) overlap, as the RCCL form's chunked pipeline
// does.  Every element still goes through the same chain on the same owner,
// so the result is the whole-bucket round's bit for bit.  The host residual
// is zeroed once its sub-round has reached HBM.
int xgmi_pull_grads_host(ono_ring *r, float *res_host, float *grad_host, size_t sub_elems, bool reg) {
    int rc = ensure_connected(r, r->cstream);
    if (rc) return rc;
    XgmiState *x = r->xgmi;
    const int n = r->n;
    const size_t sub = std::max<size_t>(64, sub_elems / (size_t)n / 64 * 64);  // keeps the 4-element phases
    const size_t S = (r->maxc + sub - 1) / sub;
    while (x->ev.size() < 3 * S) {
        hipEvent_t ev;  // 3 j + 1: sub-round j's result, read next by the D2H copy
        ONO_HIP(hipEventCreateWithFlags(&ev, x->ev.size() % 3 == 1 ? copy_event_flags() : hipEventDisableTiming));
        x->ev.push_back(ev);
    }
    std::vector<size_t> st(n), ln(n);
    auto piece = [&](size_t j) {
        for (int q = 0; q < n; q++) {
            const size_t L = r->off[q + 1] - r->off[q], lo = std::min(L, j * sub);
            st[q] = r->off[q] + lo;
            ln[q] = std::min(L - lo, sub);
        }
    };
    auto zero_host = [&](size_t j) -> int {  // sub-round j has reached HBM: zero its host residual
        ONO_HIP(hipEventSynchronize(x->ev[3 * j]));
        piece(j);
        for (int q = 0; q < n; q++)
            if (ln[q]) memset(res_host + st[q], 0, ln[q] * sizeof(float));
        return ONO_OK;
    };
    // How the bucket reaches HBM.  Round 6's records of the host-fed wrong result put
    // it before the owners' chains: one rank's residual read back as zeros at scattered 128-B lines, the data
    // the copy engine had written there not seen by the kernels.  The residual is therefore written by a
    // kernel, as every other buffer the round reads is: the caller's bucket read in place when it is
    // registered, else copied by the host pool into a pinned, mapped, coherent staging slot (two slots of n
    // pieces, each at the residual's 4-element phase) — read system-coherent by one launch on the copy
    // stream (launch_xgmi_host_in) that the round's stream waits for.
    // ONO_XGMI_HOST_IN=dma keeps the copy engine's H2D (with the fences below, round 6's first attempt).
    // Before each D2H a system-scope L2 write-back on every XCD (ONO_XGMI_HOST_FENCE=0 drops it; =1 adds the
    // write-back + invalidate fences around the copy-engine input as well).
    const char *ie = getenv("ONO_XGMI_HOST_IN"), *fe = getenv("ONO_XGMI_HOST_FENCE");
    const bool dma_in = ie && strcmp(ie, "dma") == 0, plain_in = ie && strcmp(ie, "plain") == 0;
    const bool fence = !(fe && strcmp(fe, "0") == 0), in_fences = dma_in && fence;
    const float *res_dev = nullptr;  // the caller's registered bucket, as the device addresses it
    if (!dma_in && reg) {
        void *p = nullptr;
        if (hipHostGetDevicePointer(&p, res_host, 0) == hipSuccess) res_dev = static_cast<const float *>(p);
        else (void)hipGetLastError();  // (not mapped: staged; the error must not reach a later launch check)
    }
    const size_t pad = sub + 4;  // a staging piece: sub elements at any 4-element phase
    if (!dma_in && !res_dev && x->hin_elems < 2 * (size_t)n * pad) {
        if (x->hin) ONO_HIP(hipHostFree(x->hin));
        x->hin = x->hin_dev = nullptr;
        x->hin_elems = 0;
        ONO_HIP(hipHostMalloc((void **)&x->hin, 2 * (size_t)n * pad * sizeof(float),
                              hipHostMallocMapped | hipHostMallocCoherent));
        ONO_HIP(hipHostGetDevicePointer((void **)&x->hin_dev, x->hin, 0));
        x->hin_elems = 2 * (size_t)n * pad;
    }
    auto input = [&](size_t j) -> int {  // sub-round j's pieces into the residual; ev[3 j] after them
        if (dma_in) {
            for (int q = 0; q < n; q++)
                if (ln[q])
                    ONO_HIP(hipMemcpyAsync(r->residual + st[q], res_host + st[q], ln[q] * sizeof(float),
                                           hipMemcpyHostToDevice, r->hstream));
            ONO_HIP(hipEventRecord(x->ev[3 * j], r->hstream));
            ONO_HIP(hipStreamWaitEvent(r->cstream, x->ev[3 * j], 0));
            if (in_fences) ONO_HIP(launch_xgmi_fence_all(r->cstream, true));
            return ONO_OK;
        }
        const size_t b = j & 1;
        if (!res_dev && j >= 2) ONO_HIP(hipEventSynchronize(x->ev[3 * (j - 2)]));  // the slot was read
        XSegs in{};
        for (int q = 0; q < n; q++) {
            if (!ln[q]) continue;
            const float *src = res_dev ? res_dev + st[q] : nullptr;
            if (!res_dev) {
                const size_t at = (b * (size_t)n + (size_t)q) * pad + (st[q] & 3);
                host_copy(r, x->hin + at, res_host + st[q], ln[q] * sizeof(float));
                src = x->hin_dev + at;
            }
            XSeg &sg = in.s[in.nseg++];
            sg.src = src;
            sg.dst = r->residual + st[q];
            sg.n = ln[q];
            sg.head = head_of(sg.src, 4, sg.dst, 4);
        }
        // (on the copy stream, so it overlaps the previous sub-round's round; the round waits for it)
        ONO_HIP(launch_xgmi_host_in(in, r->hstream, !plain_in));
        ONO_HIP(hipEventRecord(x->ev[3 * j], r->hstream));
        ONO_HIP(hipStreamWaitEvent(r->cstream, x->ev[3 * j], 0));
        return ONO_OK;
    };
    auto rounds = [&]() -> int {
        // (the copy-engine form: dirty lines an earlier kernel left on these addresses reach HBM first)
        if (in_fences) ONO_HIP(launch_xgmi_fence_all(r->hstream, true));
        for (size_t j = 0; j < S; j++) {
            piece(j);
            int rc2 = input(j);
            if (rc2) return rc2;
            rc2 = r->wire == ONO_WIRE_F16
                      ? xgmi_round<uint16_t>(r, r->residual, r->grad, r->cstream, st.data(), ln.data())
                      : xgmi_round<float>(r, r->residual, r->grad, r->cstream, st.data(), ln.data());
            if (rc2) return rc2;
            if (fence) ONO_HIP(launch_xgmi_fence_all(r->cstream, in_fences));
            ONO_HIP(hipEventRecord(x->ev[3 * j + 1], r->cstream));
            ONO_HIP(hipStreamWaitEvent(r->dstream, x->ev[3 * j + 1], 0));
            for (int q = 0; q < n; q++)
                if (ln[q])
                    ONO_HIP(hipMemcpyAsync(grad_host + st[q], r->grad + st[q], ln[q] * sizeof(float),
                                           hipMemcpyDeviceToHost, r->dstream));
            ONO_HIP(hipEventRecord(x->ev[3 * j + 2], r->dstream));
            if (j > 0 && (rc2 = zero_host(j - 1))) return rc2;
        }
        return zero_host(S - 1);
    };
    rc = rounds();
    // Every copy into or out of the caller's buffers is done before we return,
    // whether or not the round failed (the buffers are the caller's again).
    const hipError_t e1 = hipStreamSynchronize(r->hstream), e2 = hipStreamSynchronize(r->cstream),
                     e3 = hipStreamSynchronize(r->dstream);
    if (rc) return rc;
    for (hipError_t e : {e1, e2, e3})
        if (e != hipSuccess) return hip_error(e, "host-fed xGMI round", __FILE__, __LINE__);
    // A barrier that gave up let the later kernels run on partly landed slots:
    // the round's output is invalid and the host residual has already been
    // zeroed, so it must not report success (ono_ring_check's condition).
    if (uint32_t w = __atomic_load_n(x->err, __ATOMIC_ACQUIRE)) return xgmi_err(w);
    return ONO_OK;
}

// ono_ring_abort: barriers still spinning on the device give up (they poll
// the host-mapped error word), so an aborted round drains instead of waiting
// for the timeout.
void xgmi_abort(ono_ring *r) {
    if (r->xgmi && r->xgmi->err) __atomic_store_n(r->xgmi->err, 2u, __ATOMIC_RELEASE);
}

// Teardown is collective and ordered: a region goes back to the pool (where
// the next ring resets its flags) only after every peer has said it is done
// with it.  Once this rank's own work is complete (device synchronised: its
// last pushes into and pulls from peer regions are over), it stores each
// peer's ring id into that peer's teardown slot `pos` (system-scope stores
// through its mapping, which stays in the process's table); it then waits
// until its own region holds its id in every peer's slot.  A peer that never
// arrives costs the timeout, no more; after a barrier timeout or an abort this
// rank does not wait.
void xgmi_free(ono_ring *r) {
    XgmiState *x = r->xgmi;
    if (!x) return;
    DeviceGuard g(r->device);
    // after a barrier timeout or an abort this rank does not wait, but still
    // releases its peers' regions so that they do not wait for it
    bool wait = x->connected && !__atomic_load_n(x->err, __ATOMIC_ACQUIRE);
    if (x->connected) {
        bool ok = hipDeviceSynchronize() == hipSuccess;
        XSignal sig{};
        for (int q = 0; q < r->n; q++) {
            sig.peer_done[q] = q == r->pos ? nullptr : reinterpret_cast<uint64_t *>(x->peer[q] + kDoneOff);
            sig.peer_id[q] = x->peer_id[q];
        }
        sig.n = r->n;
        sig.pos = r->pos;
        ok = ok && launch_xgmi_signal(sig, nullptr) == hipSuccess && hipDeviceSynchronize() == hipSuccess;
        wait &= ok;
    }
    // a region that never left this process is nobody else's; one whose
    // peers all marked it is free again; anything else is quarantined
    bool released = !x->exported;
    if (wait) {  // every peer's marker in this region (uncached: a D2H copy reads what landed)
        const auto t0 = std::chrono::steady_clock::now();
        std::vector<uint64_t> done(r->n);
        for (;;) {
            if (hipMemcpy(done.data(), x->xbuf + kDoneOff, r->n * sizeof(uint64_t), hipMemcpyDeviceToHost) !=
                hipSuccess)
                break;
            bool all = true;
            for (int q = 0; q < r->n; q++) all &= q == r->pos || done[q] == x->id;
            if (all) released = true;
            if (all || r->aborted.load()) break;
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > x->timeout_s) break;
            std::this_thread::sleep_for(std::chrono::microseconds(200));
        }
    }
    for (hipEvent_t ev : x->ev) (void)hipEventDestroy(ev);
    if (x->hin) (void)hipHostFree(x->hin);
    // the region goes back to the pool (or into quarantine); peer mappings stay in the process's table
    if (x->counted) pool().release_ring(x->xbuf, released);
    if (x->err) (void)hipHostFree(x->err);
    delete x;
    r->xgmi = nullptr;
}

}  // namespace ono

extern "C" {

int ono_ring_create_xgmi(ono_ring **out, int pos, int nranks, size_t size, int device, int wire) {
    if (!out) return set_error(ONO_E_ARG, "out is NULL");
    *out = nullptr;
    if (nranks < 1 || nranks > ONO_MAX_INPUTS || pos < 0 || pos >= nranks)
        return set_error(ONO_E_ARG, "pos=%d nranks=%d (xGMI schedule: 1..%d ranks)", pos, nranks, ONO_MAX_INPUTS);
    if (wire != ONO_WIRE_F32 && wire != ONO_WIRE_F16) return set_error(ONO_E_ARG, "wire=%d", wire);
    if (size < (size_t)nranks)  // reference: chunks[pos] out of bounds (worker_ring.rs:120-122)
        return set_error(ONO_E_SIZE, "bucket of %zu elements cannot be split over %d ranks", size, nranks);
    ono_ring *r = nullptr;
    int rc = ono_ring_create(&r, 0, 1, size, device, nullptr, wire);  // buckets + streams, no communicator
    if (rc) return rc;
    r->n = nranks;
    r->pos = pos;
    r->off = split_chunks(size, (size_t)nranks);
    r->maxc = r->off[1] - r->off[0];
    r->algo = ONO_ALGO_XGMI;
    if (nranks > 1 && (rc = xgmi_alloc(r))) {
        ono_ring_destroy(r);
        return rc;
    }
    *out = r;
    return ONO_OK;
}

int ono_ring_xgmi_handle(ono_ring *r, uint8_t handle[ONO_XGMI_HANDLE_BYTES]) {
    if (!r || !handle) return set_error(ONO_E_ARG, "NULL argument");
    memset(handle, 0, ONO_XGMI_HANDLE_BYTES);
    if (r->n == 1) return ONO_OK;
    int rc = xgmi_alloc(r);
    if (rc) return rc;
    make_blob(r->xgmi, handle);
    r->xgmi->exported = true;
    return ONO_OK;
}

int ono_xgmi_pool_close_imports(size_t *closed_imports) {
    std::string msg;
    int rc = pool().close_imports(closed_imports, msg);
    return rc ? set_error(rc, "%s", msg.c_str()) : ONO_OK;
}

int ono_xgmi_pool_free_exports(size_t *freed_bytes, size_t *kept, double wait_s) {
    if (!(wait_s >= 0) || wait_s > 1e7) return set_error(ONO_E_ARG, "wait %g s", wait_s);
    std::string msg;
    int rc = pool().free_exports(wait_s, freed_bytes, kept, msg);
    return rc ? set_error(rc, "%s", msg.c_str()) : ONO_OK;
}

int ono_xgmi_pool_release(size_t *freed_bytes, size_t *closed_imports) {
    if (freed_bytes) *freed_bytes = 0;
    if (closed_imports) *closed_imports = 0;
    int rc = ono_xgmi_pool_close_imports(closed_imports);
    if (rc) return rc;
    // the peers close their imports of this process's regions in their own release: wait for them a short
    // while (ONO_XGMI_RELEASE_WAIT_S, 30 s by default; a region still mapped by a peer after it is kept, and
    // retired from reuse)
    const char *e = getenv("ONO_XGMI_RELEASE_WAIT_S");
    const double wait = e && atof(e) > 0 ? atof(e) : 30.0;
    return ono_xgmi_pool_free_exports(freed_bytes, nullptr, wait);
}

int ono_xgmi_pool_stats(size_t *regions, size_t *region_bytes, size_t *quarantined, size_t *imports) {
    const XgmiPool::Stats st = pool().stats();
    if (regions) *regions = st.regions;
    if (region_bytes) *region_bytes = st.region_bytes;
    if (quarantined) *quarantined = st.quarantined;
    if (imports) *imports = st.imports;
    return ONO_OK;
}

int ono_ring_check(const ono_ring *r) {
    if (!r) return set_error(ONO_E_ARG, "ring is NULL");
    if (r->aborted.load()) return set_error(ONO_E_ABORTED, "ring aborted");
    if (r->xgmi && r->xgmi->err) {
        const uint32_t w = __atomic_load_n(r->xgmi->err, __ATOMIC_ACQUIRE);
        if (w == 1u || w == 3u) return xgmi_err(w);
    }
    return ONO_OK;
}

int ono_ring_set_xgmi_timeout(ono_ring *r, double seconds) {
    if (!r) return set_error(ONO_E_ARG, "ring is NULL");
    if (!(seconds >= 0) || seconds > 1e7) return set_error(ONO_E_ARG, "timeout %g s", seconds);
    std::lock_guard<std::mutex> lk(r->mu);  // a round in flight reads the ticks under the same lock
    r->xgmi_timeout_s = seconds;
    xgmi_set_timeout(r);  // later barriers use it (an allocated region keeps its flags)
    return ONO_OK;
}

int ono_ring_xgmi_connect(ono_ring *r, const uint8_t *handles) {
    if (!r || !handles) return set_error(ONO_E_ARG, "NULL argument");
    if (r->n == 1) return ONO_OK;
    int rc = xgmi_alloc(r);
    if (rc) return rc;
    return xgmi_connect(r, handles);
}

}  // extern "C"
