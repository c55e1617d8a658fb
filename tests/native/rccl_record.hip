// rccl_record.hip — TEST INFRASTRUCTURE ONLY (never linked into the product).
//
// A stand-in for the RCCL calls libono_reduce.so makes, preloaded
// (LD_PRELOAD) into ONE test process whose ranks are threads sharing one GPU
// (tests/rccl_record_worker.py).  RCCL itself refuses two ranks per device,
// so without this the mapping of an exchange-plan step to its RCCL call
// (run_plan, ono_ring.cpp) would first execute on the driver's 8-GPU node.
//
// Every call is RECORDED (JSON lines into $ONO_RCCL_RECORD: rank, op,
// pointers, count, dtype, peer, stream, group) and CARRIED OUT with the
// semantics RCCL documents, stream-ordered:
//   ncclSend / ncclRecv      matched per (communicator, sender, receiver) in
//                            issue order; the receiver's stream waits for the
//                            sender's data (event), copies it (D2D), and the
//                            sender's stream waits for that copy before its
//                            buffer can be reused.  Inside ncclGroupStart /
//                            ncclGroupEnd all sends are posted before any
//                            receive waits, so grouped exchanges never block
//                            each other.  A count or dtype mismatch between a
//                            matched pair fails both calls.
//   ncclAllReduce(sum)       dst_r = ((src_0 + src_1) + ...) + src_{n-1}: the
//                            rank-order f32 sum (RCCL's own order differs for
//                            n >= 3; the tests compare with the same rank-order
//                            restatement)
//   ncclReduceScatter(sum)   dst_r = rank-order sum of src_q[r count, (r+1) count)
//   ncclAllGather            dst_r[q count, (q+1) count) = src_q
// Collectives snapshot every rank's source first, so in-place calls are safe.
// ncclCommInitRank returns a communicator object of this library (no network,
// no device resources); ncclGetUniqueId draws random bytes.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <unistd.h>

#include <algorithm>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <tuple>
#include <vector>

namespace {

struct FakeComm {
    uint64_t key;
    int n, rank;
    uint64_t coll_seq = 0;  // this rank's collectives so far
};

std::mutex g_mu;
std::condition_variable g_cv;
FILE *g_log = nullptr;
uint64_t g_group_id = 0;
std::vector<void *> g_scratch;  // collective snapshots, freed at communicator destruction

size_t dtype_size(ncclDataType_t t) {
    switch (t) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: return 0;
    }
}

void log_line(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
void log_line(const char *fmt, ...) {
    if (!g_log) {
        const char *p = getenv("ONO_RCCL_RECORD");
        if (!p) return;
        g_log = fopen(p, "a");
        if (!g_log) return;
    }
    va_list ap;
    va_start(ap, fmt);
    vfprintf(g_log, fmt, ap);
    va_end(ap);
    fputc('\n', g_log);
    fflush(g_log);
}

struct SendPost {
    const void *ptr;
    size_t count;
    ncclDataType_t dtype;
    hipEvent_t ready = nullptr, done = nullptr;
    bool has_done = false, failed = false;
};
std::map<std::tuple<uint64_t, int, int>, std::deque<std::shared_ptr<SendPost>>> g_posts;

struct P2P {
    bool send;
    FakeComm *c;
    void *ptr;
    size_t count;
    ncclDataType_t dtype;
    int peer;
    hipStream_t s;
};
thread_local int t_depth = 0;
thread_local std::vector<P2P> t_ops;
thread_local uint64_t t_group = 0;

hipEvent_t new_event() {
    hipEvent_t e = nullptr;
    (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
    return e;
}

ncclResult_t run_group(std::vector<P2P> &ops) {
    std::vector<std::shared_ptr<SendPost>> mine(ops.size());
    ncclResult_t rc = ncclSuccess;
    {  // 1. post every send
        std::lock_guard<std::mutex> lk(g_mu);
        for (size_t i = 0; i < ops.size(); i++) {
            if (!ops[i].send) continue;
            auto p = std::make_shared<SendPost>();
            p->ptr = ops[i].ptr;
            p->count = ops[i].count;
            p->dtype = ops[i].dtype;
            p->ready = new_event();
            (void)hipEventRecord(p->ready, ops[i].s);
            g_posts[{ops[i].c->key, ops[i].c->rank, ops[i].peer}].push_back(p);
            mine[i] = p;
        }
    }
    g_cv.notify_all();
    for (size_t i = 0; i < ops.size(); i++) {  // 2. every receive: the matching send's data
        if (ops[i].send) continue;
        std::unique_lock<std::mutex> lk(g_mu);
        auto &q = g_posts[{ops[i].c->key, ops[i].peer, ops[i].c->rank}];
        g_cv.wait(lk, [&] { return !q.empty(); });
        auto p = q.front();
        q.pop_front();
        lk.unlock();
        if (p->count != ops[i].count || p->dtype != ops[i].dtype) {
            log_line("{\"rank\": %d, \"op\": \"mismatch\", \"peer\": %d, \"send_count\": %zu, \"recv_count\": %zu}",
                     ops[i].c->rank, ops[i].peer, p->count, ops[i].count);
            p->failed = true;
            rc = ncclInvalidUsage;
        } else {
            (void)hipStreamWaitEvent(ops[i].s, p->ready, 0);
            (void)hipMemcpyAsync(ops[i].ptr, p->ptr, p->count * dtype_size(p->dtype), hipMemcpyDeviceToDevice,
                                 ops[i].s);
        }
        p->done = new_event();
        (void)hipEventRecord(p->done, ops[i].s);
        {
            std::lock_guard<std::mutex> lk2(g_mu);
            p->has_done = true;
        }
        g_cv.notify_all();
    }
    for (size_t i = 0; i < ops.size(); i++) {  // 3. a send buffer is free once its copy ran
        if (!ops[i].send) continue;
        std::unique_lock<std::mutex> lk(g_mu);
        g_cv.wait(lk, [&] { return mine[i]->has_done; });
        lk.unlock();
        if (mine[i]->failed) rc = ncclInvalidUsage;
        (void)hipStreamWaitEvent(ops[i].s, mine[i]->done, 0);
    }
    return rc;
}

constexpr int kMaxRanks = 16;
struct Srcs {
    const float *p[kMaxRanks];
};
__global__ void sum_kernel(float *dst, Srcs s, int k, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        float a = s.p[0][i];
        for (int j = 1; j < k; j++) a = a + s.p[j][i];
        dst[i] = a;
    }
}

struct Coll {
    int kind = 0;  // 0 all-reduce, 1 reduce-scatter, 2 all-gather
    size_t count = 0;
    ncclDataType_t dtype = ncclFloat32;
    int arrived = 0, finished = 0;
    bool failed = false;
    std::vector<void *> snap;  // every rank's source, snapshotted on its stream
    std::vector<hipEvent_t> ready, done;
};
std::map<std::pair<uint64_t, uint64_t>, std::shared_ptr<Coll>> g_colls;

ncclResult_t collective(int kind, const void *src, void *dst, size_t count, ncclDataType_t dtype, FakeComm *c,
                        hipStream_t s) {
    if (!c) return ncclInvalidArgument;
    const size_t es = dtype_size(dtype);
    const size_t src_elems = kind == 1 ? count * (size_t)c->n : count;
    std::unique_lock<std::mutex> lk0(g_mu);
    log_line("{\"rank\": %d, \"op\": \"%s\", \"src\": %llu, \"dst\": %llu, \"count\": %zu, \"dtype\": %d, "
             "\"stream\": %llu, \"seq\": %llu}",
             c->rank, kind == 0 ? "all_reduce" : kind == 1 ? "reduce_scatter" : "all_gather",
             (unsigned long long)(uintptr_t)src, (unsigned long long)(uintptr_t)dst, count, (int)dtype,
             (unsigned long long)(uintptr_t)s, (unsigned long long)c->coll_seq);
    lk0.unlock();
    if (es == 0 || (kind != 2 && dtype != ncclFloat32)) return ncclInvalidArgument;
    void *snap = nullptr;
    if (hipMalloc(&snap, std::max<size_t>(src_elems * es, 4)) != hipSuccess) return ncclSystemError;
    (void)hipMemcpyAsync(snap, src, src_elems * es, hipMemcpyDeviceToDevice, s);
    std::shared_ptr<Coll> co;
    {
        std::unique_lock<std::mutex> lk(g_mu);
        g_scratch.push_back(snap);
        auto &slot = g_colls[{c->key, c->coll_seq++}];
        if (!slot) {
            slot = std::make_shared<Coll>();
            slot->kind = kind;
            slot->count = count;
            slot->dtype = dtype;
            slot->snap.assign(c->n, nullptr);
            slot->ready.assign(c->n, nullptr);
            slot->done.assign(c->n, nullptr);
        }
        co = slot;
        if (co->kind != kind || co->count != count || co->dtype != dtype) co->failed = true;
        co->snap[c->rank] = snap;
        co->ready[c->rank] = new_event();
        (void)hipEventRecord(co->ready[c->rank], s);
        co->arrived++;
        g_cv.notify_all();
        g_cv.wait(lk, [&] { return co->arrived == c->n; });
    }
    if (co->failed) {
        log_line("{\"rank\": %d, \"op\": \"mismatch\", \"collective\": %d}", c->rank, kind);
        return ncclInvalidUsage;
    }
    for (int q = 0; q < c->n; q++) (void)hipStreamWaitEvent(s, co->ready[q], 0);
    if (kind == 2) {
        for (int q = 0; q < c->n; q++)
            (void)hipMemcpyAsync(static_cast<char *>(dst) + (size_t)q * count * es, co->snap[q], count * es,
                                 hipMemcpyDeviceToDevice, s);
    } else if (count) {
        Srcs sp{};
        for (int q = 0; q < c->n; q++)
            sp.p[q] = static_cast<const float *>(co->snap[q]) + (kind == 1 ? (size_t)c->rank * count : 0);
        const unsigned blocks = (unsigned)std::min<size_t>((count + 255) / 256, 65535);
        hipLaunchKernelGGL(sum_kernel, dim3(blocks), dim3(256), 0, s, static_cast<float *>(dst), sp, c->n, count);
    }
    {
        std::unique_lock<std::mutex> lk(g_mu);
        co->done[c->rank] = new_event();
        (void)hipEventRecord(co->done[c->rank], s);
        co->finished++;
        g_cv.notify_all();
        g_cv.wait(lk, [&] { return co->finished == c->n; });
    }
    for (int q = 0; q < c->n; q++) (void)hipStreamWaitEvent(s, co->done[q], 0);  // snapshots stay until all read
    return ncclSuccess;
}

}  // namespace

extern "C" {

ncclResult_t ncclGetUniqueId(ncclUniqueId *id) {
    static std::mt19937_64 rng(std::random_device{}() ^ ((uint64_t)getpid() << 17));
    std::lock_guard<std::mutex> lk(g_mu);
    for (size_t i = 0; i < sizeof(id->internal); i += 8) {
        const uint64_t v = rng();
        memcpy(id->internal + i, &v, std::min<size_t>(8, sizeof(id->internal) - i));
    }
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t *comm, int nranks, ncclUniqueId commId, int rank) {
    if (!comm || nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks) return ncclInvalidArgument;
    uint64_t key = 1469598103934665603ULL;  // FNV-1a of the id
    for (char ch : commId.internal) key = (key ^ (uint8_t)ch) * 1099511628211ULL;
    auto *c = new FakeComm{key, nranks, rank};
    *comm = reinterpret_cast<ncclComm_t>(c);
    std::lock_guard<std::mutex> lk(g_mu);
    log_line("{\"rank\": %d, \"op\": \"init\", \"nranks\": %d, \"comm\": %llu}", rank, nranks,
             (unsigned long long)key);
    return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
    auto *c = reinterpret_cast<FakeComm *>(comm);
    if (!c) return ncclSuccess;
    (void)hipDeviceSynchronize();
    std::lock_guard<std::mutex> lk(g_mu);
    log_line("{\"rank\": %d, \"op\": \"destroy\"}", c->rank);
    delete c;
    return ncclSuccess;
}

ncclResult_t ncclCommAbort(ncclComm_t comm) { return ncclCommDestroy(comm); }

ncclResult_t ncclGroupStart() {
    if (t_depth++ == 0) {
        std::lock_guard<std::mutex> lk(g_mu);
        t_group = ++g_group_id;
        t_ops.clear();
    }
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
    if (t_depth == 0) return ncclInvalidUsage;
    if (--t_depth > 0) return ncclSuccess;
    int rank = t_ops.empty() ? -1 : t_ops[0].c->rank;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        log_line("{\"rank\": %d, \"op\": \"group\", \"group\": %llu, \"calls\": %zu}", rank,
                 (unsigned long long)t_group, t_ops.size());
    }
    std::vector<P2P> ops;
    ops.swap(t_ops);
    return run_group(ops);
}

static ncclResult_t p2p(bool send, const void *buf, size_t count, ncclDataType_t dtype, int peer, ncclComm_t comm,
                        hipStream_t s) {
    auto *c = reinterpret_cast<FakeComm *>(comm);
    if (!c || peer < 0 || peer >= c->n || peer == c->rank || dtype_size(dtype) == 0) return ncclInvalidArgument;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        log_line("{\"rank\": %d, \"op\": \"%s\", \"ptr\": %llu, \"count\": %zu, \"dtype\": %d, \"peer\": %d, "
                 "\"stream\": %llu, \"group\": %llu}",
                 c->rank, send ? "send" : "recv", (unsigned long long)(uintptr_t)buf, count, (int)dtype, peer,
                 (unsigned long long)(uintptr_t)s, (unsigned long long)(t_depth ? t_group : 0));
    }
    P2P op{send, c, const_cast<void *>(buf), count, dtype, peer, s};
    if (t_depth) {
        t_ops.push_back(op);
        return ncclSuccess;
    }
    std::vector<P2P> one{op};
    return run_group(one);
}

ncclResult_t ncclSend(const void *sendbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm,
                      hipStream_t stream) {
    return p2p(true, sendbuff, count, datatype, peer, comm, stream);
}

ncclResult_t ncclRecv(void *recvbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm,
                      hipStream_t stream) {
    return p2p(false, recvbuff, count, datatype, peer, comm, stream);
}

ncclResult_t ncclAllReduce(const void *sendbuff, void *recvbuff, size_t count, ncclDataType_t datatype, ncclRedOp_t op,
                           ncclComm_t comm, hipStream_t stream) {
    if (op != ncclSum) return ncclInvalidArgument;
    return collective(0, sendbuff, recvbuff, count, datatype, reinterpret_cast<FakeComm *>(comm), stream);
}

ncclResult_t ncclReduceScatter(const void *sendbuff, void *recvbuff, size_t recvcount, ncclDataType_t datatype,
                               ncclRedOp_t op, ncclComm_t comm, hipStream_t stream) {
    if (op != ncclSum) return ncclInvalidArgument;
    return collective(1, sendbuff, recvbuff, recvcount, datatype, reinterpret_cast<FakeComm *>(comm), stream);
}

ncclResult_t ncclAllGather(const void *sendbuff, void *recvbuff, size_t sendcount, ncclDataType_t datatype,
                           ncclComm_t comm, hipStream_t stream) {
    return collective(2, sendbuff, recvbuff, sendcount, datatype, reinterpret_cast<FakeComm *>(comm), stream);
}

}  // extern "C"
