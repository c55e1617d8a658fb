// ono_ring.cpp — the ring all-reduce (WorkerRingManager) over RCCL/xGMI, the
// co-resident "local ring", and the multi-GPU parameter-server step.
//
// Reference: worker/src/middlewares/worker_ring.rs:82-204.  Two wires:
//   ONO_WIRE_F32 — ncclAllReduce(sum) + one fused kernel (grad /= n,
//                  residual = 0).  RCCL picks its own ring/channel order.
//   ONO_WIRE_F16 — the reference's exact hop schedule, point-to-point over
//                  RCCL (ncclSend/ncclRecv), with fused codec kernels:
//                    scatter hop 0      encode_zero        (:122, :133)
//                    scatter hops 1..   add_encode_zero    (:141-143 then :122, :133)
//                    last scatter hop   add_finish         (:141-143, :166, :191-193, ÷n)
//                    gather hops        decode_scale       (:200, ÷n) + forward the
//                                       received bytes (f16(f32(h)) == h)
// The division by n is applied to the same value the reference divides at
// the end (param_manager.rs:183-188), so fusing it is bit-identical.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <atomic>
#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "ono_internal.h"
#include "ono_plan.h"
#include "ono_ring_impl.h"


using namespace ono;

static_assert(sizeof(ncclUniqueId) == ONO_UID_BYTES, "ncclUniqueId size");

namespace ono {

// Host-side copy pool for the pageable host-fed form: the CPU copies between
// the caller's pageable buckets and the pinned bounce slots (and the residual
// zeroing) are split over T threads, so they keep up with PCIe Gen5 DMA.
// T = env ONO_HOST_THREADS (default 16, at most the hardware threads).  The
// registered form does not use it: its only CPU work is zeroing the residual,
// and a single thread there leaves the host memory bandwidth to the DMA.
// The pool's threads run on the CPUs of the GPU's NUMA node (the node that
// /sys reports for its PCI function, intersected with the process's allowed
// CPUs): the bounce slots are pinned there, and the round-to-round spread of
// the pageable rate (21-33 GiB/s unbound) came from copies that
// the scheduler moved across sockets.  ONO_HOST_NUMA=0 leaves them unbound.
static bool gpu_node_cpus(int device, cpu_set_t *out) {
    const char *e = getenv("ONO_HOST_NUMA");
    if (e && !strcmp(e, "0")) return false;
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof bus, device) != hipSuccess) return false;
    for (char *c = bus; *c; c++) *c = (char)tolower(*c);
    char path[256];
    snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bus);
    FILE *f = fopen(path, "r");
    if (!f) return false;
    int node = -1;
    if (fscanf(f, "%d", &node) != 1) node = -1;
    fclose(f);
    if (node < 0) return false;
    snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
    f = fopen(path, "r");
    if (!f) return false;
    cpu_set_t set;
    CPU_ZERO(&set);
    int a, b;
    char sep;
    while (fscanf(f, "%d", &a) == 1) {  // "0-63,128-191"
        b = a;
        if (fscanf(f, "%c", &sep) == 1 && sep == '-') {
            if (fscanf(f, "%d", &b) != 1) break;
            if (fscanf(f, "%c", &sep) != 1) sep = 0;
        }
        for (int c = a; c <= b && c < CPU_SETSIZE; c++) CPU_SET(c, &set);
        if (sep != ',') break;
    }
    fclose(f);
    cpu_set_t allowed;
    if (sched_getaffinity(0, sizeof allowed, &allowed) == 0) CPU_AND(&set, &set, &allowed);
    if (CPU_COUNT(&set) == 0) return false;
    *out = set;
    return true;
}

class HostPool {
public:
    HostPool(int t, int device) : nt_(std::max(1, t)) {
        cpu_set_t set;
        const bool bind = gpu_node_cpus(device, &set);
        numa_bound_ = bind;
        for (int i = 1; i < nt_; i++)
            th_.emplace_back([this, i, bind, set] {
                if (bind) (void)pthread_setaffinity_np(pthread_self(), sizeof set, &set);
                loop(i);
            });
    }
    bool numa_bound() const { return numa_bound_; }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    int threads() const { return nt_; }
    // f(part, nparts) on every thread (the caller runs part 0); returns when all are done
    void run(const std::function<void(int, int)> &f) {
        if (nt_ == 1) { f(0, 1); return; }
        {
            std::lock_guard<std::mutex> lk(m_);
            job_ = &f;
            pending_ = nt_ - 1;
            gen_++;
        }
        cv_.notify_all();
        f(0, nt_);
        std::unique_lock<std::mutex> lk(m_);
        done_.wait(lk, [this] { return pending_ == 0; });
        job_ = nullptr;
    }
    void copy(void *dst, const void *src, size_t bytes) {
        run([&](int i, int k) {
            size_t lo, len;
            part(bytes, i, k, lo, len);
            if (len) memcpy(static_cast<char *>(dst) + lo, static_cast<const char *>(src) + lo, len);
        });
    }
    void zero(void *dst, size_t bytes) {
        run([&](int i, int k) {
            size_t lo, len;
            part(bytes, i, k, lo, len);
            if (len) memset(static_cast<char *>(dst) + lo, 0, len);
        });
    }

private:
    static void part(size_t bytes, int i, int k, size_t &lo, size_t &len) {
        size_t per = ((bytes + k - 1) / k + 4095) & ~size_t(4095);  // page-aligned pieces
        lo = std::min(bytes, per * i);
        len = std::min(bytes - lo, per);
    }
    void loop(int i) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(int, int)> *f;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                f = job_;
            }
            (*f)(i, nt_);
            std::lock_guard<std::mutex> lk(m_);
            if (--pending_ == 0) done_.notify_one();
        }
    }
    int nt_;
    bool numa_bound_ = false;
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<void(int, int)> *job_ = nullptr;
    int pending_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

// Device-to-device copies and zero fills of the schedules run on the library's
// own stream kernels (ono_copy_f32 / ono_fill_f32's skeleton): the runtime's
// blit kernels reach 0.62 (copy) / 0.73 (fill) of 8 TB/s at 64 MiB against 0.79
// / 0.77 for these (profiles/r04_launch_phases_s3.txt, bench copy_ceiling).
hipError_t dev_copy(void *dst, const void *src, size_t bytes, hipStream_t s) {
    if (!bytes) return hipSuccess;
    if (((uintptr_t)dst | (uintptr_t)src | bytes) % 4 == 0)
        return launch_copy<float>(static_cast<float *>(dst), static_cast<const float *>(src), bytes / 4, s);
    if (((uintptr_t)dst | (uintptr_t)src | bytes) % 2 == 0)
        return launch_copy<uint16_t>(static_cast<uint16_t *>(dst), static_cast<const uint16_t *>(src), bytes / 2, s);
    return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s);
}
hipError_t dev_zero(void *dst, size_t bytes, hipStream_t s) {
    if (!bytes) return hipSuccess;
    if (((uintptr_t)dst | bytes) % 4 == 0) return launch_fill<float>(static_cast<float *>(dst), 0.0f, bytes / 4, s);
    if (((uintptr_t)dst | bytes) % 2 == 0)
        return launch_fill<uint16_t>(static_cast<uint16_t *>(dst), (uint16_t)0, bytes / 2, s);
    return hipMemsetAsync(dst, 0, bytes, s);
}

// The CPUs this process may actually keep busy: its affinity mask, and under a
// cgroup v2 CPU quota (cpu.max "quota period") the quota's whole CPUs.  A pool
// as wide as the machine under a 16-CPU quota is throttled for the rest of a
// scheduling period whenever the copy threads, the caller and the HIP
// runtime's threads together overrun it — round 4's occasional pageable round
// at half the median rate.
static long usable_cpus() {
    long n = (long)std::thread::hardware_concurrency();
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof set, &set) == 0) n = std::min(n > 0 ? n : 1L, (long)CPU_COUNT(&set));
    if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[32] = {0};
        long period = 0;
        if (fscanf(f, "%31s %ld", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0) {
            const long quota = atol(q) / period;
            if (quota > 0) n = std::min(n, quota);
        }
        fclose(f);
    }
    return std::max(1L, n);
}

int host_threads();
void host_copy(ono_ring *r, void *dst, const void *src, size_t bytes) {
    if (!r->pool) r->pool.reset(new HostPool(host_threads(), r->device));
    r->pool->copy(dst, src, bytes);
}

int host_threads() {
    const char *e = getenv("ONO_HOST_THREADS");
    if (e && atol(e) > 0) return (int)std::min(atol(e), usable_cpus());
    // default: 16, leaving two CPUs of the quota to the caller's thread and the runtime's
    return (int)std::max(1L, std::min(16L, usable_cpus() - 2));
}

}  // namespace ono

namespace {

// ---- the plan interpreter ----------------------------------------------
// Every RCCL schedule (ALLREDUCE and its segments, HOPS, DIRECT, the PS step)
// is a list of steps built by ono_plan.cpp and executed here; the same lists
// are checked and run on the CPU by tests/test_plans.py.  Schedules:
//   HOPS    worker_ring.rs:112-204 as ncclSend/ncclRecv pairs, with the fused
//           codec kernels between hops:
//             scatter hop 0      encode_zero        (:122, :133)
//             scatter hops 1..   add_encode_zero    (:141-143 then :122, :133)
//             last scatter hop   add_finish         (:141-143, :166, :191-193, ÷n)
//             gather hops        decode_scale       (:200, ÷n) + forward the
//                                received bytes (f16(f32(h)) == h)
//   DIRECT  built for the fully connected xGMI of one node (every GPU pair has
//           its own link): instead of n-1 dependent hops over one link,
//           1. all-to-all (grouped ncclSend/ncclRecv to every peer): rank q
//              receives every rank's slice of the chunk it owns, c = q+1
//              (worker_ring.rs:162-166);
//           2. one fused kernel on the owner replays the reference chain for
//              chunk c in the reference order c, c+1, ..., c+n-1 (DirectOp):
//              bit-exact with the hop ring for both wires at every n;
//              grad[c] = chain / n; own slice zeroed;
//           3. the rest of the residual is zeroed on the side stream, beside
//           4. the all-gather of the owned chunk (f32 values, or the f16
//              message the reference forwards hop by hop), decoded and divided
//              on arrival.  Bytes per rank on the wire: (n-1)/n (4 + 4) N for
//              f32, (n-1)/n (4 + 2) N for f16 — all links busy at once.
//   ALLREDUCE  ncclAllReduce(sum) + the fused finaliser (÷n, residual = 0);
//           with k segments the finaliser of segment j runs on the side stream
//           while segment j+1 is on the wire.
struct PlanCtx {
    void *base[ONO_PB_COUNT] = {};
    int wire = ONO_WIRE_F32;
    const OptLaunch *opt = nullptr;  // OPT_UPDATE: the PS optimizer and its shard state
    float *v = nullptr, *s = nullptr;
};

size_t plan_esize(const PlanCtx &c, int buf) {
    switch (buf) {
    case ONO_PB_WIRE0:
    case ONO_PB_WIRE1: return c.wire == ONO_WIRE_F16 ? 2 : 4;
    case ONO_PB_GSTAGE:
    case ONO_PB_MSG: return 2;
    default: return 4;
    }
}
void *plan_ptr(const PlanCtx &c, const ono_plan_step &st, int i) {
    const int b = st.buf[i];
    if (b < 0 || b >= ONO_PB_COUNT || !c.base[b]) return nullptr;
    return static_cast<char *>(c.base[b]) + st.off[i] * plan_esize(c, b);
}

int side_stream(ono_ring *r) {
    if (!r->astream) {
        ONO_HIP(hipStreamCreateWithFlags(&r->astream, hipStreamNonBlocking));
        ONO_HIP(hipEventCreateWithFlags(&r->ev_ajoin, hipEventDisableTiming));
    }
    return ONO_OK;
}

template <class W>
hipError_t plan_kernel(const PlanCtx &c, const ono_plan_step &st, hipStream_t q) {
    auto p = [&](int i) { return plan_ptr(c, st, i); };
    const size_t n = st.count;
    switch (st.op) {
    case ONO_POP_ENCODE_ZERO:
        return launch_encode_zero<W>(static_cast<W *>(p(0)), static_cast<float *>(p(1)), n, q);
    case ONO_POP_ADD_ENCODE_ZERO:
        return launch_add_encode_zero<W>(static_cast<W *>(p(0)), static_cast<float *>(p(1)),
                                         static_cast<const W *>(p(2)), n, q);
    case ONO_POP_ADD_FINISH:
        return launch_add_finish<W>(static_cast<float *>(p(0)), static_cast<W *>(p(1)), static_cast<float *>(p(2)),
                                    static_cast<const W *>(p(3)), n, st.divisor, q);
    case ONO_POP_DECODE_SCALE:
        return launch_decode_scale<W>(static_cast<float *>(p(0)), static_cast<const W *>(p(1)), n, st.divisor, q);
    case ONO_POP_DIRECT: {
        const float *ins[ONO_MAX_INPUTS];
        const int k = st.nref - 2;
        if (k < 1 || k > ONO_MAX_INPUTS) return hipErrorInvalidValue;
        for (int j = 0; j < k; j++) ins[j] = static_cast<const float *>(p(2 + j));
        return launch_direct<W>(static_cast<float *>(p(0)), static_cast<W *>(p(1)), ins, k, n, st.divisor,
                                st.flag != 0, q);
    }
    case ONO_POP_SCALE_ZERO:
        return launch_scale_zero(static_cast<float *>(p(0)), static_cast<const float *>(p(1)), n, st.divisor,
                                 static_cast<float *>(p(2)), q);
    case ONO_POP_OPT_UPDATE:
        if (!c.opt) return hipErrorInvalidValue;
        return launch_opt_update(*c.opt, static_cast<float *>(p(0)), static_cast<float *>(p(1)), c.v, c.s, n,
                                 st.flag != 0, q);
    default:
        return hipErrorInvalidValue;
    }
}

ncclDataType_t plan_nccl_type(int dtype) { return dtype == ONO_WIRE_F16 ? ncclFloat16 : ncclFloat32; }

int run_plan(ono_ring *r, const std::vector<ono_plan_step> &plan, const PlanCtx &c, hipStream_t s) {
    size_t forks = 0;
    for (const auto &st : plan) forks += st.kind == ONO_PLAN_FORK;
    if (forks) {
        int rc = side_stream(r);
        if (rc) return rc;
        while (r->ev_seg.size() < forks) {
            hipEvent_t ev;
            ONO_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            r->ev_seg.push_back(ev);
        }
    }
    size_t fork = 0;
    EventPair grp;
    for (size_t i = 0; i < plan.size(); i++) {
        const ono_plan_step &st = plan[i];
        hipStream_t q = st.stream ? r->astream : s;
        switch (st.kind) {
        case ONO_PLAN_GROUP_BEGIN:
            if (r->aborted.load()) return set_error(ONO_E_ABORTED, "ring aborted");
            if (r->timer.on) ONO_HIP(r->timer.begin(s, grp, ONO_PHASE_RCCL));
            ONO_NCCL(ncclGroupStart());
            break;
        case ONO_PLAN_SEND:
            ONO_NCCL(ncclSend(plan_ptr(c, st, 0), st.count, plan_nccl_type(st.dtype), st.peer, r->comm, s));
            break;
        case ONO_PLAN_RECV:
            ONO_NCCL(ncclRecv(plan_ptr(c, st, 0), st.count, plan_nccl_type(st.dtype), st.peer, r->comm, s));
            break;
        case ONO_PLAN_GROUP_END:
            ONO_NCCL(ncclGroupEnd());
            if (r->timer.on) ONO_HIP(r->timer.end(s, grp));
            break;
        case ONO_PLAN_ALLREDUCE:
        case ONO_PLAN_REDUCE_SCATTER:
        case ONO_PLAN_ALL_GATHER: {
            if (r->aborted.load()) return set_error(ONO_E_ABORTED, "ring aborted");
            int rc = timed(r, s, ONO_PHASE_RCCL, [&]() -> int {
                const void *src = plan_ptr(c, st, 0);
                void *dst = plan_ptr(c, st, 1);
                if (st.kind == ONO_PLAN_ALLREDUCE)
                    ONO_NCCL(ncclAllReduce(src, dst, st.count, ncclFloat32, ncclSum, r->comm, s));
                else if (st.kind == ONO_PLAN_REDUCE_SCATTER)
                    ONO_NCCL(ncclReduceScatter(src, dst, st.count, ncclFloat32, ncclSum, r->comm, s));
                else
                    ONO_NCCL(ncclAllGather(src, dst, st.count, ncclFloat32, r->comm, s));
                return ONO_OK;
            });
            if (rc) return rc;
            break;
        }
        case ONO_PLAN_KERNEL:
            if (c.wire == ONO_WIRE_F16 && st.dtype == ONO_WIRE_F16)
                ONO_K(r, q, plan_kernel<uint16_t>(c, st, q));
            else
                ONO_K(r, q, plan_kernel<float>(c, st, q));
            break;
        case ONO_PLAN_MEMSET:
            ONO_HIP(dev_zero(plan_ptr(c, st, 0), st.count * plan_esize(c, st.buf[0]), q));
            break;
        case ONO_PLAN_COPY:
            ONO_HIP(dev_copy(plan_ptr(c, st, 0), plan_ptr(c, st, 1), st.count * plan_esize(c, st.buf[0]), q));
            break;
        case ONO_PLAN_FORK:
            ONO_HIP(hipEventRecord(r->ev_seg[fork], s));
            ONO_HIP(hipStreamWaitEvent(r->astream, r->ev_seg[fork], 0));
            fork++;
            break;
        case ONO_PLAN_JOIN:
            ONO_HIP(hipEventRecord(r->ev_ajoin, r->astream));
            ONO_HIP(hipStreamWaitEvent(s, r->ev_ajoin, 0));
            break;
        default:
            return set_error(ONO_E_ARG, "plan step %zu: kind %d", i, st.kind);
        }
    }
    return ONO_OK;
}

// AUTO: the f32 wire is one RCCL all-reduce; the f16 wire (the reference's
// exact arithmetic) takes the DIRECT schedule — bit-identical to the hop ring
// but over every link at once instead of 2(n-1) dependent single-link hops —
// up to ONO_MAX_INPUTS ranks, the hop ring beyond (and always on a TCP ring).
int resolved_algo(const ono_ring *r) {
    if (r->algo != ONO_ALGO_AUTO) return r->algo;
    if (r->wire == ONO_WIRE_F32) return ONO_ALGO_ALLREDUCE;
    return (r->fd_next < 0 && r->n <= ONO_MAX_INPUTS) ? ONO_ALGO_DIRECT : ONO_ALGO_HOPS;
}

int ar_segments(ono_ring *r) {
    if (r->segments <= 0) {
        const char *v = getenv("ONO_AR_SEGMENTS");
        const int k = v ? atoi(v) : 0;
        r->segments = k > 0 ? k : 4;
    }
    const size_t by_size = std::max<size_t>(1, r->size / (size_t(4) << 20));  // >= 16 MiB per segment
    return (int)std::min<size_t>((size_t)r->segments, by_size);
}

// n == 1 with ONO_ALGO_ALLREDUCE (tests, bench plumbing): a one-rank communicator
int ensure_comm(ono_ring *r) {
    if (r->comm) return ONO_OK;
    ncclUniqueId id;
    ONO_NCCL(ncclGetUniqueId(&id));
    ONO_NCCL(ncclCommInitRank(&r->comm, 1, id, 0));
    return ONO_OK;
}

// the direct schedule's buffers: all-to-all receive slots, f16 all-gather
// staging, the owner's f16 message
int alloc_direct(ono_ring *r) {
    if (r->rbuf) return ONO_OK;
    const size_t slot = r->maxc + 4;
    ONO_HIP(hipMalloc((void **)&r->rbuf, (size_t)r->n * slot * sizeof(float)));
    ONO_HIP(hipMalloc((void **)&r->gstage, (size_t)r->n * slot * sizeof(uint16_t)));
    ONO_HIP(hipMalloc((void **)&r->msg, slot * sizeof(uint16_t)));
    return ONO_OK;
}

// pull_grads over RCCL: the rank's plan for (algo, wire, segments), cached
int plan_pull_grads_impl(ono_ring *r, int algo, float *res, float *grad, hipStream_t s) {
    int rc = ONO_OK;
    if (algo == ONO_ALGO_ALLREDUCE && (rc = ensure_comm(r))) return rc;
    if (algo == ONO_ALGO_DIRECT && (rc = alloc_direct(r))) return rc;
    const int segs = algo == ONO_ALGO_ALLREDUCE ? ar_segments(r) : 0;
    if (r->plan.empty() || r->plan_algo != algo || r->plan_segments != segs) {
        std::vector<ono_plan_step> p;
        if ((rc = plan_pull_grads(p, algo, r->wire, r->pos, r->n, r->size, segs))) return rc;
        r->plan.swap(p);
        r->plan_algo = algo;
        r->plan_segments = segs;
    }
    PlanCtx c;
    c.wire = r->wire;
    c.base[ONO_PB_RESIDUAL] = res;
    c.base[ONO_PB_GRAD] = grad;
    c.base[ONO_PB_WIRE0] = r->wbuf[0];
    c.base[ONO_PB_WIRE1] = r->wbuf[1];
    c.base[ONO_PB_RBUF] = r->rbuf;
    c.base[ONO_PB_GSTAGE] = r->gstage;
    c.base[ONO_PB_MSG] = r->msg;
    return run_plan(r, r->plan, c, s);
}

int pull_grads_impl(ono_ring *r, float *res, float *grad, hipStream_t s) {
    if (r->aborted.load()) return set_error(ONO_E_ABORTED, "ring aborted");
    if (r->n == 1 && r->algo != ONO_ALGO_ALLREDUCE) {  // worker_ring.rs:166-171: grad = residual; residual = 0; no ÷
        ONO_K(r, s, launch_scale_zero(grad, res, r->size, 1.0f, res, s));
        return ONO_OK;
    }
    const int algo = resolved_algo(r);
    switch (algo) {
    case ONO_ALGO_HOPS:
        if (r->fd_next >= 0) return tcp_pull_grads(r, res, grad, s);
        return plan_pull_grads_impl(r, algo, res, grad, s);
    case ONO_ALGO_ALLREDUCE:
    case ONO_ALGO_DIRECT:
        return plan_pull_grads_impl(r, algo, res, grad, s);
    case ONO_ALGO_XGMI:
        return xgmi_pull_grads(r, res, grad, s);
    default:
        return set_error(ONO_E_ARG, "algo %d", r->algo);
    }
}

}  // namespace

extern "C" {

int ono_ring_unique_id(uint8_t uid[ONO_UID_BYTES]) {
    if (!uid) return set_error(ONO_E_ARG, "uid is NULL");
    ncclUniqueId id;
    ONO_NCCL(ncclGetUniqueId(&id));
    memcpy(uid, &id, sizeof id);
    return ONO_OK;
}

static int ring_validate(ono_ring **out, int pos, int nranks, size_t size, int wire) {
    if (!out) return set_error(ONO_E_ARG, "out is NULL");
    *out = nullptr;
    if (nranks < 1 || pos < 0 || pos >= nranks) return set_error(ONO_E_ARG, "pos=%d nranks=%d", pos, nranks);
    if (wire != ONO_WIRE_F32 && wire != ONO_WIRE_F16) return set_error(ONO_E_ARG, "wire=%d", wire);
    if (size < (size_t)nranks)  // reference: chunks[pos] out of bounds (worker_ring.rs:120-122)
        return set_error(ONO_E_SIZE, "bucket of %zu elements cannot be split over %d ranks", size, nranks);
    return ONO_OK;
}

int ono_ring_create(ono_ring **out, int pos, int nranks, size_t size, int device,
                    const uint8_t *uid, int wire) {
    int vrc = ring_validate(out, pos, nranks, size, wire);
    if (vrc) return vrc;
    if (nranks > 1 && !uid) return set_error(ONO_E_ARG, "uid required for nranks > 1");
    ono_ring *r = new ono_ring();
    r->pos = pos; r->n = nranks; r->size = size; r->device = device; r->wire = wire;
    r->off = split_chunks(size, (size_t)nranks);
    r->maxc = r->off[1] - r->off[0];
    DeviceGuard g(device);
    auto fail = [&](int rc) { ono_ring_destroy(r); return rc; };
    hipError_t e;
    if ((e = hipSetDevice(device)) != hipSuccess) return fail(hip_error(e, "hipSetDevice", __FILE__, __LINE__));
    // the buckets are zeroed by the library's fill kernel on the ring's own stream, waited for before the
    // ring is handed out (a null-stream hipMemset is not ordered with the non-blocking streams the host-fed
    // forms run on)
    if ((e = hipMalloc((void **)&r->grad, size * sizeof(float))) != hipSuccess ||
        (e = hipMalloc((void **)&r->residual, size * sizeof(float))) != hipSuccess ||
        (e = hipStreamCreateWithFlags(&r->hstream, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipStreamCreateWithFlags(&r->cstream, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipStreamCreateWithFlags(&r->dstream, hipStreamNonBlocking)) != hipSuccess ||
        (e = dev_zero(r->grad, size * sizeof(float), r->cstream)) != hipSuccess ||
        (e = dev_zero(r->residual, size * sizeof(float), r->cstream)) != hipSuccess ||
        (e = hipStreamSynchronize(r->cstream)) != hipSuccess)
        return fail(hip_error(e, "bucket allocation", __FILE__, __LINE__));
    if (nranks > 1) {  // hop-ring wire buffers, sized for either wire
        for (int b = 0; b < 2; b++)
            if ((e = hipMalloc(&r->wbuf[b], (r->maxc + 4) * sizeof(float))) != hipSuccess)
                return fail(hip_error(e, "wire buffer allocation", __FILE__, __LINE__));
    }
    if (nranks > 1) {
        ncclUniqueId id;
        memcpy(&id, uid, sizeof id);
        ncclResult_t nr = ncclCommInitRank(&r->comm, nranks, id, pos);
        if (nr != ncclSuccess)
            return fail(set_error(ONO_E_RCCL, "ncclCommInitRank(rank %d of %d): %s", pos, nranks,
                                  ncclGetErrorString(nr)));
    }
    *out = r;
    return ONO_OK;
}

int ono_ring_destroy(ono_ring *r) {
    if (!r) return ONO_OK;
    {
        DeviceGuard g(r->device);
        xgmi_free(r);
        if (r->hstream) (void)hipStreamSynchronize(r->hstream);
        if (r->comm) {
            if (r->aborted.load()) ncclCommAbort(r->comm);
            else ncclCommDestroy(r->comm);
        }
        r->timer.destroy();
        (void)hipFree(r->grad);
        (void)hipFree(r->residual);
        (void)hipFree(r->wbuf[0]);
        (void)hipFree(r->wbuf[1]);
        for (hipStream_t st : {r->cstream, r->dstream})
            if (st) (void)hipStreamSynchronize(st);
        if (r->pin_in) (void)hipHostFree(r->pin_in);
        if (r->pin_out) (void)hipHostFree(r->pin_out);
        for (hipEvent_t ev : r->tx_ev) (void)hipEventDestroy(ev);
        for (uint8_t *z : r->zc)
            if (z) (void)hipHostFree(z);
        for (uint8_t *h : {r->tx, r->rx, r->sp_rx, r->sp_tx})
            if (h) (void)hipHostFree(h);
        (void)hipFree(r->sp_dev);
        (void)hipFree(r->sp_tmp);
        sample_ahead_free(r->ahead);  // (joins its thread before its buffer goes)
        if (r->sample_idx) (void)hipHostFree(r->sample_idx);
        (void)hipFree(r->sp_idx_dev);
        (void)hipFree(r->sp_t_dev);
        (void)hipFree(r->sp_rx_dev);
        if (r->sp_status) (void)hipHostFree(r->sp_status);
        if (r->tcp_word) (void)hipHostFree(r->tcp_word);
        if (r->dn_arrive) (void)hipFree(r->dn_arrive);
        for (auto &reg : r->registered) (void)hipHostUnregister(reg.first);
        for (auto *v : {&r->ev_h, &r->ev_c, &r->ev_d})
            for (hipEvent_t ev : *v) (void)hipEventDestroy(ev);
        if (r->astream) (void)hipStreamSynchronize(r->astream);
        for (hipEvent_t ev : r->ev_seg) (void)hipEventDestroy(ev);
        if (r->ev_ajoin) (void)hipEventDestroy(r->ev_ajoin);
        (void)hipFree(r->rbuf);
        (void)hipFree(r->gstage);
        (void)hipFree(r->msg);
        for (hipStream_t st : {r->hstream, r->cstream, r->dstream, r->astream})
            if (st) (void)hipStreamDestroy(st);
    }
    delete r;
    return ONO_OK;
}

float *ono_ring_grad(ono_ring *r) { return r ? r->grad : nullptr; }
float *ono_ring_residual(ono_ring *r) { return r ? r->residual : nullptr; }
size_t ono_ring_size(const ono_ring *r) { return r ? r->size : 0; }

int ono_ring_acc_residual(ono_ring *r, const float *grad_dev, void *stream) {
    if (!r || !grad_dev) return set_error(ONO_E_ARG, "NULL argument");
    DeviceGuard g(r->device);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    ONO_K(r, s, launch_acc(r->residual, grad_dev, r->size, s, true));
    return ONO_OK;
}

int ono_ring_pull_grads(ono_ring *r, void *stream) {
    if (!r) return set_error(ONO_E_ARG, "ring is NULL");
    DeviceGuard g(r->device);
    return pull_grads_impl(r, r->residual, r->grad, reinterpret_cast<hipStream_t>(stream));
}

int ono_ring_pull_grads_dev(ono_ring *r, float *res, float *grad, size_t n, void *stream) {
    if (!r || !res || !grad) return set_error(ONO_E_ARG, "NULL argument");
    if (n != r->size) return set_error(ONO_E_SIZE, "buffer of %zu elements, ring of %zu", n, r->size);
    if (res == grad) return set_error(ONO_E_ARG, "residual and grad must not alias");
    DeviceGuard g(r->device);
    return pull_grads_impl(r, res, grad, reinterpret_cast<hipStream_t>(stream));
}

// ---- host-fed form (buckets arrive from comms/ in host memory)
// Chunked three-stage pipeline: H2D (hstream) -> reduce (cstream: per-chunk RCCL
// all-reduce + finalise, or copy+zero at n = 1) -> D2H (dstream), chunks of
// ONO_HOST_CHUNK_MIB (16 MiB).  Registered caller buffers (ono_ring_register_host)
// are DMA'd in place; others go through kSlots pinned bounce slots whose CPU
// copies overlap the DMA of other chunks.  The host residual is zeroed by the
// CPU as soon as its chunk has left for the device.  The f16 wire runs the
// exact hop schedule on the whole bucket (chunking would move chunk owners).
static constexpr int kSlots = 3;

static size_t host_chunk_elems() {
    static size_t v = [] {
        const char *e = getenv("ONO_HOST_CHUNK_MIB");
        long m = e ? atol(e) : 16;
        return (size_t)(m > 0 ? m : 16) << 18;  // MiB -> f32 elements
    }();
    return v;
}

static bool is_registered(ono_ring *r, const void *p, size_t bytes) {
    for (auto &reg : r->registered)
        if ((const char *)p >= (const char *)reg.first &&
            (const char *)p + bytes <= (const char *)reg.first + reg.second)
            return true;
    return false;
}

static int ensure_events(ono_ring *r, size_t nchunks) {
    for (auto *v : {&r->ev_h, &r->ev_c, &r->ev_d})
        while (v->size() < nchunks) {
            hipEvent_t ev;  // ev_c: a chunk's result, read next by the D2H copy
            ONO_HIP(hipEventCreateWithFlags(&ev, v == &r->ev_c ? copy_event_flags() : hipEventDisableTiming));
            v->push_back(ev);
        }
    return ONO_OK;
}

// reduce one chunk [lo, lo+len) of the device buckets on cstream
static int reduce_chunk(ono_ring *r, size_t lo, size_t len) {
    hipStream_t s = r->cstream;
    if (r->n == 1) {
        ONO_HIP(launch_scale_zero(r->grad + lo, r->residual + lo, len, 1.0f, r->residual + lo, s));
        return ONO_OK;
    }
    ONO_NCCL(ncclAllReduce(r->residual + lo, r->grad + lo, len, ncclFloat32, ncclSum, r->comm, s));
    ONO_HIP(launch_scale_zero(r->grad + lo, r->grad + lo, len, (float)r->n, r->residual + lo, s));
    return ONO_OK;
}

extern "C" int ono_ring_register_host(ono_ring *r, void *p, size_t bytes) {
    if (!r || !p || !bytes) return set_error(ONO_E_ARG, "NULL argument");
    std::lock_guard<std::mutex> lk(r->mu);
    if (is_registered(r, p, bytes)) return ONO_OK;
    DeviceGuard g(r->device);
    ONO_HIP(hipHostRegister(p, bytes, hipHostRegisterDefault));
    r->registered.emplace_back(p, bytes);
    return ONO_OK;
}

extern "C" int ono_ring_unregister_host(ono_ring *r, void *p) {
    if (!r || !p) return set_error(ONO_E_ARG, "NULL argument");
    std::lock_guard<std::mutex> lk(r->mu);
    DeviceGuard g(r->device);
    for (size_t i = 0; i < r->registered.size(); i++)
        if (r->registered[i].first == p) {
            ONO_HIP(hipHostUnregister(p));
            r->registered.erase(r->registered.begin() + (long)i);
            return ONO_OK;
        }
    return set_error(ONO_E_ARG, "pointer was not registered");
}

// Host-fed round of the exact RCCL schedules (HOPS, DIRECT), as the xGMI form
// does it (ono_xgmi.cpp): sub-round j takes elements [j sub, (j+1) sub) of
// every chunk, so every element keeps its owner and its chain (the result is
// the whole-bucket round's bit for bit) while the H2D of sub-round j+1
// (hstream), the exchange of j (cstream) and the D2H of j-1 (dstream) overlap.
// The host residual is zeroed once its sub-round has reached HBM.
static int exact_pull_grads_host(ono_ring *r, int algo, float *res_host, float *grad_host) {
    int rc = algo == ONO_ALGO_DIRECT ? alloc_direct(r) : ONO_OK;
    if (rc) return rc;
    const size_t want = std::max<size_t>(1, host_chunk_elems() / (size_t)r->n);
    const size_t S = plan_sub_rounds(r->n, r->size, want), sub = plan_sub_elems(want);
    if ((rc = ensure_events(r, S))) return rc;
    const int n = r->n;
    std::vector<size_t> st(n), ln(n);
    auto piece = [&](size_t j) {
        for (int q = 0; q < n; q++) {
            const size_t L = r->off[q + 1] - r->off[q], lo = std::min(L, j * sub);
            st[q] = r->off[q] + lo;
            ln[q] = std::min(L - lo, sub);
        }
    };
    PlanCtx c;
    c.wire = r->wire;
    c.base[ONO_PB_RESIDUAL] = r->residual;
    c.base[ONO_PB_GRAD] = r->grad;
    c.base[ONO_PB_WIRE0] = r->wbuf[0];
    c.base[ONO_PB_WIRE1] = r->wbuf[1];
    c.base[ONO_PB_RBUF] = r->rbuf;
    c.base[ONO_PB_GSTAGE] = r->gstage;
    c.base[ONO_PB_MSG] = r->msg;
    auto zero_host = [&](size_t j) -> int {  // sub-round j has reached HBM: zero its host residual
        ONO_HIP(hipEventSynchronize(r->ev_h[j]));
        piece(j);
        for (int q = 0; q < n; q++)
            if (ln[q]) memset(res_host + st[q], 0, ln[q] * sizeof(float));
        return ONO_OK;
    };
    auto rounds = [&]() -> int {
        std::vector<ono_plan_step> plan;
        for (size_t j = 0; j < S; j++) {
            piece(j);
            for (int q = 0; q < n; q++)
                if (ln[q])
                    ONO_HIP(hipMemcpyAsync(r->residual + st[q], res_host + st[q], ln[q] * sizeof(float),
                                           hipMemcpyHostToDevice, r->hstream));
            ONO_HIP(hipEventRecord(r->ev_h[j], r->hstream));
            ONO_HIP(hipStreamWaitEvent(r->cstream, r->ev_h[j], 0));
            int rc2 = plan_pull_grads_sub(plan, algo, r->wire, r->pos, n, r->size, want, j);
            if (!rc2) rc2 = run_plan(r, plan, c, r->cstream);
            if (rc2) return rc2;
            ONO_HIP(hipEventRecord(r->ev_c[j], r->cstream));
            ONO_HIP(hipStreamWaitEvent(r->dstream, r->ev_c[j], 0));
            for (int q = 0; q < n; q++)
                if (ln[q])
                    ONO_HIP(hipMemcpyAsync(grad_host + st[q], r->grad + st[q], ln[q] * sizeof(float),
                                           hipMemcpyDeviceToHost, r->dstream));
            ONO_HIP(hipEventRecord(r->ev_d[j], r->dstream));
            if (j > 0 && (rc2 = zero_host(j - 1))) return rc2;
        }
        return zero_host(S - 1);
    };
    rc = rounds();
    // every copy into or out of the caller's buffers is done before we return, failed or not
    const hipError_t e1 = hipStreamSynchronize(r->hstream), e2 = hipStreamSynchronize(r->cstream),
                     e3 = hipStreamSynchronize(r->dstream);
    if (rc) return rc;
    for (hipError_t e : {e1, e2, e3})
        if (e != hipSuccess) return hip_error(e, "host-fed exchange round", __FILE__, __LINE__);
    return ONO_OK;
}

int ono_ring_pull_grads_host(ono_ring *r, float *res_host, float *grad_host, size_t n) {
    if (!r || !res_host || !grad_host) return set_error(ONO_E_ARG, "NULL argument");
    if (n != r->size) return set_error(ONO_E_SIZE, "buffer of %zu elements, ring of %zu", n, r->size);
    if (r->aborted.load()) return set_error(ONO_E_ABORTED, "ring aborted");
    std::lock_guard<std::mutex> lk(r->mu);
    DeviceGuard g(r->device);
    const size_t bytes = n * sizeof(float);
    const bool reg = is_registered(r, res_host, bytes) && is_registered(r, grad_host, bytes);
    const size_t CH = host_chunk_elems();

    if (r->n > 1 && resolved_algo(r) == ONO_ALGO_XGMI)  // sub-round pipeline (ono_xgmi.cpp)
        return xgmi_pull_grads_host(r, res_host, grad_host, CH, reg);
    const int algo = resolved_algo(r);
    if (r->n > 1 && (algo == ONO_ALGO_HOPS || algo == ONO_ALGO_DIRECT) && r->fd_next < 0 && r->sparse_r <= 0.0f)
        return exact_pull_grads_host(r, algo, res_host, grad_host);  // sub-round pipeline
    if (r->n > 1 && algo != ONO_ALGO_ALLREDUCE) {  // whole-bucket: the TCP edge (its own pieces), sparse mode
        ONO_HIP(hipMemcpyAsync(r->residual, res_host, bytes, hipMemcpyHostToDevice, r->cstream));
        int rc = pull_grads_impl(r, r->residual, r->grad, r->cstream);
        if (rc) return rc;
        ONO_HIP(hipMemcpyAsync(grad_host, r->grad, bytes, hipMemcpyDeviceToHost, r->cstream));
        if (r->sparse_r > 0.0f)  // SparseCapable: the residual keeps what was not sent (worker_ring.rs:126-133)
            ONO_HIP(hipMemcpyAsync(res_host, r->residual, bytes, hipMemcpyDeviceToHost, r->cstream));
        ONO_HIP(hipStreamSynchronize(r->cstream));
        if (r->sparse_r <= 0.0f) memset(res_host, 0, bytes);
        return ONO_OK;
    }

    const size_t nch = (n + CH - 1) / CH;
    int rc = ensure_events(r, nch);
    if (rc) return rc;
    if (!reg && !r->pool) r->pool.reset(new HostPool(host_threads(), r->device));
    if (!reg && !r->pin_in) {
        ONO_HIP(hipHostMalloc((void **)&r->pin_in, kSlots * CH * sizeof(float), hipHostMallocDefault));
        ONO_HIP(hipHostMalloc((void **)&r->pin_out, kSlots * CH * sizeof(float), hipHostMallocDefault));
    }
    auto lo_of = [&](size_t c) { return c * CH; };
    auto len_of = [&](size_t c) { return std::min(CH, n - c * CH); };
    auto drain_out = [&](size_t c) -> int {  // bounce path: wait D2H of chunk c, copy to caller
        ONO_HIP(hipEventSynchronize(r->ev_d[c]));
        r->pool->copy(grad_host + lo_of(c), r->pin_out + (c % kSlots) * CH, len_of(c) * sizeof(float));
        return ONO_OK;
    };
    for (size_t c = 0; c < nch; c++) {
        const size_t lo = lo_of(c), len = len_of(c), cb = len * sizeof(float);
        const float *src = res_host + lo;
        float *dst = grad_host + lo;
        if (!reg) {
            if (c >= (size_t)kSlots && (rc = drain_out(c - kSlots))) return rc;  // slot free again
            float *slot_in = r->pin_in + (c % kSlots) * CH;
            r->pool->copy(slot_in, src, cb);
            src = slot_in;
            dst = r->pin_out + (c % kSlots) * CH;
        }
        ONO_HIP(hipMemcpyAsync(r->residual + lo, src, cb, hipMemcpyHostToDevice, r->hstream));
        ONO_HIP(hipEventRecord(r->ev_h[c], r->hstream));
        ONO_HIP(hipStreamWaitEvent(r->cstream, r->ev_h[c], 0));
        if ((rc = reduce_chunk(r, lo, len))) return rc;
        ONO_HIP(hipEventRecord(r->ev_c[c], r->cstream));
        ONO_HIP(hipStreamWaitEvent(r->dstream, r->ev_c[c], 0));
        ONO_HIP(hipMemcpyAsync(dst, r->grad + lo, cb, hipMemcpyDeviceToHost, r->dstream));
        ONO_HIP(hipEventRecord(r->ev_d[c], r->dstream));
        if (!reg) {
            r->pool->zero(res_host + lo, cb);  // already copied to the bounce slot
        } else if (c > 0) {
            ONO_HIP(hipEventSynchronize(r->ev_h[c - 1]));  // chunk c-1 has reached HBM
            memset(res_host + lo_of(c - 1), 0, len_of(c - 1) * sizeof(float));  // one thread: leaves the
                                                                                 // host memory to the DMA
        }
    }
    if (reg) {
        ONO_HIP(hipEventSynchronize(r->ev_h[nch - 1]));
        memset(res_host + lo_of(nch - 1), 0, len_of(nch - 1) * sizeof(float));
        ONO_HIP(hipStreamSynchronize(r->dstream));
    } else {
        for (size_t c = nch > (size_t)kSlots ? nch - kSlots : 0; c < nch; c++)
            if ((rc = drain_out(c))) return rc;
    }
    return ONO_OK;
}

int ono_ring_allreduce_avg_dev(ono_ring *r, float *buf, size_t n, void *stream) {
    if (!r || !buf) return set_error(ONO_E_ARG, "NULL argument");
    if (n != r->size) return set_error(ONO_E_SIZE, "buffer of %zu elements, ring of %zu", n, r->size);
    DeviceGuard g(r->device);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (r->aborted.load()) return set_error(ONO_E_ABORTED, "ring aborted");
    if (r->n == 1) return ONO_OK;
    if (resolved_algo(r) == ONO_ALGO_ALLREDUCE) {
        int rc = timed(r, s, 1, [&]() -> int {
            ONO_NCCL(ncclAllReduce(buf, buf, n, ncclFloat32, ncclSum, r->comm, s));
            return ONO_OK;
        });
        if (rc) return rc;
        ONO_K(r, s, launch_scale_zero(buf, buf, n, (float)r->n, nullptr, s));
        return ONO_OK;
    }
    int rc = pull_grads_impl(r, buf, r->grad, s);
    if (rc) return rc;
    ONO_HIP(dev_copy(buf, r->grad, n * sizeof(float), s));
    return ONO_OK;
}

int ono_ring_set_algo(ono_ring *r, int algo) {
    if (!r) return set_error(ONO_E_ARG, "ring is NULL");
    if (algo < ONO_ALGO_AUTO || algo > ONO_ALGO_XGMI) return set_error(ONO_E_ARG, "algo %d", algo);
    if (r->n > 1 && !r->comm && r->fd_next < 0) {  // ono_ring_create_xgmi: no communicator
        if (algo != ONO_ALGO_XGMI && algo != ONO_ALGO_AUTO)
            return set_error(ONO_E_ARG, "an xGMI ring (no RCCL communicator) runs the xGMI schedule only");
        return ONO_OK;
    }
    if (algo == ONO_ALGO_XGMI && r->n > ONO_MAX_INPUTS)
        return set_error(ONO_E_ARG, "xGMI schedule supports up to %d ranks", ONO_MAX_INPUTS);
    if (algo == ONO_ALGO_ALLREDUCE && r->wire == ONO_WIRE_F16)
        return set_error(ONO_E_ARG, "an RCCL all-reduce cannot carry the f16 wire semantics");
    if (algo == ONO_ALGO_DIRECT && r->n > ONO_MAX_INPUTS)
        return set_error(ONO_E_ARG, "direct schedule supports up to %d ranks", ONO_MAX_INPUTS);
    if (r->fd_next >= 0 && algo != ONO_ALGO_HOPS && algo != ONO_ALGO_AUTO)
        return set_error(ONO_E_ARG, "a TCP ring runs the reference hop schedule only");
    std::lock_guard<std::mutex> lk(r->mu);
    r->algo = r->fd_next >= 0 ? ONO_ALGO_HOPS : algo;
    return ONO_OK;
}

int ono_ring_set_pipeline(ono_ring *r, int segments) {
    if (!r) return set_error(ONO_E_ARG, "ring is NULL");
    if (segments < 0) return set_error(ONO_E_ARG, "segments %d", segments);
    std::lock_guard<std::mutex> lk(r->mu);
    r->segments = segments;  // 0: back to the default
    return ONO_OK;
}

int ono_ring_abort(ono_ring *r) {
    if (!r) return set_error(ONO_E_ARG, "ring is NULL");
    r->aborted.store(true);
    xgmi_abort(r);
    return ONO_OK;
}

int ono_ring_timing_enable(ono_ring *r, int enable) {
    if (!r) return set_error(ONO_E_ARG, "ring is NULL");
    std::lock_guard<std::mutex> lk(r->mu);
    DeviceGuard g(r->device);
    ONO_HIP(r->timer.drain());
    r->timer.on = enable != 0;
    r->timer.reset();
    return ONO_OK;
}

int ono_ring_timing_phases(ono_ring *r, double *ms, int64_t *count) {
    if (!r || !ms || !count) return set_error(ONO_E_ARG, "NULL argument");
    std::lock_guard<std::mutex> lk(r->mu);
    DeviceGuard g(r->device);
    ONO_HIP(r->timer.drain());
    for (int i = 0; i < ONO_PHASES; i++) {
        ms[i] = r->timer.phase_ms[i];
        count[i] = r->timer.phase_n[i];
    }
    return ONO_OK;
}

int ono_ring_timing_read(ono_ring *r, double *kernel_ms, int64_t *launches, double *coll_ms,
                         int64_t *colls) {
    if (!r) return set_error(ONO_E_ARG, "ring is NULL");
    std::lock_guard<std::mutex> lk(r->mu);
    DeviceGuard g(r->device);
    ONO_HIP(r->timer.drain());
    if (kernel_ms) *kernel_ms = r->timer.kernel_ms;
    if (launches) *launches = r->timer.kernels;
    if (coll_ms) *coll_ms = r->timer.coll_ms;
    if (colls) *colls = r->timer.colls;
    return ONO_OK;
}

}  // extern "C"

// ------------------------------------------------------------ local ring ----
// All ranks of one round on one device, lockstep.  Rank r at scatter step s
// reads the message rank r-1 produced at step s (parity s%2) and writes its
// own step-s+1 message (parity (s+1)%2).  The gather is each replica decoding
// the owner's final message — the exact bytes the reference forwards hop by
// hop (f16(f32(h)) == h).
template <class W>
static int local_ring(float *const *res, float *const *grad, int R, size_t n, hipStream_t s) {
    auto off = split_chunks(n, (size_t)R);
    if (off.size() - 1 < (size_t)R)
        return set_error(ONO_E_SIZE, "bucket of %zu elements cannot be split over %d ranks", n, R);
    const size_t maxc = off[1] - off[0], slot_elems = maxc + 4;
    auto len = [&](int c) { return off[c + 1] - off[c]; };
    W *msg = nullptr;
    ONO_HIP(hipMallocAsync((void **)&msg, 2 * (size_t)R * slot_elems * sizeof(W), s));
    auto M = [&](int par, int rank, int c) { return msg + ((size_t)par * R + rank) * slot_elems + ph(off[c]); };
    const float fn = (float)R;
    std::vector<int> idx(R);
    int rc = ONO_OK;
    auto chk = [&](hipError_t e) { if (e != hipSuccess && rc == ONO_OK) rc = hip_error(e, "local ring kernel", __FILE__, __LINE__); };
    for (int r = 0; r < R; r++) {
        idx[r] = r;
        chk(launch_encode_zero<W>(M(0, r, r), res[r] + off[r], len(r), s));
    }
    for (int st = 0; st < R - 1; st++) {
        for (int r = 0; r < R; r++) {
            int p = (r + R - 1) % R;
            int c = (idx[r] + R - 1) % R;
            const W *in = M(st & 1, p, c);
            if (st < R - 2) chk(launch_add_encode_zero<W>(M((st + 1) & 1, r, c), res[r] + off[c], in, len(c), s));
            else chk(launch_add_finish<W>(grad[r] + off[c], M((st + 1) & 1, r, c), res[r] + off[c], in, len(c), fn, s));
            idx[r] = c;
        }
    }
    const int fin = (R - 1) & 1;
    for (int r = 0; r < R; r++) {
        int own = (r + 1) % R;
        for (int c = 0; c < R; c++) {
            if (c == own) continue;
            int owner = (c + R - 1) % R;
            chk(launch_decode_scale<W>(grad[r] + off[c], M(fin, owner, c), len(c), fn, s));
        }
    }
    hipError_t e = hipFreeAsync(msg, s);
    if (rc) return rc;
    ONO_HIP(e);
    return ONO_OK;
}

// Co-resident direct schedule: for each chunk c the owner's kernel reads all
// ranks' slices in the reference order straight from HBM (no all-to-all on one
// device) and zeroes them; replicas then take the owner's f32 value or decode
// its f16 message.
template <class W>
static int local_direct(float *const *res, float *const *grad, int R, size_t n, hipStream_t s) {
    auto off = split_chunks(n, (size_t)R);
    if (off.size() - 1 < (size_t)R)
        return set_error(ONO_E_SIZE, "bucket of %zu elements cannot be split over %d ranks", n, R);
    constexpr bool f16 = sizeof(W) == 2;
    const size_t slot = off[1] - off[0] + 4;
    auto len = [&](int c) { return off[c + 1] - off[c]; };
    uint16_t *msg = nullptr;
    if (f16) ONO_HIP(hipMallocAsync((void **)&msg, (size_t)R * slot * sizeof(uint16_t), s));
    int rc = ONO_OK;
    auto chk = [&](hipError_t e) { if (e != hipSuccess && rc == ONO_OK) rc = hip_error(e, "local direct", __FILE__, __LINE__); };
    for (int c = 0; c < R; c++) {
        const int owner = (c + R - 1) % R;
        const float *ins[ONO_MAX_INPUTS];
        for (int k = 0; k < R; k++) ins[k] = res[(c + k) % R] + off[c];
        W *out = f16 ? reinterpret_cast<W *>(msg + (size_t)c * slot + ph(off[c])) : nullptr;
        chk(launch_direct<W>(grad[owner] + off[c], out, ins, R, len(c), (float)R, true, s));
    }
    for (int c = 0; c < R; c++) {
        const int owner = (c + R - 1) % R;
        for (int r = 0; r < R; r++) {
            if (r == owner) continue;
            if (f16)
                chk(launch_decode_scale<uint16_t>(grad[r] + off[c], msg + (size_t)c * slot + ph(off[c]), len(c),
                                                  (float)R, s));
            else
                chk(dev_copy(grad[r] + off[c], grad[owner] + off[c], len(c) * sizeof(float), s));
        }
    }
    if (f16) chk(hipFreeAsync(msg, s));
    return rc;
}

// ---------------------------------------------- plans on one device ------
// Every rank's exchange plan executed by co-resident ranks on ONE device, in
// lockstep: each rank runs its local steps (kernels, memsets, copies) up to
// its next communication step; when every rank is there, the group's sends
// are matched with the peers' receives (k-th send r -> q with q's k-th
// receive from r) and carried out as device copies, and a collective is
// carried out by the library's kernels (all-reduce / reduce-scatter: the sum
// over ranks in rank order; all-gather: copies).  One stream, so forks and
// joins are moot.  The kernel steps go through plan_kernel — the very code the
// RCCL interpreter (run_plan) launches — so this runs the N > 1 schedules'
// device work on a one-GPU box, where RCCL refuses two ranks per device.
namespace {

struct LocalRank {
    std::vector<ono_plan_step> plan;
    size_t pc = 0;
    PlanCtx ctx;
    std::vector<void *> owned;
};

bool is_comm(int kind) {
    return kind == ONO_PLAN_GROUP_BEGIN || kind == ONO_PLAN_ALLREDUCE || kind == ONO_PLAN_REDUCE_SCATTER ||
           kind == ONO_PLAN_ALL_GATHER;
}

size_t dtype_size(int dtype) { return dtype == ONO_WIRE_F16 ? 2 : 4; }

int run_local_step(LocalRank &R, const ono_plan_step &st, hipStream_t s) {
    const PlanCtx &c = R.ctx;
    switch (st.kind) {
    case ONO_PLAN_KERNEL:
        ONO_HIP(c.wire == ONO_WIRE_F16 && st.dtype == ONO_WIRE_F16 ? plan_kernel<uint16_t>(c, st, s)
                                                                   : plan_kernel<float>(c, st, s));
        return ONO_OK;
    case ONO_PLAN_MEMSET:
        ONO_HIP(dev_zero(plan_ptr(c, st, 0), st.count * plan_esize(c, st.buf[0]), s));
        return ONO_OK;
    case ONO_PLAN_COPY:
        ONO_HIP(dev_copy(plan_ptr(c, st, 0), plan_ptr(c, st, 1), st.count * plan_esize(c, st.buf[0]), s));
        return ONO_OK;
    case ONO_PLAN_FORK:
    case ONO_PLAN_JOIN:
        return ONO_OK;
    default:
        return set_error(ONO_E_ARG, "plan step kind %d outside a group", st.kind);
    }
}

int run_plans_local(std::vector<LocalRank> &ranks, hipStream_t s) {
    const int n = (int)ranks.size();
    for (;;) {
        int done = 0;
        for (LocalRank &R : ranks) {  // local work up to the next communication step
            while (R.pc < R.plan.size() && !is_comm(R.plan[R.pc].kind)) {
                int rc = run_local_step(R, R.plan[R.pc], s);
                if (rc) return rc;
                R.pc++;
            }
            if (R.pc == R.plan.size()) done++;
        }
        if (done == n) return ONO_OK;
        if (done) return set_error(ONO_E_ARG, "plans end at different communication steps");
        const int kind = ranks[0].plan[ranks[0].pc].kind;
        for (LocalRank &R : ranks)
            if (R.plan[R.pc].kind != kind) return set_error(ONO_E_ARG, "plans disagree on a communication step");
        if (kind == ONO_PLAN_GROUP_BEGIN) {
            struct P2P { int self, peer, k; const ono_plan_step *st; };
            std::vector<P2P> sends, recvs;
            for (int r = 0; r < n; r++) {
                LocalRank &R = ranks[r];
                std::vector<int> ns(n, 0), nr(n, 0);
                for (R.pc++; R.pc < R.plan.size() && R.plan[R.pc].kind != ONO_PLAN_GROUP_END; R.pc++) {
                    const ono_plan_step &st = R.plan[R.pc];
                    if (st.peer < 0 || st.peer >= n) return set_error(ONO_E_ARG, "peer %d", st.peer);
                    if (st.kind == ONO_PLAN_SEND) sends.push_back({r, st.peer, ns[st.peer]++, &st});
                    else if (st.kind == ONO_PLAN_RECV) recvs.push_back({r, st.peer, nr[st.peer]++, &st});
                    else return set_error(ONO_E_ARG, "step kind %d inside a group", st.kind);
                }
                if (R.pc == R.plan.size()) return set_error(ONO_E_ARG, "group without its end");
                R.pc++;  // past GROUP_END
            }
            if (sends.size() != recvs.size()) return set_error(ONO_E_ARG, "unmatched sends / receives");
            for (const P2P &rv : recvs) {
                const P2P *sd = nullptr;
                for (const P2P &x : sends)
                    if (x.self == rv.peer && x.peer == rv.self && x.k == rv.k) { sd = &x; break; }
                if (!sd || sd->st->count != rv.st->count || sd->st->dtype != rv.st->dtype)
                    return set_error(ONO_E_ARG, "receive of rank %d from %d has no matching send", rv.self, rv.peer);
                void *dst = plan_ptr(ranks[rv.self].ctx, *rv.st, 0);
                const void *src = plan_ptr(ranks[sd->self].ctx, *sd->st, 0);
                if (rv.st->count) ONO_HIP(dev_copy(dst, src, rv.st->count * dtype_size(rv.st->dtype), s));
            }
            continue;
        }
        // collectives: f32, the sum over ranks in rank order
        const size_t count = ranks[0].plan[ranks[0].pc].count;
        std::vector<const float *> src(n);
        for (int q = 0; q < n; q++) src[q] = static_cast<const float *>(plan_ptr(ranks[q].ctx, ranks[q].plan[ranks[q].pc], 0));
        for (int r = 0; r < n; r++) {
            const ono_plan_step &st = ranks[r].plan[ranks[r].pc];
            float *dst = static_cast<float *>(plan_ptr(ranks[r].ctx, st, 1));
            if (st.count != count) return set_error(ONO_E_ARG, "collective counts differ");
            if (kind == ONO_PLAN_ALL_GATHER) {
                for (int q = 0; q < n; q++)
                    if (count) ONO_HIP(dev_copy(dst + (size_t)q * count, src[q], count * 4, s));
                continue;
            }
            std::vector<const float *> ins(n);
            for (int q = 0; q < n; q++) ins[q] = src[q] + (kind == ONO_PLAN_REDUCE_SCATTER ? (size_t)r * count : 0);
            if (n > ONO_MAX_INPUTS) return set_error(ONO_E_ARG, "%d ranks", n);
            if (count) ONO_HIP(launch_sum_scale(dst, ins.data(), n, count, 1.0f, s));
        }
        for (LocalRank &R : ranks) R.pc++;
    }
}

int alloc_plan_buffers(std::vector<LocalRank> &ranks, int n, size_t size, size_t nparams, int wire) {
    uint64_t cnt[ONO_PB_COUNT];
    plan_buffers(n, size, nparams, cnt);
    for (LocalRank &R : ranks) {
        R.ctx.wire = wire;
        for (int b : {ONO_PB_WIRE0, ONO_PB_WIRE1, ONO_PB_RBUF, ONO_PB_GSTAGE, ONO_PB_MSG}) {
            if (R.ctx.base[b]) continue;
            void *p = nullptr;
            const size_t bytes = std::max<size_t>(cnt[b] * plan_esize(R.ctx, b), 16);
            ONO_HIP(hipMalloc(&p, bytes));
            R.owned.push_back(p);
            R.ctx.base[b] = p;
        }
    }
    return ONO_OK;
}

void free_plan_buffers(std::vector<LocalRank> &ranks) {
    for (LocalRank &R : ranks)
        for (void *p : R.owned) (void)hipFree(p);
}

}  // namespace

extern "C" {

int ono_plan_run_local(int algo, int wire, int nranks, size_t size, int segments, float *const *residuals,
                       float *const *grads, void *stream) {
    if (!residuals || !grads || nranks < 1 || nranks > ONO_MAX_INPUTS)
        return set_error(ONO_E_ARG, "nranks must be in [1, %d]", ONO_MAX_INPUTS);
    for (int r = 0; r < nranks; r++)
        if (!residuals[r] || !grads[r]) return set_error(ONO_E_ARG, "NULL bucket for rank %d", r);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    std::vector<LocalRank> ranks(nranks);
    for (int r = 0; r < nranks; r++) {
        int rc = plan_pull_grads(ranks[r].plan, algo, wire, r, nranks, size, std::max(segments, 1));
        if (rc) return rc;
        ranks[r].ctx.base[ONO_PB_RESIDUAL] = residuals[r];
        ranks[r].ctx.base[ONO_PB_GRAD] = grads[r];
    }
    int rc = alloc_plan_buffers(ranks, nranks, size, 0, wire);
    if (!rc) rc = run_plans_local(ranks, s);
    const hipError_t e = hipStreamSynchronize(s);  // the scratch is freed below
    free_plan_buffers(ranks);
    if (rc) return rc;
    if (e != hipSuccess) return hip_error(e, "local plans", __FILE__, __LINE__);
    return ONO_OK;
}

int ono_plan_run_local_sub(int algo, int wire, int nranks, size_t size, size_t sub_elems, float *const *residuals,
                           float *const *grads, void *stream) {
    if (!residuals || !grads || nranks < 2 || nranks > ONO_MAX_INPUTS)
        return set_error(ONO_E_ARG, "nranks must be in [2, %d]", ONO_MAX_INPUTS);
    if (sub_elems == 0) return set_error(ONO_E_ARG, "sub_elems is 0 (the whole bucket: ono_plan_run_local)");
    for (int r = 0; r < nranks; r++)
        if (!residuals[r] || !grads[r]) return set_error(ONO_E_ARG, "NULL bucket for rank %d", r);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    std::vector<LocalRank> ranks(nranks);
    for (int r = 0; r < nranks; r++) {
        ranks[r].ctx.base[ONO_PB_RESIDUAL] = residuals[r];
        ranks[r].ctx.base[ONO_PB_GRAD] = grads[r];
    }
    int rc = alloc_plan_buffers(ranks, nranks, size, 0, wire);
    const size_t S = rc ? 0 : plan_sub_rounds(nranks, size, sub_elems);
    for (size_t j = 0; !rc && j < S; j++) {  // the sub-rounds one after another, as the host-fed round orders them
        for (int r = 0; r < nranks && !rc; r++) rc = plan_pull_grads_sub(ranks[r].plan, algo, wire, r, nranks, size,
                                                                         sub_elems, j);
        for (auto &R : ranks) R.pc = 0;
        if (!rc) rc = run_plans_local(ranks, s);
    }
    const hipError_t e = hipStreamSynchronize(s);  // the scratch is freed below
    free_plan_buffers(ranks);
    if (rc) return rc;
    if (e != hipSuccess) return hip_error(e, "local sub-round plans", __FILE__, __LINE__);
    return ONO_OK;
}

int ono_plan_run_local_ps(int nranks, size_t nparams, const float *const *grads, float *const *params,
                          float *const *shards, float *const *v, float *const *s_, const ono_opt_spec *opt,
                          float step_size, void *stream) {
    if (!grads || !params || !shards || !opt || nranks < 2 || nranks > ONO_MAX_INPUTS)
        return set_error(ONO_E_ARG, "bad arguments");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const size_t n = (size_t)nranks, C = (nparams + n - 1) / n;
    OptLaunch o{opt->kind, opt->lr, opt->momentum, opt->beta1, opt->beta2, opt->eps, step_size, (float)nranks};
    std::vector<LocalRank> ranks(nranks);
    std::vector<void *> pads;
    int rc = ONO_OK;
    for (int r = 0; r < nranks && !rc; r++) {
        LocalRank &R = ranks[r];
        rc = plan_ps_step(R.plan, r, nranks, nparams);
        R.ctx.base[ONO_PB_GIN] = const_cast<float *>(grads[r]);
        R.ctx.base[ONO_PB_PARAMS] = params[r];
        R.ctx.opt = &o;
        R.ctx.v = v ? v[r] : nullptr;
        R.ctx.s = s_ ? s_[r] : nullptr;
        // the padded copies: GPAD zero-filled, PPAD holding every shard (rank r's current shard at r C)
        void *gpad = nullptr, *ppad = nullptr, *gsh = nullptr;
        if (!rc && hipMalloc(&gpad, C * n * 4) == hipSuccess) pads.push_back(gpad); else rc = rc ? rc : ONO_E_HIP;
        if (!rc && hipMalloc(&ppad, C * n * 4) == hipSuccess) pads.push_back(ppad); else rc = rc ? rc : ONO_E_HIP;
        if (!rc && hipMalloc(&gsh, C * 4) == hipSuccess) pads.push_back(gsh); else rc = rc ? rc : ONO_E_HIP;
        if (!rc && (dev_zero(gpad, C * n * 4, s) != hipSuccess || dev_zero(ppad, C * n * 4, s) != hipSuccess))
            rc = ONO_E_HIP;
        const size_t lo = std::min(nparams, (size_t)r * C), len = std::min(nparams, lo + C) - lo;
        if (!rc && len && dev_copy(static_cast<float *>(ppad) + (size_t)r * C, shards[r], len * 4, s) != hipSuccess)
            rc = ONO_E_HIP;
        R.ctx.base[ONO_PB_GPAD] = gpad;
        R.ctx.base[ONO_PB_PPAD] = ppad;
        R.ctx.base[ONO_PB_GSHARD] = gsh;
    }
    if (rc == ONO_E_HIP) set_error(ONO_E_HIP, "local PS plan scratch");
    if (!rc) rc = run_plans_local(ranks, s);
    for (int r = 0; r < nranks && !rc; r++) {  // the updated shard back to the caller's state
        const size_t lo = std::min(nparams, (size_t)r * C), len = std::min(nparams, lo + C) - lo;
        if (len && dev_copy(shards[r], static_cast<float *>(ranks[r].ctx.base[ONO_PB_PPAD]) + (size_t)r * C,
                                  len * 4, s) != hipSuccess)
            rc = set_error(ONO_E_HIP, "shard copy-back");
    }
    const hipError_t e = hipStreamSynchronize(s);
    for (void *p : pads) (void)hipFree(p);
    if (rc) return rc;
    if (e != hipSuccess) return hip_error(e, "local PS plans", __FILE__, __LINE__);
    return ONO_OK;
}

int ono_local_direct_pull_grads(float *const *residuals, float *const *grads, int nranks, size_t n,
                                int wire, void *stream) {
    if (!residuals || !grads || nranks < 1 || nranks > ONO_MAX_INPUTS)
        return set_error(ONO_E_ARG, "nranks must be in [1, %d]", ONO_MAX_INPUTS);
    for (int r = 0; r < nranks; r++)
        if (!residuals[r] || !grads[r]) return set_error(ONO_E_ARG, "NULL bucket for rank %d", r);
    if (n < (size_t)nranks)
        return set_error(ONO_E_SIZE, "bucket of %zu elements cannot be split over %d ranks", n, nranks);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (nranks == 1) {
        ONO_HIP(launch_scale_zero(grads[0], residuals[0], n, 1.0f, residuals[0], s));
        return ONO_OK;
    }
    if (wire == ONO_WIRE_F16) return local_direct<uint16_t>(residuals, grads, nranks, n, s);
    if (wire == ONO_WIRE_F32) return local_direct<float>(residuals, grads, nranks, n, s);
    return set_error(ONO_E_ARG, "wire=%d", wire);
}

int ono_local_ring_pull_grads(float *const *residuals, float *const *grads, int nranks,
                              size_t n, int wire, void *stream) {
    if (!residuals || !grads || nranks < 1 || nranks > 4096) return set_error(ONO_E_ARG, "bad arguments");
    for (int r = 0; r < nranks; r++)
        if (!residuals[r] || !grads[r]) return set_error(ONO_E_ARG, "NULL bucket for rank %d", r);
    if (n < (size_t)nranks)
        return set_error(ONO_E_SIZE, "bucket of %zu elements cannot be split over %d ranks", n, nranks);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (nranks == 1) {
        ONO_HIP(launch_scale_zero(grads[0], residuals[0], n, 1.0f, residuals[0], s));
        return ONO_OK;
    }
    if (wire == ONO_WIRE_F16) return local_ring<uint16_t>(residuals, grads, nranks, n, s);
    if (wire == ONO_WIRE_F32) return local_ring<float>(residuals, grads, nranks, n, s);
    return set_error(ONO_E_ARG, "wire=%d", wire);
}

// --------------------------------------------------- multi-GPU PS mode -----
// Sharded synchronizer (BlockingStore + BarrierSync across n workers):
// reduce-scatter of the gradients (store.rs:84-91 accumulate) -> fused
// ÷nworkers + optimizer on the owned shard (shard.rs:74-92) -> all-gather of
// the parameters (store.rs:110-124 pull).  Shards are padded to ceil(N/n).
struct ono_ps {
    ono_ring *ring = nullptr;
    size_t nparams = 0, shard = 0, padded = 0;
    float *gpad = nullptr, *ppad = nullptr, *gshard = nullptr, *v = nullptr, *s = nullptr;
    OptLaunch opt{};
    float beta1_t = 1.0f, beta2_t = 1.0f;
    std::vector<ono_plan_step> plan;  // the RCCL step of this rank (n > 1)
};

int ono_ps_create(ono_ps **out, ono_ring *ring, const float *init, size_t nparams,
                  const ono_opt_spec *opt) {
    if (!out || !ring || !init || !opt) return set_error(ONO_E_ARG, "NULL argument");
    if (opt->kind < ONO_OPT_GD || opt->kind > ONO_OPT_ADD) return set_error(ONO_E_ARG, "optimizer kind %d", opt->kind);
    *out = nullptr;
    if (ring->fd_next >= 0) return set_error(ONO_E_ARG, "the sharded PS needs an RCCL ring, not a TCP ring");
    DeviceGuard g(ring->device);
    ono_ps *p = new ono_ps();
    p->ring = ring;
    p->nparams = nparams;
    const size_t n = (size_t)ring->n;
    p->shard = (nparams + n - 1) / n;
    p->padded = p->shard * n;
    p->opt = OptLaunch{opt->kind, opt->lr, opt->momentum, opt->beta1, opt->beta2, opt->eps, 0.0f, (float)ring->n};
    auto fail = [&](hipError_t e) { ono_ps_destroy(p); return hip_error(e, "ps allocation", __FILE__, __LINE__); };
    hipError_t e;
    const size_t pb = p->padded * sizeof(float), sb = p->shard * sizeof(float);
    if ((e = hipMalloc((void **)&p->gpad, pb)) != hipSuccess || (e = hipMemset(p->gpad, 0, pb)) != hipSuccess ||
        (e = hipMalloc((void **)&p->ppad, pb)) != hipSuccess || (e = hipMemset(p->ppad, 0, pb)) != hipSuccess ||
        (e = hipMalloc((void **)&p->gshard, sb)) != hipSuccess ||
        (e = hipMalloc((void **)&p->v, sb)) != hipSuccess || (e = hipMemset(p->v, 0, sb)) != hipSuccess ||
        (e = hipMalloc((void **)&p->s, sb)) != hipSuccess || (e = hipMemset(p->s, 0, sb)) != hipSuccess)
        return fail(e);
    if ((e = hipMemcpy(p->ppad, init, nparams * sizeof(float), hipMemcpyHostToDevice)) != hipSuccess) return fail(e);
    *out = p;
    return ONO_OK;
}

int ono_ps_destroy(ono_ps *p) {
    if (!p) return ONO_OK;
    {
        DeviceGuard g(p->ring->device);
        (void)hipFree(p->gpad); (void)hipFree(p->ppad); (void)hipFree(p->gshard); (void)hipFree(p->v); (void)hipFree(p->s);
    }
    delete p;
    return ONO_OK;
}

int ono_ps_step(ono_ps *p, const float *grad, float *params, void *stream) {
    if (!p || !grad || !params) return set_error(ONO_E_ARG, "NULL argument");
    ono_ring *r = p->ring;
    if (r->aborted.load()) return set_error(ONO_E_ABORTED, "ring aborted");
    DeviceGuard g(r->device);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const size_t N = p->nparams, C = p->shard;
    const size_t lo = std::min(N, (size_t)r->pos * C), hi = std::min(N, lo + C);
    // adam.rs:76-80 in f32 on the host.  The powers advance only when an update
    // is actually enqueued (a step refused before launching anything leaves
    // the bias correction where it was, as a reference update that never ran).
    OptLaunch o = p->opt;
    float b1t = p->beta1_t, b2t = p->beta2_t;
    if (o.kind == ONO_OPT_ADAM) {
        b1t *= o.beta1;
        b2t *= o.beta2;
        float bc1 = 1.0f - b1t, bc2 = 1.0f - b2t;
        o.step_size = o.lr * (std::sqrt(bc2) / bc1);
    }
    auto commit = [&](int rc) {
        if (rc == ONO_OK) {
            p->beta1_t = b1t;
            p->beta2_t = b2t;
        }
        return rc;
    };
    if (r->n > 1 && resolved_algo(r) == ONO_ALGO_XGMI)  // peer-access form, no padding needed
        return commit(xgmi_ps_step(r, grad, params, N, C, p->gshard, p->ppad + (size_t)r->pos * C, o, p->v, p->s, s));
    if (r->n > 1) {  // reduce-scatter -> fused update -> all-gather, as a plan (ono_plan.cpp)
        if (p->plan.empty()) {
            int rc = plan_ps_step(p->plan, r->pos, r->n, N);
            if (rc) return rc;
        }
        PlanCtx c;
        c.base[ONO_PB_GIN] = const_cast<float *>(grad);
        c.base[ONO_PB_GPAD] = p->gpad;
        c.base[ONO_PB_GSHARD] = p->gshard;
        c.base[ONO_PB_PPAD] = p->ppad;
        c.base[ONO_PB_PARAMS] = params;
        c.opt = &o;
        c.v = p->v;
        c.s = p->s;
        return commit(run_plan(r, p->plan, c, s));
    }
    // one worker: the store's update on the whole vector
    ONO_HIP(dev_copy(p->gshard, grad, N * sizeof(float), s));
    if (hi > lo) ONO_K(r, s, launch_opt_update(o, p->gshard, p->ppad, p->v, p->s, hi - lo, true, s));
    ONO_HIP(dev_copy(params, p->ppad, N * sizeof(float), s));
    return commit(ONO_OK);
}

}  // extern "C"
