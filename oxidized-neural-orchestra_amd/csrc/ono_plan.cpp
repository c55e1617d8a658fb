// ono_plan.cpp — the N > 1 exchange schedules as data (pure host code).
//
// Each builder returns the whole round of one rank as a list of steps:
// grouped sends / receives, RCCL collectives, the fused kernels between them,
// memsets, copies and the forks / joins of the side stream.  ono_ring.cpp
// executes the list (run_plan); tests/test_plans.py checks the lists of every
// rank against each other and runs them with host copies against the oracle,
// which is how these schedules are verified without an 8-GPU node.
//
// Reference: worker/src/middlewares/worker_ring.rs:82-204 (the hop order and
// the chunk ownership every schedule reproduces), middlewares/mod.rs:15-59
// (split_chunks), parameter_server/src/storage/blocking/store.rs:84-124 (the
// sharded store the PS plan distributes).
#include <algorithm>
#include <vector>

#include "ono_internal.h"
#include "ono_plan.h"

namespace ono {

namespace {

struct Ref {
    int buf;
    uint64_t off;
};
constexpr Ref kNone{ONO_PB_NONE, 0};

class Builder {
public:
    std::vector<ono_plan_step> steps;

    ono_plan_step &add(int kind) {
        steps.emplace_back();
        ono_plan_step &s = steps.back();
        s = ono_plan_step{};
        s.kind = kind;
        s.divisor = 1.0f;
        for (int i = 0; i < ONO_PLAN_REFS; i++) s.buf[i] = ONO_PB_NONE;
        return s;
    }
    static void ref(ono_plan_step &s, int i, Ref r) {
        s.buf[i] = r.buf;
        s.off[i] = r.off;
        if (i + 1 > s.nref) s.nref = i + 1;
    }
    void group_begin() { add(ONO_PLAN_GROUP_BEGIN); }
    void group_end() { add(ONO_PLAN_GROUP_END); }
    void p2p(int kind, int peer, Ref r, uint64_t count, int dtype) {
        ono_plan_step &s = add(kind);
        s.peer = peer;
        s.count = count;
        s.dtype = dtype;
        ref(s, 0, r);
    }
    void coll(int kind, Ref src, Ref dst, uint64_t count) {
        ono_plan_step &s = add(kind);
        s.count = count;
        s.dtype = ONO_WIRE_F32;
        ref(s, 0, src);
        ref(s, 1, dst);
    }
    ono_plan_step &kernel(int op, std::initializer_list<Ref> refs, uint64_t count, int dtype, float divisor = 1.0f,
                          int stream = 0) {
        ono_plan_step &s = add(ONO_PLAN_KERNEL);
        s.op = op;
        s.count = count;
        s.dtype = dtype;
        s.divisor = divisor;
        s.stream = stream;
        int i = 0;
        for (const Ref &r : refs) ref(s, i++, r);
        return s;
    }
    void memset(Ref r, uint64_t count, int stream) {
        ono_plan_step &s = add(ONO_PLAN_MEMSET);
        s.count = count;
        s.dtype = ONO_WIRE_F32;
        s.stream = stream;
        ref(s, 0, r);
    }
    void copy(Ref dst, Ref src, uint64_t count) {
        ono_plan_step &s = add(ONO_PLAN_COPY);
        s.count = count;
        s.dtype = ONO_WIRE_F32;
        ref(s, 0, dst);
        ref(s, 1, src);
    }
    void fork() { add(ONO_PLAN_FORK).stream = 1; }
    void join() { add(ONO_PLAN_JOIN); }
};

int mod(int x, int n) { return ((x % n) + n) % n; }

// The part of every chunk one round works on: st[c], ln[c] (the whole chunks
// for a whole-bucket round; a slice of each for a host-fed sub-round).  Steps
// over an empty piece are left out on both sides of every exchange.
struct Pieces {
    std::vector<size_t> st, ln;
    size_t slot;  // the receive-slot stride of the direct schedule (the largest chunk + 4)
    bool whole;   // the pieces are the chunks themselves
};

// worker_ring.rs:112-204 as ncclSend/ncclRecv pairs, the fused codec kernels
// between hops (see ono_ring.cpp's header for the kernel <-> line mapping).
void hops(Builder &b, int wire, int pos, int n, const Pieces &pc) {
    auto len = [&](int c) { return (uint64_t)pc.ln[c]; };
    auto slot = [&](int w, int c) { return Ref{ONO_PB_WIRE0 + w, ph(pc.st[c])}; };
    auto at = [&](int buf, int c) { return Ref{buf, pc.st[c]}; };
    const int next = mod(pos + 1, n), prev = mod(pos - 1, n);
    const float fn = (float)n;
    if (len(pos)) b.kernel(ONO_POP_ENCODE_ZERO, {slot(0, pos), at(ONO_PB_RESIDUAL, pos)}, len(pos), wire);
    for (int st = 0; st < n - 1; st++) {  // scatter: out slot 0, in slot 1
        const int cs = mod(pos - st, n), cr = mod(pos - st - 1, n);
        b.group_begin();
        if (len(cs)) b.p2p(ONO_PLAN_SEND, next, slot(0, cs), len(cs), wire);
        if (len(cr)) b.p2p(ONO_PLAN_RECV, prev, slot(1, cr), len(cr), wire);
        b.group_end();
        if (!len(cr)) continue;
        if (st < n - 2)
            b.kernel(ONO_POP_ADD_ENCODE_ZERO, {slot(0, cr), at(ONO_PB_RESIDUAL, cr), slot(1, cr)}, len(cr), wire);
        else
            b.kernel(ONO_POP_ADD_FINISH, {at(ONO_PB_GRAD, cr), slot(0, cr), at(ONO_PB_RESIDUAL, cr), slot(1, cr)},
                     len(cr), wire, fn);
    }
    int bo = 0, bi = 1;  // gather: forward what arrived, alternate the slots
    for (int j = 0; j < n - 1; j++) {
        const int cs = mod(pos + 1 - j, n), cr = mod(pos - j, n);
        b.group_begin();
        if (len(cs)) b.p2p(ONO_PLAN_SEND, next, slot(bo, cs), len(cs), wire);
        if (len(cr)) b.p2p(ONO_PLAN_RECV, prev, slot(bi, cr), len(cr), wire);
        b.group_end();
        if (len(cr)) b.kernel(ONO_POP_DECODE_SCALE, {at(ONO_PB_GRAD, cr), slot(bi, cr)}, len(cr), wire, fn);
        std::swap(bo, bi);
    }
}

// The direct schedule (ono_ring.cpp): all-to-all of chunk slices, the owner's
// chain kernel in the reference order, the residual zeroed on the side stream
// beside the all-gather of the owned chunk.
void direct(Builder &b, int wire, int pos, int n, size_t size, const Pieces &pc) {
    auto len = [&](int c) { return (uint64_t)pc.ln[c]; };
    const size_t slot = pc.slot;
    const int c = mod(pos + 1, n);
    const bool f16 = wire == ONO_WIRE_F16;
    const size_t sc = pc.st[c];
    b.group_begin();  // 1. rank q receives every rank's slice of the chunk it owns, c_q = q + 1
    for (int q = 0; q < n; q++) {
        if (q == pos) continue;
        const int cq = mod(q + 1, n), k = mod(q - c, n);
        if (len(cq)) b.p2p(ONO_PLAN_SEND, q, Ref{ONO_PB_RESIDUAL, pc.st[cq]}, len(cq), ONO_WIRE_F32);
        if (len(c)) b.p2p(ONO_PLAN_RECV, q, Ref{ONO_PB_RBUF, (uint64_t)k * slot + ph(sc)}, len(c), ONO_WIRE_F32);
    }
    b.group_end();
    // 2. the chain c, c+1, ..., c+n-1 (the owner's own slice last), grad = p / n
    if (len(c)) {
        ono_plan_step &s = b.kernel(ONO_POP_DIRECT, {Ref{ONO_PB_GRAD, sc}, f16 ? Ref{ONO_PB_MSG, ph(sc)} : kNone},
                                    len(c), wire, (float)n);
        for (int k = 0; k < n - 1; k++) Builder::ref(s, 2 + k, Ref{ONO_PB_RBUF, (uint64_t)k * slot + ph(sc)});
        Builder::ref(s, 2 + n - 1, Ref{ONO_PB_RESIDUAL, sc});
        s.flag = 0;  // zero the own slice only
    }
    // 3. the sent slices are zeroed on the side stream
    b.fork();
    if (pc.whole) {
        if (sc > 0) b.memset(Ref{ONO_PB_RESIDUAL, 0}, sc, 1);
        if (sc + len(c) < size) b.memset(Ref{ONO_PB_RESIDUAL, sc + len(c)}, size - (sc + len(c)), 1);
    } else {
        for (int q = 0; q < n; q++)
            if (q != c && len(q)) b.memset(Ref{ONO_PB_RESIDUAL, pc.st[q]}, len(q), 1);
    }
    // 4. all-gather of the owned chunk: f32 values, or the f16 message decoded on arrival
    b.group_begin();
    for (int q = 0; q < n; q++) {
        if (q == pos) continue;
        const int cq = mod(q + 1, n);
        if (f16) {
            if (len(c)) b.p2p(ONO_PLAN_SEND, q, Ref{ONO_PB_MSG, ph(sc)}, len(c), ONO_WIRE_F16);
            if (len(cq))
                b.p2p(ONO_PLAN_RECV, q, Ref{ONO_PB_GSTAGE, (uint64_t)q * slot + ph(pc.st[cq])}, len(cq), ONO_WIRE_F16);
        } else {
            if (len(c)) b.p2p(ONO_PLAN_SEND, q, Ref{ONO_PB_GRAD, sc}, len(c), ONO_WIRE_F32);
            if (len(cq)) b.p2p(ONO_PLAN_RECV, q, Ref{ONO_PB_GRAD, pc.st[cq]}, len(cq), ONO_WIRE_F32);
        }
    }
    b.group_end();
    if (f16)
        for (int q = 0; q < n; q++) {
            if (q == pos) continue;
            const int cq = mod(q + 1, n);
            if (!len(cq)) continue;
            b.kernel(ONO_POP_DECODE_SCALE,
                     {Ref{ONO_PB_GRAD, pc.st[cq]}, Ref{ONO_PB_GSTAGE, (uint64_t)q * slot + ph(pc.st[cq])}}, len(cq),
                     ONO_WIRE_F16, (float)n);
        }
    b.join();
}

// ncclAllReduce(sum) + the fused finaliser (grad /= n, residual = 0); with k
// segments the finaliser of segment j runs on the side stream beside the
// all-reduce of segment j+1 (256-B aligned segments).
void allreduce(Builder &b, int n, size_t size, int segments) {
    const float fn = (float)n;
    if (segments <= 1) {
        b.coll(ONO_PLAN_ALLREDUCE, Ref{ONO_PB_RESIDUAL, 0}, Ref{ONO_PB_GRAD, 0}, size);
        b.kernel(ONO_POP_SCALE_ZERO, {Ref{ONO_PB_GRAD, 0}, Ref{ONO_PB_GRAD, 0}, Ref{ONO_PB_RESIDUAL, 0}}, size,
                 ONO_WIRE_F32, fn);
        return;
    }
    const size_t seg = ((size + (size_t)segments - 1) / (size_t)segments + 63) & ~size_t(63);
    for (int k = 0; k < segments && (size_t)k * seg < size; k++) {
        const size_t lo = (size_t)k * seg, len = std::min(seg, size - lo);
        b.coll(ONO_PLAN_ALLREDUCE, Ref{ONO_PB_RESIDUAL, lo}, Ref{ONO_PB_GRAD, lo}, len);
        b.fork();
        b.kernel(ONO_POP_SCALE_ZERO, {Ref{ONO_PB_GRAD, lo}, Ref{ONO_PB_GRAD, lo}, Ref{ONO_PB_RESIDUAL, lo}}, len,
                 ONO_WIRE_F32, fn, 1);
    }
    b.join();
}

int emit(const Builder &b, ono_plan_step *out, size_t cap, size_t *count) {
    *count = b.steps.size();
    if (out && cap) std::copy_n(b.steps.begin(), std::min(cap, b.steps.size()), out);
    if (out && cap && cap < b.steps.size()) return set_error(ONO_E_SIZE, "plan of %zu steps, room for %zu", b.steps.size(), cap);
    return ONO_OK;
}

}  // namespace

int plan_pull_grads(std::vector<ono_plan_step> &out, int algo, int wire, int pos, int n, size_t size, int segments) {
    // one rank plans only the all-reduce (a one-rank communicator: tests, bench plumbing)
    if (n < (algo == ONO_ALGO_ALLREDUCE ? 1 : 2) || pos < 0 || pos >= n)
        return set_error(ONO_E_ARG, "no plan for pos %d of %d ranks", pos, n);
    if (wire != ONO_WIRE_F32 && wire != ONO_WIRE_F16) return set_error(ONO_E_ARG, "wire=%d", wire);
    if (size < (size_t)n) return set_error(ONO_E_SIZE, "bucket of %zu elements cannot be split over %d ranks", size, n);
    Builder b;
    if (algo == ONO_ALGO_ALLREDUCE) {
        if (wire != ONO_WIRE_F32) return set_error(ONO_E_ARG, "an RCCL all-reduce cannot carry the f16 wire semantics");
        allreduce(b, n, size, segments);
        out.swap(b.steps);
        return ONO_OK;
    }
    return plan_pull_grads_sub(out, algo, wire, pos, n, size, 0, 0);
}

size_t plan_sub_elems(size_t sub_elems) { return std::max<size_t>(64, sub_elems / 64 * 64); }

size_t plan_sub_rounds(int n, size_t size, size_t sub_elems) {
    if (n < 1 || size < (size_t)n) return 0;
    const std::vector<size_t> off = split_chunks(size, (size_t)n);
    const size_t maxc = off[1] - off[0], sub = plan_sub_elems(sub_elems);
    return std::max<size_t>(1, (maxc + sub - 1) / sub);
}

int plan_pull_grads_sub(std::vector<ono_plan_step> &out, int algo, int wire, int pos, int n, size_t size,
                        size_t sub_elems, size_t j) {
    if (n < 2 || pos < 0 || pos >= n) return set_error(ONO_E_ARG, "no plan for pos %d of %d ranks", pos, n);
    if (wire != ONO_WIRE_F32 && wire != ONO_WIRE_F16) return set_error(ONO_E_ARG, "wire=%d", wire);
    if (size < (size_t)n) return set_error(ONO_E_SIZE, "bucket of %zu elements cannot be split over %d ranks", size, n);
    const std::vector<size_t> off = split_chunks(size, (size_t)n);
    Pieces pc;
    pc.slot = off[1] - off[0] + 4;
    pc.whole = sub_elems == 0;
    pc.st.resize(n);
    pc.ln.resize(n);
    // sub-round j: elements [j sub, (j + 1) sub) of every chunk (sub a multiple of 64, so every
    // piece keeps its chunk's 4-element phase); every element keeps its owner and its chain
    const size_t sub = pc.whole ? 0 : plan_sub_elems(sub_elems);
    if (!pc.whole && j >= plan_sub_rounds(n, size, sub_elems))
        return set_error(ONO_E_ARG, "sub-round %zu of %zu", j, plan_sub_rounds(n, size, sub_elems));
    for (int c = 0; c < n; c++) {
        const size_t L = off[c + 1] - off[c], lo = pc.whole ? 0 : std::min(L, j * sub);
        pc.st[c] = off[c] + lo;
        pc.ln[c] = pc.whole ? L : std::min(L - lo, sub);
    }
    Builder b;
    switch (algo) {
    case ONO_ALGO_HOPS:
        hops(b, wire, pos, n, pc);
        break;
    case ONO_ALGO_DIRECT:
        if (n > ONO_MAX_INPUTS) return set_error(ONO_E_ARG, "direct schedule supports up to %d ranks", ONO_MAX_INPUTS);
        direct(b, wire, pos, n, size, pc);
        break;
    default:
        return set_error(ONO_E_ARG, "no %s plan for algo %d", pc.whole ? "exchange" : "sub-round", algo);
    }
    out.swap(b.steps);
    return ONO_OK;
}

// BlockingStore + BarrierSync over n workers as one collective step
// (store.rs:84-124): reduce-scatter of the gradients (the accumulate), the
// fused (+0, / n, optimizer) update of the owned shard (shard.rs:74-92), the
// all-gather of the parameters (pull_params).
int plan_ps_step(std::vector<ono_plan_step> &out, int pos, int n, size_t N) {
    if (n < 2 || pos < 0 || pos >= n) return set_error(ONO_E_ARG, "a plan needs 2 or more ranks (pos %d of %d)", pos, n);
    const size_t C = (N + (size_t)n - 1) / (size_t)n, padded = C * (size_t)n;
    const size_t lo = std::min(N, (size_t)pos * C), hi = std::min(N, lo + C);
    Builder b;
    Ref gsrc{ONO_PB_GIN, 0};
    if (padded != N) {  // the tail of GPAD stays zero
        b.copy(Ref{ONO_PB_GPAD, 0}, Ref{ONO_PB_GIN, 0}, N);
        gsrc = Ref{ONO_PB_GPAD, 0};
    }
    b.coll(ONO_PLAN_REDUCE_SCATTER, gsrc, Ref{ONO_PB_GSHARD, 0}, C);
    if (hi > lo) {
        ono_plan_step &s = b.kernel(ONO_POP_OPT_UPDATE, {Ref{ONO_PB_GSHARD, 0}, Ref{ONO_PB_PPAD, (uint64_t)pos * C}},
                                    hi - lo, ONO_WIRE_F32, (float)n);
        s.flag = 1;  // g.fill(0) (shard.rs:89)
    }
    const Ref dst = padded != N ? Ref{ONO_PB_PPAD, 0} : Ref{ONO_PB_PARAMS, 0};
    b.coll(ONO_PLAN_ALL_GATHER, Ref{ONO_PB_PPAD, (uint64_t)pos * C}, dst, C);
    if (padded != N) b.copy(Ref{ONO_PB_PARAMS, 0}, Ref{ONO_PB_PPAD, 0}, N);
    out.swap(b.steps);
    return ONO_OK;
}

void plan_buffers(int n, size_t size, size_t N, uint64_t *c) {
    const std::vector<size_t> off = split_chunks(size, (size_t)std::max(1, n));
    const size_t maxc = off.size() > 1 ? off[1] - off[0] : 0, slot = maxc + 4;
    const size_t C = n > 0 ? (N + (size_t)n - 1) / (size_t)n : N;
    c[ONO_PB_RESIDUAL] = c[ONO_PB_GRAD] = size;
    c[ONO_PB_WIRE0] = c[ONO_PB_WIRE1] = slot;
    c[ONO_PB_RBUF] = c[ONO_PB_GSTAGE] = (uint64_t)n * slot;
    c[ONO_PB_MSG] = slot;
    c[ONO_PB_GIN] = c[ONO_PB_PARAMS] = N;
    c[ONO_PB_GPAD] = c[ONO_PB_PPAD] = C * (size_t)n;
    c[ONO_PB_GSHARD] = C;
}

}  // namespace ono

using namespace ono;

extern "C" {

int ono_plan_pull_grads(int algo, int wire, int pos, int nranks, size_t size, int segments, ono_plan_step *steps,
                        size_t cap, size_t *count) {
    if (!count) return set_error(ONO_E_ARG, "count is NULL");
    std::vector<ono_plan_step> p;
    int rc = plan_pull_grads(p, algo, wire, pos, nranks, size, segments);
    if (rc) return rc;
    Builder b;
    b.steps.swap(p);
    return emit(b, steps, cap, count);
}

int ono_plan_pull_grads_sub(int algo, int wire, int pos, int nranks, size_t size, size_t sub_elems, size_t sub_index,
                            ono_plan_step *steps, size_t cap, size_t *count) {
    if (!count) return set_error(ONO_E_ARG, "count is NULL");
    if (sub_elems == 0) return set_error(ONO_E_ARG, "sub_elems is 0 (the whole bucket: ono_plan_pull_grads)");
    std::vector<ono_plan_step> p;
    int rc = plan_pull_grads_sub(p, algo, wire, pos, nranks, size, sub_elems, sub_index);
    if (rc) return rc;
    Builder b;
    b.steps.swap(p);
    return emit(b, steps, cap, count);
}

size_t ono_plan_sub_rounds(int nranks, size_t size, size_t sub_elems) { return plan_sub_rounds(nranks, size, sub_elems); }

int ono_plan_ps_step(int pos, int nranks, size_t nparams, ono_plan_step *steps, size_t cap, size_t *count) {
    if (!count) return set_error(ONO_E_ARG, "count is NULL");
    std::vector<ono_plan_step> p;
    int rc = plan_ps_step(p, pos, nranks, nparams);
    if (rc) return rc;
    Builder b;
    b.steps.swap(p);
    return emit(b, steps, cap, count);
}

int ono_plan_buffers(int nranks, size_t size, size_t nparams, uint64_t *counts) {
    if (!counts || nranks < 1) return set_error(ONO_E_ARG, "bad arguments");
    plan_buffers(nranks, size, nparams, counts);
    return ONO_OK;
}

}  // extern "C"
