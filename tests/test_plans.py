"""The N > 1 exchange plans, checked and executed on the CPU (no GPU).

Every RCCL schedule of the product — pull_grads' ALLREDUCE (with its
segments), HOPS and DIRECT on either wire, and the sharded PS step — is a
step list built per rank by ono_plan.cpp and run by one interpreter in
libono_reduce.so (run_plan in ono_ring.cpp).  Here the lists of all n ranks
are checked against each other and executed with host copies:

  * every group's sends and receives pair up (k-th send r->q with the k-th
    receive at q from r), with equal counts and dtypes;
  * every operand range lies inside its buffer (sizes from ono_plan_buffers);
  * the grad bucket is covered: the chunks tile [0, N) on every rank;
  * nothing on the side stream touches what the main stream touches between
    the fork that started it and the join that ends it;
  * executed in lockstep (collectives summed in rank order), the results are
    bit-exact with the oracle's restatement of worker_ring.rs:112-204 (HOPS,
    DIRECT) or with the rank-order sum (ALLREDUCE), and with the BlockingStore
    oracle (store.rs:84-124, shard.rs:74-92) for the PS step.
"""
import numpy as np
import pytest

import ono_amd
from ono_amd import plan as P
from conftest import SEED, assert_bitexact
from oracle import oracle as O

F16_BUFS = ("gstage", "msg")


def dtype_of(buf, wire):
    if buf in ("wire0", "wire1"):
        return np.uint16 if wire == "f16" else np.float32
    return np.uint16 if buf in F16_BUFS else np.float32


def enc(x, wire):
    return O.f16_encode(x) if wire == "f16" else np.array(x, np.float32, copy=True)


def dec(h, wire):
    return O.f16_decode(h) if wire == "f16" else np.array(h, np.float32, copy=True)


def div(x, d):
    return x if d == 1.0 else (x / np.float32(d)).astype(np.float32)


def accesses(st):
    """(reads, writes): lists of (buf, lo, hi) of one step."""
    k, n, refs = st["kind"], st["count"], st["refs"]
    rng = lambda i, m=1: (refs[i][0], refs[i][1], refs[i][1] + n * m)  # noqa: E731
    R, W = [], []
    if k == "send":
        R.append(rng(0))
    elif k == "recv":
        W.append(rng(0))
    elif k in ("allreduce",):
        R.append(rng(0)); W.append(rng(1))
    elif k == "memset":
        W.append(rng(0))
    elif k == "copy":
        W.append(rng(0)); R.append(rng(1))
    elif k == "kernel":
        op = st["op"]
        if op == "encode_zero":
            W += [rng(0), rng(1)]; R.append(rng(1))
        elif op == "add_encode_zero":
            W += [rng(0), rng(1)]; R += [rng(1), rng(2)]
        elif op == "add_finish":
            W += [rng(0), rng(1), rng(2)]; R += [rng(2), rng(3)]
        elif op == "decode_scale":
            W.append(rng(0)); R.append(rng(1))
        elif op == "direct":
            W.append(rng(0))
            if refs[1][0] is not None:
                W.append(rng(1))
            ins = list(range(2, len(refs)))
            R += [rng(i) for i in ins]
            W += [rng(i) for i in (ins if st["flag"] else ins[-1:])]
        elif op == "scale_zero":
            W.append(rng(0)); R.append(rng(1))
            if refs[2][0] is not None:
                W.append(rng(2))
        elif op == "opt_update":
            W += [rng(0), rng(1)]; R += [rng(0), rng(1)]
    return R, W


def overlap(a, b):
    return a[0] == b[0] and a[1] < b[2] and b[1] < a[2]


def check_streams(plan):
    """A side-stream step placed after fork f runs concurrently with every
    main-stream step issued after fork f until the join; none of those may
    touch what it writes, nor write what it reads.  Every fork is joined."""
    last_fork = None
    main = []   # (index, reads, writes) of main steps since the last join
    side = []   # (fork index, reads, writes) of side steps since the last join
    for i, st in enumerate(plan):
        k = st["kind"]
        if k == "fork":
            last_fork = i
            continue
        if k == "join":
            main, side = [], []
            continue
        if k in ("group_begin", "group_end"):
            continue
        R, W = accesses(st)
        if st["stream"] == 1:
            assert last_fork is not None, f"step {i} on the side stream before any fork"
            for mi, mR, mW in main:
                if mi < last_fork:
                    continue  # ordered before the fork the side stream waited for
                assert not any(overlap(w, x) for w in W for x in mR + mW), f"side step {i} races main step {mi}"
                assert not any(overlap(r_, x) for r_ in R for x in mW), f"side step {i} reads main step {mi}'s writes"
            side.append((last_fork, R, W))
        else:
            for f, sR, sW in side:
                assert not any(overlap(w, x) for w in W for x in sR + sW), f"main step {i} races the side stream"
                assert not any(overlap(r_, x) for r_ in R for x in sW), f"main step {i} reads side-stream writes"
            main.append((i, R, W))
    assert not side, "side-stream work is never joined"


def check_bounds(plan, sizes):
    for i, st in enumerate(plan):
        R, W = accesses(st)
        if st["kind"] in ("reduce_scatter", "all_gather"):
            continue  # checked in the executor with the rank count
        for buf, lo, hi in R + W:
            assert buf is not None and 0 <= lo <= hi <= sizes[buf], f"step {i}: {buf}[{lo}:{hi}] of {sizes[buf]}"


def kernel(st, B, wire, opt):
    op, n, refs, d = st["op"], st["count"], st["refs"], st["divisor"]
    v = lambda i: B[refs[i][0]][refs[i][1]: refs[i][1] + n]  # noqa: E731
    if op == "encode_zero":
        v(0)[:] = enc(v(1), wire); v(1)[:] = 0
    elif op == "add_encode_zero":
        x = (v(1) + dec(v(2), wire)).astype(np.float32)
        v(0)[:] = enc(x, wire); v(1)[:] = 0
    elif op == "add_finish":
        x = (v(2) + dec(v(3), wire)).astype(np.float32)
        v(0)[:] = div(x, d); v(1)[:] = enc(x, wire); v(2)[:] = 0
    elif op == "decode_scale":
        v(0)[:] = div(dec(v(1), wire), d)
    elif op == "direct":
        ins = list(range(2, len(refs)))
        p = np.array(v(ins[0]), np.float32, copy=True)
        for i in ins[1:]:
            p = (v(i) + dec(enc(p, wire), wire)).astype(np.float32)
        g = div(p, d)
        v(0)[:] = g
        if refs[1][0] is not None:
            v(1)[:] = enc(p, wire) if wire == "f16" else g
        for i in (ins if st["flag"] else ins[-1:]):
            v(i)[:] = 0
    elif op == "scale_zero":
        v(0)[:] = div(np.array(v(1), copy=True), d)
        if refs[2][0] is not None:
            v(2)[:] = 0
    elif op == "opt_update":  # the store's GD update: (g + 0) / n, w -= lr * g, g = 0
        g = (v(0) + np.float32(0)).astype(np.float32)
        g = div(g, d)
        v(1)[:] = (v(1) - np.float32(opt) * g).astype(np.float32)
        if st["flag"]:
            v(0)[:] = 0
    else:
        raise AssertionError(op)


def execute(plans, bufs, wire, opt=None):
    """Lockstep: each rank runs its local steps up to the next collective point
    (a send/recv group or an RCCL collective), then that point runs for all
    ranks at once.  Returns the grad-bucket coverage per rank."""
    n = len(plans)
    pc = [0] * n
    covered = [np.zeros(bufs[r]["grad"].size if "grad" in bufs[r] else 0, bool) for r in range(n)]

    def local(r):
        while pc[r] < len(plans[r]):
            st = plans[r][pc[r]]
            k = st["kind"]
            if k in ("group_begin", "allreduce", "reduce_scatter", "all_gather"):
                return
            B = bufs[r]
            if k == "kernel":
                kernel(st, B, wire, opt)
            elif k == "memset":
                b, o = st["refs"][0]
                B[b][o: o + st["count"]] = 0
            elif k == "copy":
                (b0, o0), (b1, o1) = st["refs"][:2]
                B[b0][o0: o0 + st["count"]] = B[b1][o1: o1 + st["count"]]
            for buf, lo, hi in accesses(st)[1]:
                if buf == "grad":
                    covered[r][lo:hi] = True
            pc[r] += 1

    while True:
        for r in range(n):
            local(r)
        done = [pc[r] >= len(plans[r]) for r in range(n)]
        if all(done):
            break
        assert not any(done), "ranks disagree on the number of collective points"
        kinds = {plans[r][pc[r]]["kind"] for r in range(n)}
        assert len(kinds) == 1, f"ranks at different collectives: {kinds}"
        kind = kinds.pop()
        if kind == "group_begin":
            ops = []
            for r in range(n):
                mine = []
                pc[r] += 1
                while plans[r][pc[r]]["kind"] != "group_end":
                    mine.append(plans[r][pc[r]])
                    pc[r] += 1
                pc[r] += 1
                ops.append(mine)
            # the k-th send r -> q pairs with the k-th receive at q from r
            payload = {}
            for r in range(n):
                sends = {}
                for st in ops[r]:
                    if st["kind"] == "send":
                        q = st["peer"]
                        assert q != r and 0 <= q < n
                        b, o = st["refs"][0]
                        payload.setdefault((r, q), []).append(
                            (st["count"], st["dtype"], np.array(bufs[r][b][o: o + st["count"]], copy=True)))
                        sends[q] = sends.get(q, 0) + 1
            for q in range(n):
                for st in ops[q]:
                    if st["kind"] != "recv":
                        continue
                    r = st["peer"]
                    assert payload.get((r, q)), f"rank {q} receives from {r}, who sends nothing"
                    cnt, dt, data = payload[(r, q)].pop(0)
                    assert cnt == st["count"] and dt == st["dtype"], f"{r}->{q}: {cnt} {dt} vs {st['count']} {st['dtype']}"
                    b, o = st["refs"][0]
                    bufs[q][b][o: o + cnt] = data
                    for buf, lo, hi in [(b, o, o + cnt)]:
                        if buf == "grad":
                            covered[q][lo:hi] = True
            assert not any(payload.values()), "unmatched sends"
        else:
            sts = [plans[r][pc[r]] for r in range(n)]
            cnt = sts[0]["count"]
            assert all(s["count"] == cnt for s in sts)
            src = [bufs[r][s["refs"][0][0]] for r, s in enumerate(sts)]
            so = [s["refs"][0][1] for s in sts]
            if kind == "allreduce":
                acc = np.array(src[0][so[0]: so[0] + cnt], copy=True)
                for r in range(1, n):
                    acc = (acc + src[r][so[r]: so[r] + cnt]).astype(np.float32)
                for r, s in enumerate(sts):
                    b, o = s["refs"][1]
                    bufs[r][b][o: o + cnt] = acc
                    if b == "grad":
                        covered[r][o: o + cnt] = True
            elif kind == "reduce_scatter":
                for q, s in enumerate(sts):
                    assert so[0] + n * cnt <= src[0].size
                    acc = np.array(src[0][so[0] + q * cnt: so[0] + (q + 1) * cnt], copy=True)
                    for r in range(1, n):
                        acc = (acc + src[r][so[r] + q * cnt: so[r] + (q + 1) * cnt]).astype(np.float32)
                    b, o = s["refs"][1]
                    bufs[q][b][o: o + cnt] = acc
            elif kind == "all_gather":
                parts = [np.array(src[r][so[r]: so[r] + cnt], copy=True) for r in range(n)]
                for q, s in enumerate(sts):
                    b, o = s["refs"][1]
                    assert o + n * cnt <= bufs[q][b].size
                    for r in range(n):
                        bufs[q][b][o + r * cnt: o + (r + 1) * cnt] = parts[r]
            for r in range(n):
                pc[r] += 1
    return covered


def pull_buffers(n, size, wire, x):
    sizes = P.buffers(n, size)
    bufs = []
    for r in range(n):
        B = {b: np.zeros(sizes[b], dtype_of(b, wire)) for b in ("grad", "wire0", "wire1", "rbuf", "gstage", "msg")}
        B["grad"][:] = np.float32(7.0)  # every element must be written
        B["residual"] = np.array(x[r], np.float32, copy=True)
        bufs.append(B)
    return sizes, bufs


SIZES = lambda n: [n, 37 if n <= 37 else n + 1, 1000 * n + 3, 4099]  # noqa: E731


@pytest.mark.parametrize("n", list(range(2, 17)))
@pytest.mark.parametrize("algo,wire", [("hops", "f16"), ("hops", "f32"), ("direct", "f16"), ("direct", "f32")])
def test_pull_grads_plans_vs_oracle(n, algo, wire):
    for size in SIZES(n):
        x = [O.synth(size, SEED + 17, r) for r in range(n)]
        plans = [P.pull_grads(algo, wire, r, n, size) for r in range(n)]
        sizes, bufs = pull_buffers(n, size, wire, x)
        for p in plans:
            check_bounds(p, sizes)
            check_streams(p)
        covered = execute(plans, bufs, wire)
        eg, er = O.ring_pull_grads(x, wire)
        for r in range(n):
            assert covered[r].all(), f"{algo}/{wire} n={n} size={size}: rank {r}'s grad not covered"
            assert_bitexact(bufs[r]["grad"], eg[r], f"{algo}/{wire} n={n} size={size} grad {r}")
            assert_bitexact(bufs[r]["residual"], er[r], f"{algo}/{wire} n={n} size={size} residual {r}")


@pytest.mark.parametrize("n", [2, 3, 5, 8, 16])
@pytest.mark.parametrize("algo,wire", [("hops", "f16"), ("hops", "f32"), ("direct", "f16"), ("direct", "f32")])
@pytest.mark.parametrize("sub", [64, 100, 1000])
def test_host_fed_sub_round_plans_vs_oracle(n, algo, wire, sub):
    """The host-fed HOPS / DIRECT round as sub-rounds (a 64-multiple slice of
    every chunk each, empty slices left out on both sides): each sub-round's
    plans match up across ranks, stay in bounds and race nothing, and the
    sub-rounds in order give the whole-bucket result bit for bit."""
    for size in (n, 1000 * n + 3, 4099):
        if size < n:
            continue
        x = [O.synth(size, SEED + 29, r) for r in range(n)]
        S = P.sub_rounds(n, size, sub)
        maxc = -(-size // n)
        assert S == max(1, -(-maxc // max(64, sub // 64 * 64)))
        sizes, bufs = pull_buffers(n, size, wire, x)
        cov = [np.zeros(size, bool) for _ in range(n)]
        for j in range(S):
            plans = [P.pull_grads_sub(algo, wire, r, n, size, sub, j) for r in range(n)]
            for p in plans:
                check_bounds(p, sizes)
                check_streams(p)
            covered = execute(plans, bufs, wire)
            for r in range(n):
                cov[r] |= covered[r]
        eg, er = O.ring_pull_grads(x, wire)
        for r in range(n):
            assert cov[r].all(), f"{algo}/{wire} n={n} size={size} sub={sub}: rank {r}'s grad not covered"
            assert_bitexact(bufs[r]["grad"], eg[r], f"{algo}/{wire} n={n} size={size} sub={sub} grad {r}")
            assert_bitexact(bufs[r]["residual"], er[r], f"{algo}/{wire} n={n} size={size} sub={sub} residual {r}")


def test_sub_round_plan_errors():
    with pytest.raises(ono_amd.InvalidArgument):
        P.pull_grads_sub("allreduce", "f32", 0, 2, 1000, 64, 0)  # the all-reduce is pipelined in chunks already
    with pytest.raises(ono_amd.InvalidArgument):
        P.pull_grads_sub("hops", "f16", 0, 2, 1000, 64, P.sub_rounds(2, 1000, 64))  # past the last sub-round
    with pytest.raises(ono_amd.InvalidArgument):
        P.pull_grads_sub("hops", "f16", 0, 2, 1000, 0, 0)
    assert P.sub_rounds(4, 3, 64) == 0


@pytest.mark.parametrize("n", [2, 3, 4, 5, 8, 13, 16])
@pytest.mark.parametrize("segments", [1, 2, 4, 7])
def test_allreduce_plans(n, segments):
    """Segments tile the bucket (256-B aligned), each finaliser runs on the side
    stream after its own segment's all-reduce and races nothing; the result is
    the all-reduce's sum / n (rank order here, so bit-exact with numpy; RCCL's
    own order is the stated n >= 3 tolerance) and a zeroed residual."""
    for size in (n, 4099, 64 * 1000 + 5):
        x = [O.synth(size, SEED + 19, r) for r in range(n)]
        plans = [P.pull_grads("allreduce", "f32", r, n, size, segments) for r in range(n)]
        assert all(p == plans[0] for p in plans), "the all-reduce plan is rank-independent"
        sizes, bufs = pull_buffers(n, size, "f32", x)
        check_bounds(plans[0], sizes)
        check_streams(plans[0])
        covered = execute(plans, bufs, "f32")
        acc = np.array(x[0], copy=True)
        for r in range(1, n):
            acc = (acc + x[r]).astype(np.float32)
        want = div(acc, float(n))
        for r in range(n):
            assert covered[r].all()
            assert_bitexact(bufs[r]["grad"], want, f"n={n} size={size} segments={segments}")
            assert not bufs[r]["residual"].view(np.uint32).any()
        eg, _ = O.ring_pull_grads(x, "f32")  # the hop-order restatement: order-only difference
        bound = 2 * (n - 1) * 2.0 ** -24 * np.sum(np.abs(np.stack(x)), axis=0) / n
        assert np.all(np.abs(bufs[0]["grad"] - eg[0]) <= bound + 1e-30)


@pytest.mark.parametrize("n", [2, 3, 4, 7, 8, 16])
@pytest.mark.parametrize("nparams", [1, 15, 100, 4099])
def test_ps_step_plans_vs_store_oracle(n, nparams):
    """Reduce-scatter of the padded gradients, the owned shard's GD update,
    all-gather of the parameters: equal to the BlockingStore oracle fed the
    workers in rank order (accumulate from +0, / n, w -= lr g)."""
    if nparams < 1:
        return
    lr = 0.1
    init = O.synth(nparams, SEED + 23, 99)
    grads = [O.synth(nparams, SEED + 23, r) for r in range(n)]
    sizes = P.buffers(n, 0, nparams)
    plans = [P.ps_step(r, n, nparams) for r in range(n)]
    bufs = []
    for r in range(n):
        B = {b: np.zeros(sizes[b], np.float32) for b in ("gpad", "gshard", "ppad", "params")}
        B["gin"] = np.array(grads[r], copy=True)
        B["ppad"][:nparams] = init
        B["params"][:] = np.float32(7.0)
        bufs.append(B)
    for p in plans:
        check_streams(p)
    execute(plans, bufs, "f32", opt=lr)
    store = O.Store(init, max(1, -(-nparams // n)), n, "gd", lr=lr)
    for g in grads:
        store.accumulate(g)
    store.update_params()
    want = store.pull_params()
    for r in range(n):
        assert_bitexact(bufs[r]["params"], want, f"n={n} nparams={nparams} rank {r}")


def test_plan_argument_errors():
    with pytest.raises(ono_amd.InvalidArgument):
        P.pull_grads("hops", "f16", 0, 1, 100)  # one rank has no exchange
    with pytest.raises(ono_amd.InvalidArgument):
        P.pull_grads("allreduce", "f16", 0, 2, 100)
    with pytest.raises(ono_amd.InvalidArgument):
        P.pull_grads("direct", "f32", 0, 17, 1000)
    with pytest.raises(ono_amd.SizeMismatch):
        P.pull_grads("hops", "f32", 0, 4, 3)


def test_stream_checker_catches_a_race():
    """The race check is live: move the direct plan's side-stream memset onto
    the grad bucket the all-gather writes, and it fails."""
    plan = P.pull_grads("direct", "f32", 1, 3, 37)
    bad = [dict(st) for st in plan]
    for st in bad:
        if st["kind"] == "memset":
            st["refs"] = [("grad", 0)]
    check_streams(plan)
    with pytest.raises(AssertionError):
        check_streams(bad)
