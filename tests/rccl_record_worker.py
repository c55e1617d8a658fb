"""One process, n ranks as threads on one GPU, every RCCL call of the library
answered by the recording stand-in tests/native/librccl_record.so (LD_PRELOAD,
set by tests/test_gpu_rccl_calls.py).  TEST INFRASTRUCTURE.

For one case it runs the real product path — ono_ring_create with an RCCL id,
ono_ring_pull_grads / ono_ring_pull_grads_host / ono_ps_step, i.e. run_plan in
ono_ring.cpp issuing ncclGroupStart/ncclSend/ncclRecv/ncclGroupEnd/
ncclAllReduce/ncclReduceScatter/ncclAllGather — and checks:
  * the calls each rank made, in order, are the communication steps of its
    exchange plan (ono_plan_pull_grads / ono_plan_ps_step): same kind, count,
    dtype, peer and group boundaries, every call on the stream the round runs on;
  * every pointer is base(buffer) + offset x element size for ONE base per plan
    buffer; the owned buckets' and the caller's buffers' bases are their real
    addresses; distinct buffers do not overlap;
  * the results, carried out by the stand-in (matched sends/receives as device
    copies, rank-order sums for the collectives), equal the oracle bit for bit:
    the reference hop ring (worker_ring.rs:112-204) for HOPS / DIRECT, the
    rank-order f32 sum / n for ALLREDUCE, the BlockingStore fed in worker order
    (blocking/store.rs:84-124) for the PS step.
usage: python rccl_record_worker.py CASE_JSON RECORD_PATH   -> one JSON line {"ok": bool, "msg": str}
"""
import json
import os
import sys
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "oxidized-neural-orchestra_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import ono_amd  # noqa: E402
from ono_amd import plan as P  # noqa: E402
from oracle import oracle as O  # noqa: E402  (checker only)

SEED = 0x0402026
NCCL_DTYPE = {"f16": 6, "f32": 7}


def esize(buf: str, wire: str) -> int:
    if buf in ("wire0", "wire1"):
        return 2 if wire == "f16" else 4
    return 2 if buf in ("gstage", "msg") else 4


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def expected_calls(steps: list) -> list:
    """The RCCL calls a plan's communication steps map to, in issue order."""
    out, group = [], None
    for st in steps:
        k = st["kind"]
        if k == "group_begin":
            group = []
        elif k in ("send", "recv"):
            group.append(st)
            out.append(st)
        elif k == "group_end":
            out.append({"kind": "group", "calls": len(group)})
            group = None
        elif k in ("allreduce", "reduce_scatter", "all_gather"):
            out.append(st)
    return out


def check_calls(rank: int, recs: list, steps: list, wire: str, known: dict, rounds: int) -> str | None:
    """recs: this rank's recorded calls; steps: its plan (one round)."""
    want = expected_calls(steps) * rounds
    got = [r for r in recs if r["op"] not in ("init", "destroy")]
    if len(got) != len(want):
        return f"rank {rank}: {len(got)} RCCL calls recorded, the plan has {len(want)}"
    bases, streams = {}, set()
    opname = {"allreduce": "all_reduce", "reduce_scatter": "reduce_scatter", "all_gather": "all_gather"}
    for i, (g, w) in enumerate(zip(got, want)):
        if w["kind"] == "group":
            if g["op"] != "group" or g["calls"] != w["calls"]:
                return f"rank {rank} call {i}: {g} is not the end of a {w['calls']}-call group"
            continue
        kind = w["kind"] if w["kind"] in ("send", "recv") else opname[w["kind"]]
        if g["op"] != kind or g["count"] != w["count"]:
            return f"rank {rank} call {i}: {g['op']} x{g['count']} where the plan has {kind} x{w['count']}"
        dt = NCCL_DTYPE[w["dtype"]] if kind in ("send", "recv") else 7
        if g["dtype"] != dt:
            return f"rank {rank} call {i}: dtype {g['dtype']} != {dt}"
        if kind in ("send", "recv"):
            if g["peer"] != w["peer"]:
                return f"rank {rank} call {i}: peer {g['peer']} != {w['peer']}"
            if g["group"] == 0:
                return f"rank {rank} call {i}: {kind} outside a group"
            ptrs = [(w["refs"][0], g["ptr"])]
        else:
            ptrs = [(w["refs"][0], g["src"]), (w["refs"][1], g["dst"])]
        streams.add(g["stream"])
        for (buf, off), ptr in ptrs:
            base = ptr - off * esize(buf, wire)
            if bases.setdefault(buf, base) != base:
                return f"rank {rank} call {i}: {buf} addressed from two bases"
    if len(streams) > 1:
        return f"rank {rank}: RCCL calls on {len(streams)} streams"
    for buf, addr in known.items():
        if buf in bases and bases[buf] != addr:
            return f"rank {rank}: {buf} base 0x{bases[buf]:x} is not the buffer at 0x{addr:x}"
    return None


def no_overlap(rank: int, bases: dict, sizes: dict, wire: str) -> str | None:
    spans = sorted((b, b + sizes[buf] * esize(buf, wire), buf) for buf, b in bases.items() if sizes.get(buf))
    for (a0, a1, x), (b0, b1, y) in zip(spans, spans[1:]):
        if b0 < a1:
            return f"rank {rank}: {x} and {y} overlap"
    return None


def run_pull(case: dict, records: list) -> str | None:
    n, size, algo, wire = case["n"], case["size"], case["algo"], case["wire"]
    rounds, host, segs = case.get("rounds", 2), case.get("host", False), case.get("segments", 0)
    uid = ono_amd.unique_id()
    rings = [ono_amd.WorkerRingManager(r, n, size, uid=uid, wire=wire, algo=algo) for r in range(n)]
    if segs:
        for rg in rings:
            rg.set_pipeline(segs)
    outs = [[None] * rounds for _ in range(n)]
    errs = []
    ins = [[O.synth(size, SEED + 17 * k, r) for r in range(n)] for k in range(rounds)]

    def rank_main(r):
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream()
            for k in range(rounds):
                if host:
                    res = ins[k][r].copy()
                    grad = np.full(size, 7.0, np.float32)
                    rings[r].pull_grads_host(res, grad)
                    outs[r][k] = (grad, res)
                else:
                    with torch.cuda.stream(s):
                        rings[r].residual.copy_(torch.from_numpy(ins[k][r]).cuda())
                        rings[r].pull_grads(stream=s)
                    s.synchronize()
                    outs[r][k] = (rings[r].grad.cpu().numpy(), rings[r].residual.cpu().numpy())
        except Exception as e:
            errs.append(f"rank {r}: {type(e).__name__}: {e}")
    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join(600)
    try:
        if errs:
            return errs[0]
        for k in range(rounds):
            if algo == "allreduce":
                exp = [O.sum_scale(ins[k], float(n))] * n
            else:
                exp, _ = O.ring_pull_grads(ins[k], wire)
            for r in range(n):
                g, res = outs[r][k]
                bad = np.flatnonzero(~O.same_or_both_nan(g, exp[r]))
                if bad.size:
                    return f"round {k} rank {r}: {bad.size}/{size} differ from the oracle, first at {bad[0]}"
                if bits(res).any():
                    return f"round {k} rank {r}: residual not zeroed"
        if host:
            return None  # sub-round plans: results checked above, the call mapping by the whole-round cases
        nseg = 0
        if algo == "allreduce":
            nseg = max(1, min(segs or 4, size // (4 << 20)))
        sizes = P.buffers(n, size)
        for r in range(n):
            steps = P.pull_grads(algo, wire, r, n, size, nseg)
            recs = [x for x in records if x.get("rank") == r]
            known = {"residual": rings[r].residual.data_ptr(), "grad": rings[r].grad.data_ptr()}
            msg = check_calls(r, recs, steps, wire, known, rounds)
            if msg:
                return msg
            bases = {}
            for st in steps:
                for buf, off in st["refs"]:
                    if buf in ("residual", "grad"):
                        bases[buf] = known[buf]
            msg = no_overlap(r, bases, sizes, wire)
            if msg:
                return msg
        return None
    finally:
        for rg in rings:
            rg.close()


def run_ps(case: dict, records: list) -> str | None:
    n, nparams, kind, steps = case["n"], case["size"], case["opt"], case.get("steps", 3)
    opt = {"gd": ono_amd.GradientDescent(0.1), "momentum": ono_amd.GradientDescentWithMomentum(0.1, 0.9),
           "adam": ono_amd.Adam(0.1, 0.9, 0.999, 1e-8)}[kind]
    uid = ono_amd.unique_id()
    init = O.synth(nparams, SEED, 99)
    rings = [ono_amd.WorkerRingManager(r, n, nparams, uid=uid) for r in range(n)]
    pss = [ono_amd.ShardedParamServer(rings[r], init, opt) for r in range(n)]
    gs = [[O.synth(nparams, SEED + 10 * st, w) for w in range(n)] for st in range(steps)]
    outs = [[None] * steps for _ in range(n)]
    ptrs = [None] * n
    errs = []

    def rank_main(r):
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream()
            params = torch.empty(nparams, device="cuda")
            g = torch.empty(nparams, device="cuda")
            ptrs[r] = {"gin": g.data_ptr(), "params": params.data_ptr()}
            for st in range(steps):
                with torch.cuda.stream(s):
                    g.copy_(torch.from_numpy(gs[st][r]).cuda())
                    pss[r].step(g, params, stream=s)
                s.synchronize()
                outs[r][st] = params.cpu().numpy()
        except Exception as e:
            errs.append(f"rank {r}: {type(e).__name__}: {e}")
    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join(600)
    try:
        if errs:
            return errs[0]
        ref = O.Store(init, 1000, n, kind, lr=0.1, momentum=0.9, beta1=0.9, beta2=0.999, eps=1e-8)
        for st in range(steps):
            for w in range(n):
                ref.accumulate(gs[st][w])
            ref.update_params()
            exp = ref.pull_params()
            for r in range(n):
                bad = np.flatnonzero(bits(outs[r][st]) != bits(exp))
                if bad.size:
                    return f"step {st} rank {r}: {bad.size}/{nparams} differ from the store oracle, first at {bad[0]}"
        for r in range(n):
            plan = P.ps_step(r, n, nparams)
            recs = [x for x in records if x.get("rank") == r]
            msg = check_calls(r, recs, plan, "f32", ptrs[r], steps)
            if msg:
                return msg
        return None
    finally:
        for p in pss:
            p.close()
        for rg in rings:
            rg.close()


def main() -> int:
    case, path = json.loads(sys.argv[1]), sys.argv[2]
    torch.cuda.set_device(0)
    try:
        mode = case.get("mode", "pull")
        # the recorder appends as the calls happen; read it back after the run
        runner = run_ps if mode == "ps" else run_pull
        records = []
        holder = {}

        def load():
            with open(path) as f:
                return [json.loads(line) for line in f if line.strip()]

        class Lazy(list):  # the records are read after the ranks finished (inside the runner)
            def __iter__(self):
                if "r" not in holder:
                    holder["r"] = load()
                return iter(holder["r"])
        records = Lazy()
        msg = runner(case, records)
        mism = [x for x in load() if x.get("op") == "mismatch"]
        if msg is None and mism:
            msg = f"the stand-in saw mismatched calls: {mism[:2]}"
    except Exception as e:
        msg = f"{type(e).__name__}: {e}"
    print(json.dumps({"ok": msg is None, "msg": msg or ""}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
