"""One rank of a multi-process xGMI-schedule test (tests/test_gpu_xgmi.py).

Every rank is its own process (as on an 8-GPU node: one process per GPU); on
the one-GPU test box all ranks share cuda:0, so the peer regions they map are
IPC imports of the same device — the same code path (export, import, peer
loads/stores, flag barriers), with HBM standing in for the xGMI links.  The
128-byte handles travel over a gloo group (the control channel the reference
would use is its ring TCP links).

usage: python xgmi_worker.py RANK NRANKS (PORT | file://PATH) CASES_JSON
Prints one JSON line: {"rank": r, "results": [{"case": ..., "ok": bool, "msg": str}, ...]}.
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "oxidized-neural-orchestra_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import ono_amd  # noqa: E402
from oracle import oracle as O  # noqa: E402  (checker only)

SEED = 0x0402026


def allgather(b: bytes) -> list:
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, b)
    return out


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def run_case(rank: int, n: int, case: dict) -> str | None:
    """None when the case passes, else a message."""
    length, wire, rounds = case["length"], case["wire"], case.get("rounds", 2)
    form = case.get("form", "owned")  # owned | dev | dev_offset
    ring = ono_amd.WorkerRingManager.over_xgmi(rank, n, length, allgather, wire=wire)
    try:
        for rd in range(rounds):
            gen = O.synth_special if case.get("special") else O.synth
            ins = [gen(length, SEED + 100 * rd + case.get("seed", 0), r) for r in range(n)]
            expect, _ = O.ring_pull_grads(ins, wire)
            if form in ("host", "host_registered"):  # host-fed: sub-round pipeline (pageable / page-locked)
                res_h = np.ascontiguousarray(ins[rank]).copy()
                grad_h = np.full(length, 7.0, np.float32)
                if form == "host_registered":
                    ring.register_host(res_h)
                    ring.register_host(grad_h)
                ring.pull_grads_host(res_h, grad_h)
                got, res_after = grad_h, res_h
                if form == "host_registered":
                    ring.unregister_host(res_h)
                    ring.unregister_host(grad_h)
            elif form == "owned":
                ring.residual.copy_(torch.from_numpy(ins[rank]))
                ring.pull_grads()
                torch.cuda.synchronize()
                got, res_after = ring.grad.cpu().numpy(), ring.residual.cpu().numpy()
            else:  # caller device buffers; dev_offset: views at different 4-element phases
                ro, go = (1, 2) if form == "dev_offset" else (0, 0)
                rbase = torch.zeros(length + 8, dtype=torch.float32, device="cuda")
                gbase = torch.full((length + 8,), 7.0, dtype=torch.float32, device="cuda")
                res, grad = rbase[ro:ro + length], gbase[go:go + length]
                res.copy_(torch.from_numpy(ins[rank]))
                ring.pull_grads_dev(res, grad)
                torch.cuda.synchronize()
                got, res_after = grad.cpu().numpy(), res.cpu().numpy()
                if gbase[:go].ne(7.0).any().item() or gbase[go + length:].ne(7.0).any().item():
                    return f"round {rd}: write outside the grad view"
                if rbase[:ro].ne(0).any().item() or rbase[ro + length:].ne(0).any().item():
                    return f"round {rd}: write outside the residual view"
            bad = np.flatnonzero(~O.same_or_both_nan(got, expect[rank]))
            if bad.size:
                i = bad[0]
                msg = (f"round {rd}: {bad.size}/{length} differ, first at {i}: "
                       f"0x{bits(got)[i]:08x} vs 0x{bits(expect[rank])[i]:08x}")
                if os.environ.get("ONO_XGMI_DIAG"):  # where the wrong elements sit (chunk, sub-round) and what they hold
                    off = [0]
                    for q in range(n):
                        off.append(off[-1] + length // n + (1 if q < length % n else 0))
                    sub = max(64, (int(os.environ.get("ONO_HOST_CHUNK_MIB", "16")) << 18) // n // 64 * 64)
                    where = {}
                    for b in bad:
                        q = int(np.searchsorted(off, b, side="right") - 1)
                        key = (q, int((b - off[q]) // sub))
                        where[key] = where.get(key, 0) + 1
                    zeros = int((got[bad] == 0).sum())
                    own = np.float32(ins[rank][bad]) / np.float32(n)
                    msg += f" | by (chunk, subround): {sorted(where.items())[:8]} zeros={zeros}"
                    msg += f" own/n={int((got[bad] == own).sum())}"
                    lo, hi = int(bad.min()), int(bad.max())
                    msg += f" span=[{lo},{hi}]"
                    # contiguous runs of wrong elements (page-sized runs point at address translation,
                    # scattered ones at ordering); host-fed: does the ring's device staging hold the
                    # right values (then the D2H copy is what went wrong)?
                    cuts = np.flatnonzero(np.diff(bad) != 1)
                    starts = np.concatenate(([bad[0]], bad[cuts + 1]))
                    ends = np.concatenate((bad[cuts], [bad[-1]])) + 1
                    runs = [(int(a), int(b - a)) for a, b in zip(starts, ends)]
                    msg += f" runs={len(runs)} first_runs={runs[:6]}"
                    if form in ("host", "host_registered"):
                        dev = ring.grad.cpu().numpy()
                        msg += f" dev_right={int(O.same_or_both_nan(dev[bad], expect[rank][bad]).sum())}"
                return msg
            if bits(res_after).any():
                return f"round {rd}: residual not zeroed ({np.count_nonzero(bits(res_after))} left)"
        return None
    finally:
        ring.close()


def run_ps(rank: int, n: int, case: dict) -> str | None:
    """ShardedParamServer over the xGMI ring (BASELINE config 5): every rank
    is a worker and the server of shard `rank`; after each step all ranks
    hold the parameters the BlockingStore oracle computes when the n workers'
    gradients arrive in rank order."""
    nparams, kind, steps = case["length"], case["opt"], case.get("steps", 3)
    opt = {"gd": ono_amd.GradientDescent(0.1), "momentum": ono_amd.GradientDescentWithMomentum(0.1, 0.9),
           "adam": ono_amd.Adam(0.1, 0.9, 0.999, 1e-8)}[kind]
    init = O.synth(nparams, SEED, 99)
    ring = ono_amd.WorkerRingManager.over_xgmi(rank, n, nparams, allgather)
    ps = ono_amd.ShardedParamServer(ring, init, opt)
    ref = O.Store(init, 1000, n, kind, lr=0.1, momentum=0.9, beta1=0.9, beta2=0.999, eps=1e-8)
    try:
        params = torch.empty(nparams, device="cuda")
        for st in range(steps):
            gs = [O.synth(nparams, SEED + 10 * st, w) for w in range(n)]
            g = torch.from_numpy(gs[rank]).cuda()
            ps.step(g, params)
            for w in range(n):
                ref.accumulate(gs[w])
            ref.update_params()
            torch.cuda.synchronize()
            if not np.array_equal(bits(g.cpu().numpy()), bits(gs[rank])):
                return f"step {st}: the worker's gradient was modified"
            got, exp = bits(params.cpu().numpy()), bits(ref.pull_params())
            bad = np.flatnonzero(got != exp)
            if bad.size:
                return f"step {st}: {bad.size}/{nparams} differ, first at {bad[0]}"
        return None
    finally:
        ps.close()
        ring.close()


def run_timing(rank: int, n: int) -> str | None:
    """ono_ring_timing_phases on the xGMI schedule: per round one scatter, two
    barriers, one gather and one local kernel (the owner chain); the RCCL
    phase stays empty; ono_ring_timing_read's collective total = phases 1..4."""
    ring = ono_amd.WorkerRingManager.over_xgmi(rank, n, 1 << 16, allgather, wire="f16")
    try:
        ring.timing(True)
        for _ in range(3):
            ring.pull_grads()
        torch.cuda.synchronize()
        ph, tot = ring.timing_phases(), ring.timing_read()
        want = {"kernel": 3, "rccl": 0, "xgmi_scatter": 3, "xgmi_barrier": 6, "xgmi_gather": 3, "sparse_codec": 0}
        got = {k: v[1] for k, v in ph.items()}
        if got != want:
            return f"phase counts {got} != {want}"
        coll = sum(v[0] for k, v in ph.items() if k not in ("kernel", "sparse_codec"))
        if abs(coll - tot["collective_ms"]) > 1e-6 or tot["collectives"] != 12 or tot["kernels"] != 3:
            return f"timing_read {tot} inconsistent with phases {ph}"
        if not all(v[0] > 0 for k, v in ph.items() if k not in ("rccl", "sparse_codec")):
            return f"empty phase time {ph}"
        return None
    finally:
        ring.close()


def run_timeout(rank: int, n: int, how: str = "env") -> str | None:
    """Rank 0 starts a round alone: its barrier gives up after the timeout and
    the next call fails with IoError instead of hanging; the late rank's
    teardown is bounded too.  how: "env" (ONO_XGMI_TIMEOUT_S when the region
    is made), "api" (ono_ring_set_xgmi_timeout on a live ring), "host" (the
    host-fed round must itself report the timed-out barrier: its output is
    invalid and the host residual already zeroed)."""
    os.environ["ONO_XGMI_TIMEOUT_S"] = "2" if how == "env" else "10"  # read when the region is allocated
    try:
        ring = ono_amd.WorkerRingManager.over_xgmi(rank, n, 4096, allgather, wire="f32")
    finally:
        os.environ["ONO_XGMI_TIMEOUT_S"] = "10"
    try:
        if how != "env":
            ring.set_xgmi_timeout(2.0)
        if rank == 0:
            t0 = time.time()
            if how == "host":
                res = np.ones(4096, np.float32)
                grad = np.zeros(4096, np.float32)
                try:
                    ring.pull_grads_host(res, grad)
                except ono_amd.IoError:
                    pass
                else:
                    return "a host-fed round over a timed-out barrier reported success"
            else:
                ring.pull_grads()
                torch.cuda.synchronize()
            waited = time.time() - t0
            try:
                ring.check()
            except ono_amd.IoError:
                pass
            else:
                return "check() after a timed-out barrier did not raise IoError"
            try:
                ring.pull_grads()
            except ono_amd.IoError:
                pass
            else:
                return "second pull_grads after a timed-out barrier did not raise IoError"
            if not 1.0 <= waited <= 30.0:
                return f"barrier waited {waited:.1f} s (timeout 2 s)"
        dist.barrier()
        return None
    finally:
        ring.close()


def describe_bad(bad, got, want, ins, prev, length, n, wire="f16", prev_ins=None) -> str:
    """What a wrong host-fed result looks like, for the next diagnosis: the runs of
    differing elements, the 1 MiB sub-rounds and the n owner chunks they fall in, and whether the wrong
    values are the previous cycle's result, one rank's unreduced input, zeros, the round without one
    rank's input (a push or chain read that saw zeroed lines) or with one rank's previous-cycle input
    (one that saw stale lines)."""
    runs = np.split(bad, np.flatnonzero(np.diff(bad) != 1) + 1)
    spans = ", ".join(f"[{r[0]}, {r[-1] + 1})" for r in runs[:6]) + (" ..." if len(runs) > 6 else "")
    sub = sorted(set((bad // (1 << 18)).tolist()))[:8]
    chunk = -(-length // n)
    owners = sorted(set((bad // chunk).tolist()))
    g = got[bad]
    kinds = []
    if prev is not None and np.array_equal(bits(g), bits(prev[bad])):
        kinds.append("= the previous cycle's result")
    for r, x in enumerate(ins):
        if np.array_equal(bits(g), bits(np.asarray(x, np.float32)[bad])):
            kinds.append(f"= rank {r}'s input")
    if not np.any(g):
        kinds.append("all zero")
    for r in range(n):  # every rank of a ring ends with the same result: e[0] stands for all
        variants = [("without", np.zeros(length, np.float32))]
        if prev_ins is not None:
            variants.append(("with the previous cycle's", np.asarray(prev_ins[r], np.float32)))
        for label, x in variants:
            alt = [np.asarray(v, np.float32) if q != r else x for q, v in enumerate(ins)]
            e, _ = O.ring_pull_grads(alt, wire)
            hit = int(np.count_nonzero(O.same_or_both_nan(g, e[0][bad])))
            if hit:
                kinds.append(f"{hit}/{bad.size} = the round {label} rank {r}'s input")
    lines = sorted(set((bad * 4 // 128 % 64).tolist()))[:8]  # 128-B line of the f32 bucket within 8 KiB
    return f"{len(runs)} runs {spans}; sub-rounds {sub}; owner chunks {owners}; lines in 8 KiB {lines}; " \
           f"wrong values {kinds or ['other']}"


# IPC handles this process has exported, across every case (a repeat of one from an earlier case is just
# as much a repeat: round 4's wrong result came in the first cycle of a case after another case's release)
SEEN_HANDLES: set = set()
POOLED: set = set()  # handles of this process's regions pooled right now (reused by design: not a repeat)
HANDLE_REPEATS = 0


def run_recreate(rank: int, n: int, case: dict) -> str | None:
    """Create, use and destroy an xGMI ring several times in the same processes
    (the situation of round 2's one wrong host-fed result: the second ring of a
    process).  Every connect verifies each peer mapping page by page against
    the ring id in that peer's handle (a stale import is an IoError at
    connect); every cycle runs the host-fed sub-round round bit-exact."""
    global HANDLE_REPEATS
    cycles, length = case.get("cycles", 6), case.get("length", (1 << 20) + 3)
    release = case.get("release", False)  # the pool released between cycles: fresh exports and imports
    freed = 0
    prev = None  # the previous cycle's expected result (stale data from an earlier ring would equal it)
    prev_ins = None  # and its inputs
    for cyc in range(cycles):
        blobs = {}

        def ag(b: bytes) -> list:
            blobs["mine"] = b
            return allgather(b)
        ring = ono_amd.WorkerRingManager.over_xgmi(rank, n, length, ag, wire=case.get("wire", "f16"))
        try:
            ipc = blobs["mine"][:64]
            if ipc in SEEN_HANDLES and ipc not in POOLED:  # a fresh region under a handle handed out before
                HANDLE_REPEATS += 1
                return f"cycle {cyc}: a fresh exchange region repeats an IPC handle exported before"
            SEEN_HANDLES.add(ipc)
            POOLED.add(ipc)  # back in the pool after close, until a release frees it
            ins = [O.synth(length, SEED + 1000 * cyc, r) for r in range(n)]
            expect, _ = O.ring_pull_grads(ins, case.get("wire", "f16"))
            res_h = np.ascontiguousarray(ins[rank]).copy()
            grad_h = np.full(length, 7.0, np.float32)
            ring.pull_grads_host(res_h, grad_h)
            bad = np.flatnonzero(~O.same_or_both_nan(grad_h, expect[rank]))
            if bad.size:
                return f"cycle {cyc}: {bad.size}/{length} differ, first at {bad[0]} (handle repeats {HANDLE_REPEATS}); " \
                       + describe_bad(bad, grad_h, expect[rank], ins, prev, length, n, case.get("wire", "f16"),
                                      prev_ins)
            prev, prev_ins = expect[rank], ins
            if bits(res_h).any():
                return f"cycle {cyc}: host residual not zeroed"
            if release:  # refused while this process's ring is alive
                try:
                    ono_amd.xgmi_pool_release()
                    return f"cycle {cyc}: pool release accepted while a ring is alive"
                except ono_amd.InvalidArgument:
                    pass
        finally:
            ring.close()
        if release:  # the two phases (ono_reduce.h): close imports everywhere, a collective step, free
            dist.barrier()  # every rank's ring destroyed
            closed = ono_amd.xgmi_pool_close_imports()
            st = ono_amd.xgmi_pool_stats()
            if closed != n - 1 or st["imports"]:
                return f"cycle {cyc}: closed {closed} imports, stats after {st}"
            dist.barrier()  # every import of every region closed before anyone frees
            r = ono_amd.xgmi_pool_free_exports(30.0)
            st = ono_amd.xgmi_pool_stats()
            if r["freed_bytes"] <= 0 or r["kept"] or st["regions"]:
                return f"cycle {cyc}: free_exports {r}, stats after {st}"
            freed += r["freed_bytes"]
            POOLED.clear()
            dist.barrier()  # every region freed before the next ring allocates
    print(json.dumps({"rank": rank, "recreate_ipc_handle_repeats": HANDLE_REPEATS, "cycles": cycles,
                      "released_bytes": freed}),
          file=sys.stderr)
    return None


def run_host_fence(rank: int, n: int, case: dict) -> str | None:
    """Host-fed rounds under each input form in turn, each bit-exact: "kernel" (the
    default: a copy kernel writes the residual from the caller's registered bucket or a pinned staging slot,
    an L2 write-back on every XCD before each D2H), "dma+fence" (the copy engine's H2D with write-back +
    invalidate fences around it), "dma" (the copy engine alone, round 5's form); ONO_XGMI_HOST_IN /
    ONO_XGMI_HOST_FENCE are read per call.  Rank 0 writes the wall times of every form to gpurun_out/ when
    it exists (their cost)."""
    length, wire, rounds = case.get("length", 1 << 22), case.get("wire", "f32"), case.get("rounds", 6)
    forms = {"kernel": {}, "kernel-nt": {"ONO_XGMI_HOST_IN": "plain"},
             "dma+fence": {"ONO_XGMI_HOST_IN": "dma", "ONO_XGMI_HOST_FENCE": "1"},
             "dma": {"ONO_XGMI_HOST_IN": "dma", "ONO_XGMI_HOST_FENCE": "0"}}
    modes = case.get("modes", list(forms))
    ring = ono_amd.WorkerRingManager.over_xgmi(rank, n, length, allgather, wire=wire)
    times = {m: [] for m in modes}
    try:
        for i in range(len(modes) * rounds):
            mode = modes[i % len(modes)]
            for k in ("ONO_XGMI_HOST_IN", "ONO_XGMI_HOST_FENCE"):
                os.environ.pop(k, None)
            os.environ.update(forms[mode])
            ins = [O.synth(length, SEED + 17 * i, r) for r in range(n)]
            expect, _ = O.ring_pull_grads(ins, wire)
            res_h = np.ascontiguousarray(ins[rank]).copy()
            grad_h = np.full(length, 7.0, np.float32)
            if case.get("registered"):
                ring.register_host(res_h)
                ring.register_host(grad_h)
            dist.barrier()
            t0 = time.perf_counter()
            ring.pull_grads_host(res_h, grad_h)
            times[mode].append((time.perf_counter() - t0) * 1e3)
            if case.get("registered"):
                ring.unregister_host(res_h)
                ring.unregister_host(grad_h)
            bad = np.flatnonzero(~O.same_or_both_nan(grad_h, expect[rank]))
            if bad.size:
                return f"round {i} ({mode}): {bad.size}/{length} differ, first at {bad[0]}"
            if bits(res_h).any():
                return f"round {i} ({mode}): host residual not zeroed"
    finally:
        for k in ("ONO_XGMI_HOST_IN", "ONO_XGMI_HOST_FENCE"):
            os.environ.pop(k, None)
        ring.close()
    out = os.path.join(ROOT, "gpurun_out")
    if rank == 0 and os.path.isdir(out):
        med = {k: float(np.median(v[1:])) for k, v in times.items()}  # the first of each: warm-up
        tag = "_registered" if case.get("registered") else ""
        with open(os.path.join(out, f"xgmi_host_fence_n{n}{tag}.json"), "w") as f:
            json.dump({"n": n, "length": length, "wire": wire, "ms": times, "median_ms_after_first": med}, f)
    return None


def main() -> int:
    rank, n, rdv = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    cases = json.loads(sys.argv[4])
    torch.cuda.set_device(0)
    # rendezvous through a file the parent made unique (no port to collide with), or a port
    init = rdv if rdv.startswith("file://") else f"tcp://127.0.0.1:{int(rdv)}"
    dist.init_process_group("gloo", rank=rank, world_size=n, init_method=init)
    results = []
    for case in cases:
        try:
            kind = case.get("kind", "ring")
            msg = run_timeout(rank, n, case.get("how", "env")) if kind == "timeout" else run_ps(rank, n, case) if kind == "ps" else \
                run_timing(rank, n) if kind == "timing" else run_recreate(rank, n, case) if kind == "recreate" else \
                run_host_fence(rank, n, case) if kind == "host_fence" else run_case(rank, n, case)
        except Exception as e:  # reported, the parent asserts
            msg = f"{type(e).__name__}: {e}"
        results.append({"case": case, "ok": msg is None, "msg": msg or ""})
        dist.barrier()
    print(json.dumps({"rank": rank, "results": results}), flush=True)
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
