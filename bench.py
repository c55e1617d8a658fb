#!/usr/bin/env python3
"""bench.py — device-resident f32 gradient all-reduce of a 256 MiB bucket.

Metric (BASELINE.json): "GiB/s device-resident f32 gradient all-reduce,
256 MiB bucket, 1/2/4/8 GPUs".

One process per GPU (python -m torch.distributed.run --nproc-per-node N
bench.py --gpus N ...; single process for N = 1).  A *step* is one
WorkerRingManager::pull_grads round (worker/src/middlewares/worker_ring.rs:82-94)
on every rank over a freshly produced 256 MiB residual bucket already
resident in HBM: grad = (sum over ranks of residual) / N, residual = 0.
  N = 1   the reference's n == 1 round: grad = residual, residual = 0 (no
          division, worker_ring.rs:166-171) — one fused gfx950 kernel.
  N > 1   RCCL all-reduce over xGMI + one fused kernel (grad /= N, residual = 0);
          --algo selects another schedule (hops, direct, xgmi).
Every timed step consumes its own pre-generated residual bucket (W + K buckets
of 256 MiB in HBM), so no step reduces an already-zeroed bucket.

value = N * bucket_bytes * K / max-over-ranks(elapsed) / 2^30: the gradient
bytes every rank fed into the reduction per second (weak scaling: the bucket
per GPU is fixed).  algbw_gib_s (bucket / time) and busbw_gib_s
(algbw * 2(N-1)/N) are reported beside it.

Extra objects on the JSON line:
  check         the last timed step against the exact average of all N inputs
                (regenerated on every rank), residual all zero
  roofline      the step's dominant kernel (N = 1: HBM) or exchange (N > 1: xGMI
                links), achieved vs peak, from HIP events on the launch stream;
                N > 1 also splits the step by phase (ono_ring_timing_phases)
  local_reduce  BASELINE config 2: the 64 MiB sum-and-scale kernel, k = 2, 4, 8
  path_kernels  the path's other kernels (acc_residual, hop codec, consumer
                optimizers) against the HBM roofline, PMC traffic beside
  sparse_codec  the device top-k codec (drop / lift) on a 64 MiB gradient
  host_fed      PCIe-inclusive pull_grads from host buffers (registered / pageable)
  ps_host_fed   the device store fed from host buffers (f32 and f16 wire payloads)
  tcp_edge      MI355X workers in a loopback-TCP ring speaking the reference's frames
  cpu_baseline  the reference-style CPU ring (TCP loopback, f16 wire, one pinned
                core per worker) on the same host, rank 0 at N = 1 only
  xgmi_coresident  N = 1: the xGMI peer-access schedule as 2 processes on the GPU
  alt_schedules N > 1: the other exchange schedules (RCCL single all-reduce,
                DIRECT f32/f16, HOPS f16, PS mode) behind a watchdog, and the
                xGMI schedule (pull / push gather, both wires, PS step) in child
                processes that are killed if they hang
  size_sweep    N > 1: the main schedule from the config-1 bucket to 1 GiB
Every informational object records its own failure instead of ending the line.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "oxidized-neural-orchestra_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "GiB/s device-resident f32 gradient all-reduce, 256 MiB bucket, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level table)
XGMI_LINK_GBS = 153.6 / 2      # per direction; 153.6 GB/s bidirectional per link (spec)
GIB = float(1 << 30)
SEED = 0x0402026
CONFIG1_ELEMS = (784 + 1) * 128 + (128 + 1) * 64 + (64 + 1) * 10  # 109,386: MLP 784-128-64-10


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--bucket-mib", type=int, default=256)
    ap.add_argument("--wire", choices=["f32", "f16"], default="f32")
    ap.add_argument("--algo", choices=["auto", "allreduce", "hops", "direct", "xgmi"], default="auto")
    ap.add_argument("--segments", type=int, default=0,
                    help="f32 all-reduce pipeline segments (0 = library default: ONO_AR_SEGMENTS or 4)")
    ap.add_argument("--alt-schedules", default="allreduce:f32:1,direct:f32,direct:f16,hops:f16",
                    help="N > 1 only: extra schedules measured after the main line "
                         "(algo:wire[:segments],...; '' = none)")
    ap.add_argument("--sweep-mib", default="1,4,16,64,256,1024",
                    help="N > 1 (or --alt-at-n1): bucket-size sweep of the main schedule, MiB list ('' = none)")
    ap.add_argument("--alt-timeout", type=float, default=300.0)
    ap.add_argument("--alt-at-n1", action="store_true", help="exercise the alternative-schedule plumbing at N = 1")
    ap.add_argument("--no-ps-mode", dest="ps_mode", action="store_false",
                    help="skip the N > 1 parameter-server (RS + update + AG) measurement")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-local-reduce", action="store_true")
    ap.add_argument("--no-host-fed", action="store_true")
    ap.add_argument("--no-tcp-edge", action="store_true")
    ap.add_argument("--no-xgmi", dest="xgmi", action="store_false",
                    help="N > 1: skip the xGMI peer-access schedule (measured in child processes)")
    ap.add_argument("--xgmi-timeout", type=float, default=240.0)
    ap.add_argument("--xgmi-coresident", type=int, default=2,
                    help="N = 1: also run the xGMI schedule with this many ranks as processes on the one GPU "
                         "(HBM stands in for the links; informational; 0 = off)")
    ap.add_argument("--xgmi-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal on a one-GPU box: every rank on device 0 (with --algo xgmi, which needs no "
                         "RCCL, the whole N > 1 flow runs: torchrun launch, rings, checks, children, JSON line)")
    ap.add_argument("--cpu-ranks", type=int, default=2)
    ap.add_argument("--cpu-rounds", type=int, default=3)
    ap.add_argument("--deadline", type=float, default=420.0,
                    help="seconds from the start for the whole line: the headline is measured and checked first, "
                         "an informational leg that would not finish in time is skipped (recorded as skipped), and "
                         "a leg still running at the deadline + 45 s is cut (the line is printed as it stands)")
    # CPU plumbing tests only: no GPU, the steps and legs are sleeps (tests/test_bench_harness.py)
    ap.add_argument("--dry-run", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--dry-leg-s", type=float, default=0.0, help=argparse.SUPPRESS)
    return ap.parse_args(argv)


# ------------------------------------------------------------- control plane
class Ctl:
    """Barrier / max / broadcast across ranks over gloo (CPU tensors only, so
    the control plane never touches the GPU streams being timed)."""

    def __init__(self, world: int, rank: int):
        self.world, self.rank = world, rank
        self.dist = None
        if world > 1:
            import torch.distributed as dist
            if not dist.is_initialized():
                rdv = os.environ.get("ONO_BENCH_RDV")  # file:// rendezvous of the xGMI children (no port to race for)
                if rdv:
                    dist.init_process_group("gloo", rank=rank, world_size=world, init_method=rdv)
                else:
                    dist.init_process_group("gloo", rank=rank, world_size=world)
            self.dist = dist

    def barrier(self) -> None:
        if self.dist:
            self.dist.barrier()

    def max(self, x: float) -> float:
        if not self.dist:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def bcast_bytes(self, b: bytes | None) -> bytes:
        if not self.dist:
            return b
        obj = [b]
        self.dist.broadcast_object_list(obj, src=0)
        return obj[0]

    def allgather_bytes(self, b: bytes) -> list:
        if not self.dist:
            return [b]
        out = [None] * self.world
        self.dist.all_gather_object(out, b)
        return out

    def close(self) -> None:
        if self.dist and self.dist.is_initialized():
            self.dist.destroy_process_group()


def timed_region(step, steps: int, warmup: int, sync, ctl: Ctl, on_start=None) -> tuple[float, float]:
    """W untimed steps, then exactly K steps bracketed by sync + barrier;
    returns (max-over-ranks elapsed, local elapsed) in seconds.  `on_start`
    runs after the warmup drained, before the opening barrier."""
    for i in range(warmup):
        step(i)
    sync()
    if on_start is not None:
        on_start()
    ctl.barrier()
    t0 = time.perf_counter()
    for i in range(steps):
        step(warmup + i)
    sync()
    t1 = time.perf_counter()
    ctl.barrier()
    local = t1 - t0
    return ctl.max(local), local


def build_line(*, value, n_gpus, steps, warmup, elapsed, bucket_bytes, wire, extra) -> dict:
    algbw = bucket_bytes * steps / elapsed / GIB
    line = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": n_gpus,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": round(elapsed / steps * 1e3, 6),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (SURVEY §8(d) distribution, counter-based generator, fresh bucket per step)",
        "config": {
            "workload": "pull_grads round: device-resident f32 all-reduce + average of a 256 MiB gradient bucket per GPU",
            "bucket_mib": bucket_bytes / (1 << 20),
            "bucket_elems": bucket_bytes // 4,
            "global_batch": n_gpus,
            "parallelism": f"dp{n_gpus}",
            "wire": wire,
            "collective": "none (n == 1)" if n_gpus == 1 else ("RCCL all-reduce over xGMI" if wire == "f32"
                                                                 else "reference f16 arithmetic, DIRECT all-to-all "
                                                                      "over RCCL p2p"),
        },
        "algbw_gib_s": round(algbw, 3),
        "busbw_gib_s": round(algbw * 2 * (n_gpus - 1) / n_gpus, 3) if n_gpus > 1 else None,
    }
    line.update(extra)
    return line


# -------------------------------------------------------------- PMC traffic
def pmc_traffic(kernel_substr: str, elems: int) -> dict | None:
    """HBM bytes per launch of the dominant kernel from the committed PMC
    summary (profiles/*pmc*.json written by tools/pmc_summary.py), matched on
    the kernel name and bucket size — the most recently recorded one
    (recorded_utc; summaries without it rank first, by file name); None when
    no such summary exists."""
    best, best_key = None, None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):
        try:
            with open(f) as fh:
                d = json.load(fh)
        except (OSError, ValueError):
            continue
        key = (d.get("recorded_utc", ""), os.path.basename(f))
        for k in d.get("kernels", []):
            if kernel_substr in k.get("name", "") and k.get("elems") == elems and (best_key is None or key >= best_key):
                best, best_key = dict(k, source=os.path.relpath(f, ROOT), commit=d.get("commit", "unknown"),
                                      session=d.get("session") or "a builder session"), key
    return best


# ------------------------------------------------------------- CPU baseline
def cpu_baseline(bucket_elems: int, ranks: int, rounds: int) -> dict:
    """The reference CPU ring restated in C (oracle/ono_cpu_ring.c): n worker
    threads, one pinned core each, loopback TCP, f16 wire, reference framing.
    Checker-side code: it is timed here as the baseline, never used by the
    product path."""
    from oracle import oracle as O  # noqa: WPS433 (cpu_baseline leg only)

    r = O.cpu_ring(ranks, bucket_elems, rounds, check=False, pin=True, timeout=900)
    hop = O.cpu_ps("hop", bucket_elems // ranks, rounds=rounds)
    ps = O.cpu_ps("ps", bucket_elems, threads=16, workers=ranks, rounds=rounds)
    try:  # -march=native variants, compiled here for this host (BASELINE.md CPU plan)
        import tempfile
        with tempfile.TemporaryDirectory() as d:
            exes = O.build_native(d)
            rn = O.cpu_ring(ranks, bucket_elems, rounds, check=False, pin=True, timeout=900,
                            exe=exes["ono_cpu_ring"])
            hn = O.cpu_ps("hop", bucket_elems // ranks, rounds=rounds, exe=exes["ono_cpu_ps"])
        native = {"ring_gib_s": round(rn["gib_s"], 4), "hop_compute_1core_gib_s": hn["gib_s"],
                  "flags": "-O3 -march=native (built on this host)"}
    except Exception as e:  # reported, never fatal
        native = {"error": f"{type(e).__name__}: {e}"[:200]}
    return {
        "value": round(r["gib_s"], 4),
        "unit": "GiB/s",
        "cores": ranks,
        "kind": "port",
        "sample": (f"one {bucket_elems * 4 / (1 << 20):.0f} MiB f32 bucket per worker, {ranks} workers "
                   f"(threads pinned to 1 core each, loopback TCP, reference framing + f16 wire), "
                   f"{rounds} pull_grads rounds, {r['s_per_round']:.3f} s/round; C -O3 default x86-64"),
        "host_cpu": _cpu_model(),
        "host_nproc": os.cpu_count(),
        # SURVEY §8(d) items (i) and (iii), same host, same run
        "hop_compute_1core": {"gib_s": hop["gib_s"], "s_per_hop": hop["s_per_hop"],
                              "sample": f"{hop['len']} elems: f16 encode + decode + f32 add, 1 core"},
        "ps_accumulate_update": {"gib_s": ps["gib_s"], "s_per_round": ps["s_per_round"], "cores": ps["threads"],
                                 "sample": f"BlockingStore: {ps['workers']} accumulates + 1 update (÷n, GD) of "
                                           f"{ps['len']} params, {ps['shards']} shards on {ps['threads']} pinned cores"},
        "march_native": native,
        "ring_by_ranks": ring_by_ranks(bucket_elems, ranks),
        "sparse_ring": sparse_ring_baseline(),
    }


def usable_cpus() -> int:
    """CPUs this process may keep busy: its affinity set, capped by the cgroup's
    cpu.max quota (a GPU box grants 16 CPUs of a 256-CPU host)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return n


def ring_by_ranks(bucket_elems: int, done: int, ranks=(2, 4, 8), rounds: int = 2) -> dict:
    """BASELINE.md's CPU plan at every GPU count of the scaling line: the reference-style CPU ring with n = 2, 4,
    8 workers (one pinned core each, as docker/gen_compose.py:9 deploys them) on the same 256 MiB bucket per
    worker, so the N = 2 / 4 / 8 GPU lines have a same-n CPU figure from one run.  An n is run only when the
    process may use n + 1 CPUs (n pinned workers and the driver); the cores used are recorded."""
    from oracle import oracle as O  # noqa: WPS433 (cpu_baseline leg only)
    cpus = usable_cpus()
    out = {"usable_cpus": cpus}
    for n in ranks:
        if n == done:
            continue  # (the line's own cpu_baseline)
        if n + 1 > cpus:
            out[str(n)] = {"skipped": f"needs {n + 1} CPUs, the process may use {cpus}"}
            continue
        try:
            r = O.cpu_ring(n, bucket_elems, rounds, check=False, pin=True, timeout=600)
            out[str(n)] = {"gib_s_per_worker": round(r["gib_s"], 4), "s_per_round": round(r["s_per_round"], 4),
                           "cores": n, "workers_pinned": r.get("workers_pinned"), "rounds": rounds,
                           "aggregate_gib_s": round(r["gib_s"] * n, 4)}
        except Exception as e:  # noqa: BLE001
            out[str(n)] = {"error": f"{type(e).__name__}: {e}"[:200]}
    return out


def sparse_ring_baseline(ratio: float = 0.1, rounds: int = 20) -> dict:
    """Config 1 with SparseCapable{ratio} workers: the reference-style CPU ring (one process per worker,
    oracle/ono_cpu_ring.c) timed beside the MI355X TCP ring, and the MI355X ring's last round checked bit
    for bit against the oracle's replay of every round (ono_ref_ring_pull_grads_sparse, the samplers'
    states carried).  Checker-side code (the cpu_baseline leg)."""
    import socket
    import tempfile
    import numpy as np
    from oracle import oracle as O  # noqa: WPS433 (cpu_baseline leg only)
    out = {"ratio": ratio, "elems": CONFIG1_ELEMS, "ranks": 2}
    try:
        ports = []
        for _ in range(2):
            with socket.socket() as so:
                so.bind(("127.0.0.1", 0))
                ports.append(so.getsockname()[1])
        ws = [O.CpuRingWorker(r, 2, CONFIG1_ELEMS, ports[(r + 1) % 2], rounds=rounds, listen_port=ports[r],
                              sparse=ratio, sparse_seed=0x5EED0000 + r) for r in range(2)]
        infos = [w.result(300)[2] for w in ws]
        out["cpu_ms_per_round"] = round(max(i["s_per_round"] for i in infos) * 1e3, 4)
        out["cpu_cores"] = 2
    except Exception as e:  # noqa: BLE001
        out["cpu_error"] = f"{type(e).__name__}: {e}"[:200]
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "r0.bin")
        g = tcp_sparse_native(CONFIG1_ELEMS, rounds, 2, ratio, dump=path)
        if not g or "error" in g:
            out["gpu_error"] = (g or {}).get("error", "tools/ono_tcp_bench not built")
            return out
        out["gpu_ms_per_round"] = g["ms"]
        got = np.fromfile(path, dtype=np.float32)
    states = [0x5EED0000 + r for r in range(2)]
    for k in range(rounds + 1):  # the tool's rounds: warmup + timed, a fresh bucket each, samplers carried
        ins = [O.synth(CONFIG1_ELEMS, 0x0402026 + k, r) for r in range(2)]
        grads, res, states = O.ring_pull_grads_sparse(ins, [ratio, ratio], states)
    L = CONFIG1_ELEMS
    bad = int((~O.same_or_both_nan(got[:L], grads[0])).sum() + (~O.same_or_both_nan(got[L:], res[0])).sum())
    out["check"] = {"ok": bad == 0, "values_differing": bad, "rounds_replayed": rounds + 1,
                    "what": "rank 0's grad and residual after the last round vs the oracle's sparse ring"}
    if out.get("cpu_ms_per_round") and out.get("gpu_ms_per_round"):
        out["speedup"] = round(out["cpu_ms_per_round"] / out["gpu_ms_per_round"], 2)
    return out


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# ---------------------------------------------------------- local reduce
def local_reduce(torch, ono_amd, steps: int, warmup: int, ks=(2, 4, 8), warm_rotations: int = 1,
                 settle_s: float = 0.0, passes: int = 3) -> dict:
    """BASELINE config 2: ono_sum_scale_f32 over k 64 MiB buckets (÷k),
    device time from one HIP event pair on the launch stream around the K
    back-to-back launches (per-launch event pairs add ~2 us to a 30 us
    kernel, tools/stream_variants.hip "pull" mode).  Launches rotate over
    enough input/output sets that every launch reads from HBM (the working
    set exceeds the 256 MiB Infinity Cache by > 4x).

    One pool of 64 MiB buffers serves every k (allocated once: the same
    kernel measured over freshly allocated buffers moved by up to 4 % with the
    placement, profiles/r04_lr_ab_s{3,4}.txt), and each k is measured in
    `passes` passes interleaved with the other k's; the reported figure is the
    median pass (min / max beside it).  The same passes time the library's
    1R2W copy (`scale_zero` with divisor 1: read one bucket, write two — the
    12 B per element of k = 2) over k = 2's sets, so config 2 also reads
    against a ceiling measured on the same buffers in the same passes
    (`copy_zero_same_pool`, `frac_of_same_pool_copy_zero`): the placement of a
    set moves a 64 MiB launch by 2-4 %, more than the kernels differ.
    ks / warm_rotations / settle_s: knobs for tools/lr_ab.py (warm-up
    rotations; a synchronised pause before it)."""
    n = 16 << 20
    out = {}
    stream = torch.cuda.Stream()  # a stream of its own (the ring's reductions run on the caller's)
    nsets = {k: 1536 // ((k + 1) * 64) + 2 for k in ks}  # > 1.5 GiB per rotation: every launch reads HBM
    pool = []
    for b in range(max(nsets[k] * (k + 1) for k in ks)):
        pool.append(ono_amd.kernels.synth(torch.empty(n, dtype=torch.float32, device="cuda"), SEED + b // 9, b % 9))
    sets = {k: [(pool[s * (k + 1):s * (k + 1) + k], pool[s * (k + 1) + k]) for s in range(nsets[k])] for k in ks}
    # the 1R2W copy over k = 2's sets: read the set's first input, write its output and a zero buffer of
    # the set's own (the inputs stay intact for the sums)
    cz_sets = []
    if 2 in ks:
        cz_sets = [(ins[0], dst, torch.zeros(n, dtype=torch.float32, device="cuda")) for ins, dst in sets[2]]
    ms = {k: [] for k in ks}
    cz_ms = []
    for _ in range(passes):
        if cz_sets:
            ns = len(cz_sets)
            warm = max(warmup, ns * warm_rotations)
            for i in range(warm):
                src, dst, zero = cz_sets[i % ns]
                ono_amd.kernels.scale_zero(dst, src, 1.0, zero, stream)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            for i in range(steps):
                src, dst, zero = cz_sets[(warm + i) % ns]
                ono_amd.kernels.scale_zero(dst, src, 1.0, zero, stream)
            b.record(stream)
            b.synchronize()
            cz_ms.append(a.elapsed_time(b) / steps)
        for k in ks:
            ns = nsets[k]
            if settle_s:
                torch.cuda.synchronize()
                time.sleep(settle_s)
            # the warm-up covers a whole rotation (every set's pages touched); no synchronisation
            # between it and the opening event: the GPU is still busy with the warm-up when `a` is
            # recorded, so the host enqueues the timed launches ahead of the GPU and the span holds K
            # back-to-back kernels, not the host's latency to the first one (~10 us through Python:
            # 0.5 us per launch at K = 20, 1.5 % of a 64 MiB sum2)
            warm = max(warmup, ns * warm_rotations)
            for i in range(warm):
                ins, dst = sets[k][i % ns]
                ono_amd.kernels.sum_scale(dst, ins, float(k), stream)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            for i in range(steps):
                ins, dst = sets[k][(warm + i) % ns]
                ono_amd.kernels.sum_scale(dst, ins, float(k), stream)
            b.record(stream)
            b.synchronize()
            ms[k].append(a.elapsed_time(b) / steps)
    for k in ks:
        v = sorted(ms[k])
        med = v[len(v) // 2]
        nbytes = (k + 1) * 4 * n
        gbs = nbytes / (med * 1e-3) / 1e9
        pmc = pmc_traffic(f"SumScaleOp<{k},", n)
        out[f"k{k}"] = {"bytes_per_launch": nbytes, "us_per_launch": round(med * 1e3, 2),
                        "achieved_gbs": round(gbs, 1), "frac_of_hbm_peak": round(gbs / HBM_PEAK_GBS, 4),
                        "us_per_launch_min": round(v[0] * 1e3, 2), "us_per_launch_max": round(v[-1] * 1e3, 2),
                        "passes": len(v), "rotating_sets": nsets[k],
                        "traffic": pmc["hbm_bytes_per_launch"] if pmc else None}
    if cz_ms:
        v = sorted(cz_ms)
        med = v[len(v) // 2]
        gbs = 12 * n / (med * 1e-3) / 1e9
        out["copy_zero_same_pool"] = {"bytes_per_launch": 12 * n, "us_per_launch": round(med * 1e3, 2),
                                      "achieved_gbs": round(gbs, 1), "frac_of_hbm_peak": round(gbs / HBM_PEAK_GBS, 4),
                                      "us_per_launch_min": round(v[0] * 1e3, 2),
                                      "us_per_launch_max": round(v[-1] * 1e3, 2), "passes": len(v),
                                      "rotating_sets": len(cz_sets),
                                      "shape": "ono_scale_zero_f32 /1 (1R2W, 12 B/elem) over k = 2's sets"}
        for k in ks:
            out[f"k{k}"]["frac_of_same_pool_copy_zero"] = round(out[f"k{k}"]["achieved_gbs"] / gbs, 4)
    del sets, pool, cz_sets
    torch.cuda.empty_cache()
    return {"workload": "sum_scale_f32, 64 MiB buckets, out = (sum of k inputs) / k", "hbm_peak_gbs": HBM_PEAK_GBS,
            "timing": f"one HIP event pair around K back-to-back launches (inter-kernel gaps included); median "
                      f"of {passes} passes interleaved across k, over one buffer pool",
            **out}


def copy_ceiling(torch, ono_amd, steps: int, warmup: int) -> dict:
    """SURVEY §8(d) "also record a measured copy-kernel ceiling": the best pure
    streams this library writes, on the path kernels' own skeleton (one-wave
    workgroups, one 16-B vector per lane, one-shot grid, nt policy), at the
    headline bucket (256 MiB) and the config-2 size (64 MiB):
      copy       ono_copy_f32          1R1W   8 B/elem
      copy_zero  ono_scale_zero_f32    1R2W  12 B/elem  (divisor 1: dst = src, zero = 0)
      fill       ono_fill_f32          0R1W   4 B/elem
    `ceiling_<size>` is the fastest of the three in algorithmic bytes per second;
    the path's kernels are read against it (`frac_of_copy_ceiling`).  The HIP
    runtime's own D2D copy and fill (torch copy_ / zero_) are timed beside them
    for reference.  Timed like the path's kernels: one event pair around K
    back-to-back launches over rotating sets larger than the Infinity Cache."""
    out = {}
    stream = torch.cuda.current_stream()
    lib_shapes = (("copy", 8, lambda st: ono_amd.kernels.copy(st[1], st[0])),
                  ("copy_zero", 12, lambda st: ono_amd.kernels.scale_zero(st[1], st[0], 1.0, st[2])),
                  ("fill", 4, lambda st: ono_amd.kernels.fill(st[1], 0.0)))
    rt_shapes = (("runtime_copy", 8, lambda st: st[1].copy_(st[0])), ("runtime_fill", 4, lambda st: st[1].zero_()))
    for mib in (256, 64):
        n = mib << 18
        nsets = max(2, 1536 // (3 * mib) + 1)
        sets = [tuple(torch.empty(n, dtype=torch.float32, device="cuda") for _ in range(3)) for _ in range(nsets)]
        for st in sets:
            ono_amd.kernels.synth(st[0], SEED, 0)
            st[1].zero_()
            st[2].zero_()
        best = None
        for name, per, fn in lib_shapes + rt_shapes:
            warm = max(warmup, nsets)
            for i in range(warm):
                fn(sets[i % nsets])
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)  # behind the warm-up, no synchronisation (see local_reduce)
            for i in range(steps):
                fn(sets[(warm + i) % nsets])
            b.record(stream)
            torch.cuda.synchronize()
            us = a.elapsed_time(b) / steps * 1e3
            gbs = per * n / (us * 1e-6) / 1e9
            row = {"bytes_per_launch": per * n, "us_per_launch": round(us, 2), "achieved_gbs": round(gbs, 1),
                   "frac_of_hbm_peak": round(gbs / HBM_PEAK_GBS, 4), "rotating_sets": nsets}
            out[f"{name}_{mib}MiB"] = row
            if not name.startswith("runtime") and (best is None or gbs > best[1]):
                best = (name, gbs)
        out[f"ceiling_{mib}MiB"] = {"shape": best[0], "achieved_gbs": round(best[1], 1),
                                    "frac_of_hbm_peak": round(best[1] / HBM_PEAK_GBS, 4)}
        del sets
        torch.cuda.empty_cache()
    return {"workload": "the library's own pure streams (ono_copy_f32 1R1W, ono_scale_zero_f32 /1 1R2W, "
                        "ono_fill_f32 0R1W) and the HIP runtime's D2D copy / fill, f32, device-resident",
            "hbm_peak_gbs": HBM_PEAK_GBS,
            "timing": "one HIP event pair around K back-to-back launches over rotating sets", **out}


def path_kernels(torch, ono_amd, steps: int, warmup: int) -> dict:
    """SURVEY §8(f) rows 1, 2 and 4 at the measurement bar: the remaining
    kernels of the path, each timed as one HIP event pair around K
    back-to-back launches over rotating buffer sets (> 1 GiB, so the Infinity
    Cache cannot serve re-reads), against the 8 TB/s HBM roofline:
      acc_residual       residual += grad (param_manager.rs:191-197)          12 B/elem
      f16_add_encode_zero  the hop kernel: acc + dec(in) -> enc -> out, acc = 0  12 B/elem
                         (worker_ring.rs:141-143 + :122, :133; the TCP edge's per-hop work)
      f16_decode_scale   gather receive (:200 + /n)                             6 B/elem
      consumer_{gd,momentum,adam}  optimize + zero_grad + params copy        20/28/36 B/elem
                         (all_reduce.rs:126-132, param_manager.rs:148-172)
    64 MiB f32 buckets (16 M elements)."""
    n = 16 << 20
    stream = torch.cuda.current_stream()
    f32 = lambda: torch.empty(n, dtype=torch.float32, device="cuda")  # noqa: E731
    u16 = lambda: torch.empty(n, dtype=torch.int16, device="cuda")  # noqa: E731
    out = {}

    def timed(name, kernel, per_elem, make_set, launch, nsets, elems=n, note=None):
        sets = [make_set(i) for i in range(nsets)]
        torch.cuda.synchronize()
        warm = max(warmup, nsets)  # a whole rotation: every set's pages touched once
        for i in range(warm):
            launch(sets[i % nsets])
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)  # behind the warm-up, no synchronisation (see local_reduce)
        for i in range(steps):
            launch(sets[(warm + i) % nsets])
        b.record(stream)
        torch.cuda.synchronize()
        us = a.elapsed_time(b) / steps * 1e3
        gbs = per_elem * elems / (us * 1e-6) / 1e9
        pmc = pmc_traffic(kernel, elems)
        out[name] = {"bytes_per_launch": per_elem * elems, "us_per_launch": round(us, 2),
                     "achieved_gbs": round(gbs, 1), "frac_of_hbm_peak": round(gbs / HBM_PEAK_GBS, 4),
                     "rotating_sets": nsets, "traffic": pmc["hbm_bytes_per_launch"] if pmc else None}
        if elems != n:
            out[name]["elems"] = elems
        if note:
            out[name]["note"] = note
        for st in sets:  # optimizer sets own device state
            for o in st:
                if hasattr(o, "close"):
                    o.close()
        del sets
        torch.cuda.empty_cache()

    def filled(i, r, m=n):
        return ono_amd.kernels.synth(torch.empty(m, dtype=torch.float32, device="cuda"), SEED + i, r)

    timed("acc_residual", "AccOp", 12, lambda i: (filled(i, 0), filled(i, 1)),
          lambda st: ono_amd.kernels.acc(st[0], st[1]), 6,
          note="ono_acc_f32 over fresh buffers (nt loads); the ring's acc_residual keeps its residual cacheable for "
               "the pull that follows (DESIGN §3)")

    def hop_set(i):
        h = u16()
        ono_amd.kernels.f16_encode(h, filled(i, 2))
        return (u16(), filled(i, 0), h)
    timed("f16_add_encode_zero", "AddEncodeZeroOp<unsigned short>", 12, hop_set,
          lambda st: ono_amd.kernels.f16_add_encode_zero(*st), 8)

    def dec_set(i):
        h = u16()
        ono_amd.kernels.f16_encode(h, filled(i, 3))
        return (f32(), h)
    timed("f16_decode_scale", "DecodeScaleOp<unsigned short", 6, dec_set,
          lambda st: ono_amd.kernels.f16_decode_scale(st[0], st[1], 8.0), 12)

    # The owner kernel of the DIRECT / XGMI schedules at the 8-GPU shape of the
    # headline bucket: 256 MiB / 8 ranks = 8 M-element chunks; 7 received
    # slices + the owner's own slice in, grad + the result message out, the
    # own slice zeroed (worker_ring.rs:122-143, :166, :133; zero_all = 0 as on
    # the xGMI ring).  f32: 8*4 + 4 + 4 + 4 = 44 B/elem; f16 message: 42.
    c8 = 8 << 20
    for wire, per in (("f32", 44), ("f16", 42)):
        def chain_set(i, wire=wire):
            ins = [filled(i, r, c8) for r in range(8)]
            msg = torch.empty(c8, dtype=torch.int16 if wire == "f16" else torch.float32, device="cuda")
            return (torch.empty(c8, dtype=torch.float32, device="cuda"), msg, ins)
        timed(f"owner_chain_{wire}_n8", "DirectOp<8, float" if wire == "f32" else "DirectOp<8, unsigned short", per,
              chain_set, lambda st, wire=wire: ono_amd.kernels.direct_chain(st[0], st[1], st[2], 8.0, wire), 5,
              elems=c8)

    # Consumer optimizers: every set has its own optimizer state, so the
    # momentum / Adam moments rotate with the gradients and parameters and no
    # launch can be served from the 256 MiB Infinity Cache (a training loop
    # reuses one state set; that regime is cache-assisted and is not an HBM figure).
    for name, kind, opt, per in (("gd", 0, ono_amd.GradientDescent(0.1), 20),
                                 ("momentum", 1, ono_amd.GradientDescentWithMomentum(0.1, 0.9), 28),
                                 ("adam", 2, ono_amd.Adam(1e-3, 0.9, 0.999, 1e-8), 36)):
        timed(f"consumer_{name}", f"OptOp<{kind},", per,
              lambda i, opt=opt: (filled(i, 4), filled(i, 5), f32(), ono_amd.DeviceOptimizer(opt, n)),
              lambda st: st[3].step(st[0], st[1], st[2]), 4)
    return {"workload": "the path's other kernels on 64 MiB f32 buckets (16 M elements), device-resident",
            "hbm_peak_gbs": HBM_PEAK_GBS,
            "timing": "one HIP event pair around K back-to-back launches over rotating sets", **out}


def sparse_codec(torch, ono_amd, rounds: int = 5) -> dict:
    """the device top-k codec (comms/src/sparse/protocol.rs:57-144) on a 64 MiB
    gradient with the threshold at the 90th |g| percentile (~10 % of the values kept, the
    reference's r = 0.9).  Drop = count (flags, compact values, chunk aggregates) + emit (each
    tile's runs and values to their place in the wire), as a blocking call (the wire length is needed
    on the host) and stream-ordered back to back; bytes = 4 N read + the wire
    written.  Lift parses the
    run headers on the host and expands on the device (host buffer in)."""
    import ctypes as C

    n = 16 << 20
    g = ono_amd.kernels.synth(torch.empty(n, dtype=torch.float32, device="cuda"), SEED, 7)
    t = float(torch.quantile(g[: 1 << 20].abs().float(), 0.9).item())
    L = ono_amd.lib()
    cap = L.ono_sparse_max_bytes(n)
    buf = torch.empty(cap + 8, dtype=torch.uint8, device="cuda")
    nb = C.c_size_t(0)
    stream = torch.cuda.current_stream()
    ts, tev = [], []
    for r in range(rounds + 1):  # device-resident: gradient in, wire buffer out, both in HBM
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        a.record(stream)
        ono_amd._lib.call("ono_sparse_drop", buf.data_ptr(), cap, C.byref(nb), g.data_ptr(), n, t,
                          stream.cuda_stream)
        b.record(stream)
        t1 = time.perf_counter()
        if r:
            ts.append(t1 - t0)
            b.synchronize()
            tev.append(a.elapsed_time(b) * 1e-3)
    td, tdev = sorted(ts)[len(ts) // 2], sorted(tev)[len(tev) // 2]
    wire = bytes(buf[: nb.value].cpu().numpy())
    # stream-ordered drops back to back (ono_sparse_drop_async: the wire length stays in HBM), one
    # event pair around K of them: the encoder's own time per drop, without the host round trip
    nbd = torch.zeros(1, dtype=torch.int64, device="cuda")
    K, NG = 24, 6  # 6 gradients in turn: 384 MiB > the 256 MiB Infinity Cache, so every drop reads HBM
    gs = [g] + [ono_amd.kernels.synth(torch.empty(n, dtype=torch.float32, device="cuda"), SEED + j, 7)
                for j in range(1, NG)]
    tg = [t] + [float(torch.quantile(x[: 1 << 20].abs().float(), 0.9).item()) for x in gs[1:]]
    for i in range(K):  # one untimed pass of the same loop first (clocks and caches as in the timed one)
        ono_amd.sparse.grad_drop_async(gs[i % NG], tg[i % NG], buf, nbd)
    ono_amd.sparse.grad_drop_async(g, t, buf, nbd)
    torch.cuda.synchronize()
    assert int(nbd.item()) == len(wire) and bytes(buf[: len(wire)].cpu().numpy()) == wire
    for i in range(8):  # the GPU busy while the timed drops are enqueued (no host gap at the opening event)
        ono_amd.sparse.grad_drop_async(gs[i % NG], tg[i % NG], buf, nbd)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for i in range(K):
        ono_amd.sparse.grad_drop_async(gs[i % NG], tg[i % NG], buf, nbd)
    b.record(stream)
    b.synchronize()
    tstream = a.elapsed_time(b) * 1e-3 / K
    del gs
    ono_amd.sparse.grad_drop_async(g, t, buf, nbd)  # buf holds g's stream again for the lifts below
    torch.cuda.synchronize()
    assert int(nbd.item()) == len(wire)
    tl = []
    for r in range(rounds + 1):
        t0 = time.perf_counter()
        back = ono_amd.sparse.grad_lift(wire, n)
        if r:
            tl.append(time.perf_counter() - t0)
    lt = sorted(tl)[len(tl) // 2]
    # device-resident lift: the stream drop left in HBM -> g (parallel parse + expand)
    out = torch.empty(n, dtype=torch.float32, device="cuda")
    ln = C.c_size_t(0)
    tdl, tdl_ev = [], []
    fb0, pm0 = L.ono_sparse_lift_fallbacks(), L.ono_sparse_lift_pattern_misses()
    for r in range(rounds + 1):
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        a.record(stream)
        ono_amd._lib.call("ono_sparse_lift_dev", out.data_ptr(), n, C.byref(ln), buf.data_ptr(), nb.value,
                          stream.cuda_stream)
        b.record(stream)
        t1 = time.perf_counter()
        if r:
            tdl.append(t1 - t0)
            b.synchronize()
            tdl_ev.append(a.elapsed_time(b) * 1e-3)
    fallbacks = L.ono_sparse_lift_fallbacks() - fb0
    pattern_misses = L.ono_sparse_lift_pattern_misses() - pm0
    # stream-ordered lifts back to back (ono_sparse_lift_dev_async), one event pair around K of them:
    # the lift's own device time, without the host wait of the blocking call
    # (6 streams and 6 outputs in turn, 0.5 GB > the Infinity Cache: every lift reads and writes HBM)
    st = torch.zeros(1, dtype=torch.int64, device="cuda")
    wires = [buf[: nb.value].clone()]
    for j in range(1, NG):
        gj = ono_amd.kernels.synth(torch.empty(n, dtype=torch.float32, device="cuda"), SEED + j, 7)
        tj = float(torch.quantile(gj[: 1 << 20].abs().float(), 0.9).item())
        wires.append(ono_amd.sparse.grad_drop_dev(gj, tj))
        del gj
    outs = [torch.empty(n, dtype=torch.float32, device="cuda") for _ in range(NG)]
    for i in range(NG):
        ono_amd.sparse.grad_lift_dev_async(wires[i], outs[i], st, stream)
    torch.cuda.synchronize()
    for i in range(NG):  # the GPU busy while the timed lifts are enqueued (no host gap at the opening event)
        ono_amd.sparse.grad_lift_dev_async(wires[i], outs[i], st, stream)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    tickets = [ono_amd.sparse.grad_lift_dev_async(wires[i % NG], outs[i % NG], st, stream) for i in range(K)]
    b.record(stream)
    b.synchronize()
    tlift_stream = a.elapsed_time(b) * 1e-3 / K
    async_refused = int(st.item()) in tickets
    async_same = bool(torch.equal(outs[0].view(torch.int32), back.view(torch.int32)))
    lift_stream_bytes = sum(w.numel() for w in wires) / NG + 4 * n
    del wires, outs
    same = bool(torch.equal(out.view(torch.int32), back.view(torch.int32)))
    dlt, dlt_ev = sorted(tdl)[len(tdl) // 2], sorted(tdl_ev)[len(tdl_ev) // 2]
    lift_bytes = len(wire) + 4 * n
    kept = int(torch.count_nonzero(back).item())
    drop_bytes = 4 * n + len(wire)  # g read once + the stream written
    return {"workload": "sparse grad_drop / grad_lift, 64 MiB f32 gradient, threshold = 90th |g| percentile",
            "kept_values": kept, "wire_bytes": len(wire),
            "drop": {"ms": round(td * 1e3, 3), "device_ms": round(tdev * 1e3, 3), "algorithmic_bytes": drop_bytes,
                     "achieved_gbs": round(drop_bytes / tdev / 1e9, 1),
                     "frac_of_hbm_peak": round(drop_bytes / tdev / 1e9 / HBM_PEAK_GBS, 4),
                     "stream_ms": round(tstream * 1e3, 4),
                     "stream_achieved_gbs": round(drop_bytes / tstream / 1e9, 1),
                     "stream_frac_of_hbm_peak": round(drop_bytes / tstream / 1e9 / HBM_PEAK_GBS, 4),
                     "note": "ms = wall time of the blocking C call; device_ms = HIP events around it on its "
                             "stream (sp_count + sp_emit, then the host read of the totals); "
                             "stream_ms = per drop of %d stream-ordered drops back to back "
                             "(ono_sparse_drop_async) over %d different 64 MiB gradients in turn "
                             "(each read from HBM), one event pair" % (K, NG)},
            "lift": {"ms": round(lt * 1e3, 3), "note": "host wire buffer in (Python bytes): H2D + device parse + "
                                                        "expand, wall time through the Python wrapper"},
            "lift_dev": {"ms": round(dlt * 1e3, 3), "device_ms": round(dlt_ev * 1e3, 3),
                         "algorithmic_bytes": lift_bytes,
                         "achieved_gbs": round(lift_bytes / dlt_ev / 1e9, 1),
                         "frac_of_hbm_peak": round(lift_bytes / dlt_ev / 1e9 / HBM_PEAK_GBS, 4),
                         "stream_ms": round(tlift_stream * 1e3, 4),
                         "stream_achieved_gbs": round(lift_stream_bytes / tlift_stream / 1e9, 1),
                         "stream_frac_of_hbm_peak": round(lift_stream_bytes / tlift_stream / 1e9 / HBM_PEAK_GBS, 4),
                         "stream_refused": async_refused, "stream_equals_host_lift": async_same,
                         "sequential_fallbacks": fallbacks, "pattern_path_misses": pattern_misses,
                         "equals_host_lift": same,
                         "note": "stream already in HBM (ono_sparse_lift_dev): the pattern path (record starts "
                                 "from the zero high halves of the headers, checked to be the sequential parse; "
                                 "each tile's range built in LDS and stored once); device_ms = HIP events around "
                                 "one blocking call (its host wait included); stream_ms = per lift of %d "
                                 "stream-ordered lifts back to back (ono_sparse_lift_dev_async) over %d different streams and outputs in turn "
                                 "(each read and written in HBM), one event pair; "
                                 "algorithmic bytes = wire + 4 B per element written" % (K, NG)}}


def host_fed(ono_amd, ring, elems: int, rounds: int) -> dict:
    """PCIe-inclusive pull_grads from host buffers (never
    `value`): the reference's buckets live in host memory and arrive from
    comms/.  Registered (page-locked once, DMA in place) and pageable (pinned
    bounce slots) forms; each round refills the host residual first (untimed)."""
    import numpy as np

    res = np.empty(elems, np.float32)
    grad = np.empty(elems, np.float32)
    src = np.random.default_rng(1).standard_normal(elems, dtype=np.float32) * np.float32(0.01)
    out = {}
    for form in ("pageable", "registered"):
        if form == "registered":
            ring.register_host(res)
            ring.register_host(grad)
        ts = []
        for r in range(rounds + 1):
            res[:] = src
            t0 = time.perf_counter()
            ring.pull_grads_host(res, grad)
            if r:
                ts.append(time.perf_counter() - t0)
        ts.sort()
        t, tmin, tmax = ts[len(ts) // 2], ts[0], ts[-1]
        out[form] = {"ms": round(t * 1e3, 3), "gib_s": round(elems * 4 / t / GIB, 2),
                     "ms_min": round(tmin * 1e3, 3), "gib_s_best": round(elems * 4 / tmin / GIB, 2),
                     "gib_s_worst": round(elems * 4 / tmax / GIB, 2), "rounds": len(ts)}
    ring.unregister_host(res)
    ring.unregister_host(grad)
    return {"workload": "pull_grads_host, 256 MiB host bucket in, 256 MiB host grad out, n = 1 device round trip",
            "pipeline": "16 MiB chunks: H2D || reduce || D2H on three HIP streams; pageable: bounce copies on "
                        "ONO_HOST_THREADS threads bound to the GPU's NUMA node",
            "stat": "ms / gib_s = median of the rounds, ms_min / gib_s_best = the fastest, gib_s_worst = the slowest",
            **out}


def host_fed_n(ono_amd, ring, elems: int, ctl, world: int, rounds: int = 5) -> dict:
    """N > 1: the end-to-end round a worker of the reference runs — host buckets
    in (registered once, as the manager's Vec<f32>s live as long as it does),
    H2D, the main schedule across the N GPUs, D2H, residual zeroed — timed
    between barriers, max over ranks.  GiB/s of one rank's bucket.  Never `value`."""
    import numpy as np

    try:
        res, grad = np.empty(elems, np.float32), np.empty(elems, np.float32)
        src = np.random.default_rng(ctl.rank).standard_normal(elems, dtype=np.float32) * np.float32(0.01)
        ring.register_host(res)
        ring.register_host(grad)
        ts = []
        for r in range(rounds + 1):
            res[:] = src
            ctl.barrier()
            t0 = time.perf_counter()
            ring.pull_grads_host(res, grad)
            t = ctl.max(time.perf_counter() - t0)
            if r:
                ts.append(t)
        ring.unregister_host(res)
        ring.unregister_host(grad)
        t = sorted(ts)[len(ts) // 2]
        if ring.wire == "f32" and ring.algo in ("auto", "allreduce"):
            how = "H2D || all-reduce || D2H in 16 MiB chunks"
        elif ring.algo == "xgmi":
            how = "upload kernel (reads the host bucket over PCIe) || xGMI round || D2H in sub-rounds (a slice of every chunk each)"
        else:
            how = f"whole bucket: H2D, {ring.algo} round, D2H"
        return {"workload": f"pull_grads_host on {world} GPUs: registered host buckets of {elems * 4 >> 20} MiB per "
                            f"rank, {how} ({ring.wire} wire)",
                "ms": round(t * 1e3, 3), "gib_s": round(elems * 4 / t / GIB, 2)}
    except Exception as e:  # noqa: BLE001 — informational
        return {"error": f"{type(e).__name__}: {e}"[:300]}
    finally:
        ring.close()


def ps_host_fed(ono_amd, elems: int, rounds: int = 3, workers: int = 2) -> dict:
    """The parameter server's own hot path (SURVEY §8(a) BlockingStore rows):
    gradients arrive in host memory from comms/, the device store accumulates
    them, the leader updates (÷n + GD), params go back to host.  Same round
    as cpu_baseline.ps_accumulate_update (workers accumulates + 1 update;
    GiB/s = workers x 4N / t), plus the pull.  Never `value`."""
    import numpy as np

    params = np.zeros(elems, np.float32)
    grads = [np.random.default_rng(w).standard_normal(elems, dtype=np.float32) * np.float32(0.01)
             for w in range(workers)]
    halfs = [g.astype(np.float16).view(np.uint16) for g in grads]  # the workers' f16 wire payloads
    out = np.empty(elems, np.float32)
    store = ono_amd.BlockingStore(max(1, elems // 32), workers, params, ono_amd.GradientDescent(0.1))
    res = {}
    for form in ("f32", "f16_wire"):
        ts, tp = [], []
        for r in range(rounds + 1):
            t0 = time.perf_counter()
            for w in range(workers):
                if form == "f32":
                    store.accumulate(grads[w])
                else:
                    store.accumulate_f16(halfs[w])
            store.update_params()
            t1 = time.perf_counter()
            store.pull_params(out)
            t2 = time.perf_counter()
            if r:
                ts.append(t1 - t0)
                tp.append(t2 - t1)
        t, p = sorted(ts)[len(ts) // 2], sorted(tp)[len(tp) // 2]
        res[form] = {"accumulate_update_ms": round(t * 1e3, 3), "gib_s": round(workers * elems * 4 / t / GIB, 3),
                     "pull_ms": round(p * 1e3, 3), "pull_gib_s": round(elems * 4 / p / GIB, 3)}
    store.close()
    return {"workload": f"BlockingStore on the device fed from host (pageable) buffers: {workers} accumulates + "
                        f"1 update (/n, GD) of {elems} params, then pull_params to host; f32 = decoded gradients, "
                        "f16_wire = the workers' f16 payloads decoded inside the accumulate kernel "
                        "(GiB/s counts f32 gradient bytes in both)", **res}


def tcp_edge_native(elems: int, rounds: int, ranks: int = 2) -> dict | None:
    """The TCP edge driven from a plain C++ host (tools/ono_tcp_bench: worker
    threads on this GPU, ono_ring_create_tcp over loopback TCP, pthread
    barriers) — the way a native Rust worker drives it, without the Python
    threading overhead of tcp_edge().  None if the tool is not built."""
    exe = os.path.join(ROOT, "tools", "ono_tcp_bench")
    if not os.path.exists(exe):
        return None
    import subprocess
    try:
        out = subprocess.run([exe, "--ranks", str(ranks), "--len", str(elems), "--rounds", str(rounds),
                              "--phases", "0"], capture_output=True, text=True, timeout=300, check=True)
        d = json.loads(out.stdout.strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001 — reported in the line
        return {"error": f"{type(e).__name__}: {e}"[:200]}
    return {"workload": f"pull_grads over loopback TCP, {ranks} workers (C++ host threads) on one GPU, "
                        f"{elems} f32 each, f16 reference frames",
            "ranks": ranks, "ms": round(d["s_per_round"] * 1e3, 4), "gib_s": round(d["gib_s"], 3)}


def tcp_sparse_native(elems: int, rounds: int, ranks: int, ratio: float, dump: str | None = None) -> dict | None:
    """The TCP edge with every worker's SparseCapable{ratio} serializer (tools/ono_tcp_bench --sparse): the
    per-round time and rank 0's phase split (socket exchange, the sparse codec's calls, the other kernels).
    dump: rank 0's grad + residual of the last round, for the checker (cpu_baseline.sparse_ring)."""
    exe = os.path.join(ROOT, "tools", "ono_tcp_bench")
    if not os.path.exists(exe):
        return None
    import subprocess
    import numpy as np
    cmd = [exe, "--ranks", str(ranks), "--len", str(elems), "--rounds", str(rounds), "--sparse",
           repr(float(np.float32(ratio)))] + (["--dump", dump] if dump else [])
    try:
        # ms from an untimed run: rank 0's per-launch event pairs of the phase split cost host time inside
        # every round (config 1: ~0.04 ms of a ~0.2 ms round), so the split comes from a second, timed run
        out = subprocess.run(cmd + ["--phases", "0"], capture_output=True, text=True, timeout=300, check=True)
        d = json.loads(out.stdout.strip().splitlines()[-1])
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, check=True)
        t = json.loads(out.stdout.strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001 — reported in the line
        return {"error": f"{type(e).__name__}: {e}"[:200]}
    return {"ranks": ranks, "elems": elems, "ratio": ratio, "ms": round(d["s_per_round"] * 1e3, 4),
            "gib_s": round(d["gib_s"], 3), "timed_run_ms": round(t["s_per_round"] * 1e3, 4),
            "phase_ms_per_round": t["phase_ms_per_round"], "codec_share_of_round": t["codec_share_of_round"]}


def tcp_sparse_legs() -> dict:
    """SURVEY §8(f) row 3 on the product path: the sparse ring end to end."""
    out = {"workload": "pull_grads over loopback TCP with SparseCapable{r} workers (SparseGrad frames, "
                       "reference framing), C++ host threads on one GPU; ms per round of an untimed run, rank 0's phase split from a second, "
                       "timed run (timed_run_ms: its round, the event pairs' host cost included)"}
    for key, e, n, r, k in (("config1_2_ranks_r0.1", CONFIG1_ELEMS, 2, 0.1, 200),
                            ("config1_2_ranks_r0.01", CONFIG1_ELEMS, 2, 0.01, 200),
                            ("config1_4_ranks_r0.1", CONFIG1_ELEMS, 4, 0.1, 200),
                            ("256MiB_2_ranks_r0.1", 1 << 26, 2, 0.1, 10),
                            ("256MiB_2_ranks_r0.01", 1 << 26, 2, 0.01, 10)):
        out[key] = tcp_sparse_native(e, k, n, r)
    return out


def tcp_edge(ono_amd, elems: int, rounds: int, ranks: int = 2) -> dict:
    """The TCP edge (never `value`): `ranks` MI355X workers on
    this one GPU, one thread each, in a loopback-TCP ring speaking the
    reference's frames — the same transport, rank count and bucket as the
    reference CPU ring of `cpu_baseline`, so the two rates compare directly.
    Per round each worker refills its residual in HBM (untimed), then all run
    pull_grads between two barriers.  Reports the per-worker bucket rate."""
    import socket
    import threading

    import torch

    lis = [socket.create_server(("127.0.0.1", 0)) for _ in range(ranks)]
    ports = [s.getsockname()[1] for s in lis]
    bar = threading.Barrier(ranks)
    times, errs = [], []

    def worker(r):
        nxt = prev = ring = None
        try:
            torch.cuda.set_device(torch.cuda.current_device())
            nxt = socket.create_connection(("127.0.0.1", ports[(r + 1) % ranks]), timeout=60)
            nxt.settimeout(None)
            nxt.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            prev, _ = lis[r].accept()
            s = torch.cuda.Stream()
            ring = ono_amd.WorkerRingManager.over_tcp(r, ranks, elems, prev, nxt)
            with torch.cuda.stream(s):
                src = torch.randn(elems, device="cuda") * 0.01
            for k in range(rounds + 1):
                with torch.cuda.stream(s):
                    ring.residual.copy_(src)
                s.synchronize()
                bar.wait()
                t0 = time.perf_counter()
                ring.pull_grads(stream=s)
                s.synchronize()
                bar.wait()
                if r == 0 and k:
                    times.append(time.perf_counter() - t0)
        except Exception as e:  # noqa: BLE001 — reported in the line
            errs.append(repr(e))
            bar.abort()
        finally:
            if ring is not None:
                ring.close()
            for sk in (nxt, prev):
                if sk is not None:
                    sk.close()

    th = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(ranks)]
    for t in th:
        t.start()
    for t in th:
        t.join(600)
    for s in lis:
        s.close()
    if errs or not times:
        return {"error": errs[0] if errs else "timed out"}
    t = sorted(times)[len(times) // 2]
    return {"workload": f"pull_grads over loopback TCP, {ranks} workers on one GPU, "
                        f"{elems * 4 >> 20} MiB bucket each, f16 reference frames",
            "ranks": ranks, "ms": round(t * 1e3, 3), "gib_s": round(elems * 4 / t / GIB, 3)}



# ------------------------------------------------------------- the step loop
class Runner:
    """W + K pull_grads rounds of a ring, each over its own freshly generated
    bucket already resident in HBM (W + K buckets of the bench size), output
    into one grad bucket."""

    def __init__(self, torch, ono_amd, args, ctl: Ctl, world: int, rank: int, elems: int):
        self.torch, self.ono_amd, self.args, self.ctl = torch, ono_amd, args, ctl
        self.world, self.rank, self.elems = world, rank, elems
        self.nb = args.warmup + args.steps
        self.residuals = [torch.empty(elems, dtype=torch.float32, device="cuda") for _ in range(self.nb)]
        self.grad = torch.empty(elems, dtype=torch.float32, device="cuda")
        self.stream = torch.cuda.current_stream()

    def refill(self) -> None:  # a fresh, distinct bucket for every step (untimed)
        for i, t in enumerate(self.residuals):
            self.ono_amd.kernels.synth(t, SEED + i, self.rank)
        self.torch.cuda.synchronize()

    def measure(self, r) -> tuple[float, dict]:
        """W + K pull_grads rounds with ring r; (max-over-ranks seconds, timing).
        N = 1: a step is exactly one kernel, so one HIP event pair around the
        timed region gives its average launch duration without per-launch
        events (which add ~6 % to a 130 us stream, tools/stream_variants.hip
        "pull" mode).  N > 1: the timed run has no per-launch events; a second
        run of the same K steps records them to split collectives and kernels
        for the roofline."""
        torch, args, nb = self.torch, self.args, self.nb
        self.refill()
        span = [torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)]

        def on_start():
            span[0].record(self.stream)

        def step(i: int) -> None:
            r.pull_grads_dev(self.residuals[i], self.grad, self.stream)
            if i == nb - 1:
                span[1].record(self.stream)

        el, _ = timed_region(step, args.steps, args.warmup, torch.cuda.synchronize, self.ctl, on_start=on_start)
        r.check()  # an xGMI barrier timeout would make the timed rounds invalid
        span_ms = span[0].elapsed_time(span[1])
        if self.world == 1:
            return el, {"kernel_ms": span_ms, "kernels": args.steps, "collective_ms": 0.0, "collectives": 0}
        self.refill()
        timed_region(step, args.steps, args.warmup, torch.cuda.synchronize, self.ctl,
                     on_start=lambda: r.timing(True))
        tim = r.timing_read()
        tim["phases"] = r.timing_phases()
        r.timing(False)
        return el, tim

    def verify(self, wire: str) -> dict:
        """Check the last measured step against the exact average: every rank
        regenerates all N inputs of that step (counter-based generator) and
        bounds |grad - sum/N| by the summation-order term 2(N-1) 2^-24 sum|g| / N
        (f16 wire: + N 2^-11 sum|g| / N + N 2^-25 for the N f16 roundings);
        the residual must be all zero.  ratio = max err / bound over all ranks
        (<= 1 passes; 0 where the bound is 0 means bit-exact)."""
        torch, n, i = self.torch, self.world, self.nb - 1
        tmp = torch.empty(self.elems, dtype=torch.float32, device="cuda")
        acc = torch.zeros(self.elems, dtype=torch.float64, device="cuda")
        mag = torch.zeros(self.elems, dtype=torch.float64, device="cuda")
        for r in range(n):
            self.ono_amd.kernels.synth(tmp, SEED + i, r)
            acc += tmp.double()
            mag += tmp.abs().double()
        bound = mag * (2 * (n - 1) * 2.0 ** -24 / n)
        if wire == "f16":
            bound += mag * 2.0 ** -11 + n * 2.0 ** -25
        err = (self.grad.double() - acc / n).abs()
        over = err > bound
        ratio = float((err / bound.clamp_min(1e-300)).max().item()) if bool(bound.gt(0).any()) else 0.0
        bad = int(over.sum().item())
        left = int(self.residuals[i].count_nonzero().item())
        del tmp, acc, mag, bound, err, over
        self.torch.cuda.empty_cache()
        ratio, bad, left = self.ctl.max(ratio), int(self.ctl.max(bad)), int(self.ctl.max(left))
        return {"ok": bad == 0 and left == 0, "max_err_over_bound": round(ratio, 4), "elems_over_bound": bad,
                "residual_nonzero": left}

# ------------------------------------------------------------ time budget
# a leg still running this long after the deadline is cut (the line printed as it stands); env for CPU tests
GRACE_S = float(os.environ.get("ONO_BENCH_GRACE_S", "45"))


class Budget:
    """The line's deadline, shared by every rank (ONO_BENCH_DEADLINE: absolute
    time set by whoever started rank 0's job).  Rank 0 decides whether a leg
    still fits and broadcasts the decision, so collective legs are entered or
    skipped by every rank together."""

    def __init__(self, ctl: Ctl, deadline: float):
        self.ctl, self.deadline = ctl, deadline

    def left(self) -> float:
        return self.deadline - time.time()

    def allow(self, est_s: float) -> bool:
        ok = b"1" if self.left() >= est_s else b"0"
        return self.ctl.bcast_bytes(ok) == b"1" if self.ctl.world > 1 else ok == b"1"


class LineBox:
    """The JSON line under a lock: legs store results into it, and the backstop
    watchdog prints it as it stands if a leg overruns the deadline."""

    def __init__(self):
        self.lock = threading.Lock()
        self.line: dict = {}
        self.running: str | None = None
        self.children: list = []  # subprocess.Popen of the xGMI legs, killed by the watchdog

    def put(self, path: tuple, value) -> None:
        with self.lock:
            d = self.line
            for k in path[:-1]:
                d = d.setdefault(k, {})
            d[path[-1]] = value

    def dump(self) -> str:
        with self.lock:
            return json.dumps(self.line)


BOX = LineBox()


def start_backstop(budget: Budget, rank: int) -> threading.Timer:
    """At deadline + GRACE_S: kill the legs' child processes, mark the leg that
    was running as cut, print the line (rank 0) and exit — the headline and every
    finished leg are in it."""
    def fire():
        for p in list(BOX.children):
            try:
                p.kill()
            except Exception:  # noqa: BLE001
                pass
        with BOX.lock:
            if BOX.running:
                d = BOX.line.setdefault("deadline", {})
                d["cut"] = BOX.running
        if rank == 0:
            print(BOX.dump(), flush=True)
        # exit 0 on purpose: the backstop only fires after the headline is in the line, and
        # the driver reads the line by the exit status; the cut leg is named in the line's deadline.cut
        os._exit(0)

    t = threading.Timer(max(0.0, budget.left() + GRACE_S), fire)
    t.daemon = True
    t.start()
    return t


def _run_ranks(args, argv: list, deadline: str, env_extra: dict) -> tuple[int, dict | None]:
    """Start the N ranks (one process per GPU, the env torch.distributed.run
    would give them) and return rank 0's exit code and JSON line (None: none).
    When rank 0 ends without a headline the others are killed at once (they may
    be waiting in a collective for it)."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    base = {k: v for k, v in os.environ.items() if not k.startswith("TORCHELASTIC_")}
    procs = []
    for r in range(args.gpus):
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus), LOCAL_WORLD_SIZE=str(args.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ONO_BENCH_DEADLINE=deadline, ONO_BENCH_RANK="1",
                   **env_extra)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL, text=True))
    out = ""
    try:  # rank 0 prints its line by deadline + GRACE_S at the latest (backstop); a little more for exit
        out, _ = procs[0].communicate(timeout=max(30.0, float(deadline) - time.time() + GRACE_S + 30.0))
    except subprocess.TimeoutExpired:
        procs[0].kill()
        out, _ = procs[0].communicate()
    lines = [ln for ln in (out or "").splitlines() if ln.startswith("{")]
    line = None
    if lines:
        try:
            line = json.loads(lines[-1])
        except ValueError:
            line = None
    failed = line is None or "headline_error" in line
    for p in procs[1:]:
        try:
            p.wait(timeout=1 if failed else 30)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    return procs[0].returncode, line


def launch_ranks(args, argv) -> int:
    """--gpus N > 1: start the N ranks from this process, which never touches
    the GPU, and relay rank 0's JSON line.  The ranks share this process's
    deadline.  If the headline schedule could not run — rank 0 reports a
    headline_error (the RCCL ring's creation failed, or the headline did not
    finish within ONO_BENCH_HEADLINE_TIMEOUT_S), or printed nothing — a fresh
    set of ranks measures the headline on the xGMI schedule, which needs no
    RCCL (the node-local form of the reference's ring, worker/src/builder.rs:
    272-311), and the line records headline_fallback {from, reason}.  No rank
    that has touched the GPU is ever asked to retry."""
    argv = list(sys.argv[1:] if argv is None else argv)
    deadline = os.environ.get("ONO_BENCH_DEADLINE") or repr(time.time() + args.deadline)
    rc, line = _run_ranks(args, argv, deadline, {})
    if (line is None or "headline_error" in line) and args.algo != "xgmi":
        frm = {"auto": "allreduce" if args.wire == "f32" else "direct"}.get(args.algo, args.algo)
        reason = line["headline_error"] if line else f"rank 0 printed no line (exit {rc})"
        fb = {"from": frm, "reason": str(reason)[:400]}
        print(f"bench.py: headline on {frm} failed ({fb['reason']}); measuring it on the xGMI schedule",
              file=sys.stderr, flush=True)
        # the RCCL schedules stay out of the fallback's legs too (alt schedules; the xGMI children would repeat it)
        argv2 = argv + ["--algo", "xgmi", "--alt-schedules", "", "--no-xgmi"]
        rc, line = _run_ranks(args, argv2, deadline, {"ONO_BENCH_FALLBACK": json.dumps(fb)})
    if line is None:
        print(f"bench.py: rank 0 printed no line (exit {rc})", file=sys.stderr)
        return rc or 1
    print(json.dumps(line), flush=True)
    return 0 if "headline_error" not in line else (rc or 1)


def headline_abort(rank: int, reason: str) -> None:
    """The headline could not be measured in this rank (its ring failed, or it did
    not finish in time): rank 0 says why in a one-key JSON line for the launcher
    (launch_ranks, which falls back to the xGMI schedule), and the process ends
    without retrying anything."""
    if rank == 0:
        print(json.dumps({"headline_error": reason[:400]}), flush=True)
    sys.stdout.flush()
    os._exit(5)


class DryRing:
    """--dry-run: a ring that only sleeps (CPU plumbing tests)."""
    def __init__(self, algo: str = "dry"):
        self.algo = algo

    def set_pipeline(self, _):
        pass

    def close(self):
        pass


# ------------------------------------------------------------------- main
def main(argv=None) -> int:
    args = parse_args(argv)
    if args.xgmi_child:
        return xgmi_child_main(args)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args, argv)
    if args.gpus > 1 and os.environ.get("TORCHELASTIC_RUN_ID") and not os.environ.get("ONO_BENCH_RANK"):
        # under torch.distributed.run: its local rank 0 becomes the GPU-free launcher of the N ranks (so that a
        # failed headline can be measured again by fresh processes), the others leave at once, before any GPU call
        if os.environ.get("LOCAL_RANK", "0") != "0":
            return 0
        return launch_ranks(args, argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = 0 if args.same_device else int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    deadline = float(os.environ.get("ONO_BENCH_DEADLINE") or time.time() + args.deadline)

    dry = args.dry_run
    if dry:
        torch = ono_amd = None
    else:
        import torch
        import ono_amd
        torch.cuda.set_device(local_rank)
    ctl = Ctl(world, rank)
    budget = Budget(ctl, deadline)
    elems = args.bucket_mib * (1 << 20) // 4
    bucket_bytes = elems * 4

    def new_ring(wire: str, algo: str, size: int = elems):
        if dry:  # (stubs: an RCCL ring that fails to come up, or never does)
            if algo != "xgmi" and os.environ.get("ONO_BENCH_DRY_RING_FAIL"):
                raise RuntimeError("RcclError: ncclCommInitRank failed (dry-run stub)")
            if algo != "xgmi" and os.environ.get("ONO_BENCH_DRY_RING_HANG"):
                time.sleep(1e6)
            return DryRing("xgmi" if algo == "xgmi" else "dry")
        if algo == "xgmi" and world > 1:  # no communicator: IPC handles over the control plane
            return ono_amd.WorkerRingManager.over_xgmi(rank, world, size, ctl.allgather_bytes, wire=wire,
                                                       device=local_rank)
        uid = ono_amd.unique_id() if (world > 1 and rank == 0) else None
        uid = ctl.bcast_bytes(uid) if world > 1 else None
        return ono_amd.WorkerRingManager(rank, world, size, uid=uid, wire=wire, device=local_rank, algo=algo)

    # ---- the headline first: measured, checked and in the line before any informational leg.  If its ring cannot
    # be created (RCCL), or the headline does not finish in time, rank 0 reports it and the process ends: the
    # launcher measures the headline again on the xGMI schedule in fresh processes (launch_ranks).
    hl_timeout = float(os.environ.get("ONO_BENCH_HEADLINE_TIMEOUT_S", "180"))
    watchdog = None
    if world > 1:
        watchdog = threading.Timer(hl_timeout, headline_abort,
                                   (rank, f"the {args.algo} headline (ring creation, {args.steps} steps and the check) "
                                          f"did not finish in {hl_timeout:.0f} s"))
        watchdog.daemon = True
        watchdog.start()
    try:
        ring = new_ring(args.wire, args.algo)
        ring.set_pipeline(args.segments)
    except Exception as e:  # noqa: BLE001
        if world == 1:
            raise
        headline_abort(rank, f"{args.algo} ring creation failed: {type(e).__name__}: {e}")
    if dry:
        run = None

        def measure(_r):
            el, _ = timed_region(lambda i: time.sleep(0.001), args.steps, args.warmup, lambda: None, ctl)
            return el, {"kernel_ms": el * 1e3, "kernels": args.steps, "collective_ms": 0.0, "collectives": 0}
        stream = None
    else:
        run = Runner(torch, ono_amd, args, ctl, world, rank, elems)
        measure, stream = run.measure, run.stream

    link = xgmi_link_probe(torch) if (world > 1 and rank == 0 and not dry) else None
    ctl.barrier()
    elapsed, tim = measure(ring)

    extra = {"check": {"ok": True, "dry_run": True} if dry else run.verify(args.wire)}
    if watchdog is not None:
        watchdog.cancel()
    if world == 1:
        avg_ms = tim["kernel_ms"] / max(tim["kernels"], 1)
        per_launch = 12 * elems  # read residual, write grad, write zeros (12 N)
        ach = per_launch / (avg_ms * 1e-3) / 1e9
        pmc = pmc_traffic("ScaleZeroOp", elems)
        extra["roofline"] = {
            "bound": "hbm", "kernel": "ew_kernel<ScaleZeroOp<SCALE_NONE>> (grad = residual; residual = 0)",
            "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
            "traffic": pmc["hbm_bytes_per_launch"] if pmc else None,
            "algorithmic_bytes_per_launch": per_launch, "avg_launch_us": round(avg_ms * 1e3, 2),
            "launches": tim["kernels"],
            "timing": "one HIP event pair on the launch stream around the K timed steps (one kernel per step)",
        }
        if pmc:
            extra["roofline"]["traffic_source"] = pmc["source"]
            extra["roofline"]["traffic_provenance"] = (
                f"committed profile {pmc['source']}@{pmc.get('commit', 'unknown')} "
                f"({pmc.get('session', 'a builder session')}); not measured in this run")
    else:
        extra["roofline"] = nx_roofline(tim, bucket_bytes, elems, world, args.wire, ring.algo, args.steps, elapsed,
                                        link)

    value = world * bucket_bytes * args.steps / elapsed / GIB
    BOX.line = build_line(value=value, n_gpus=world, steps=args.steps, warmup=args.warmup, elapsed=elapsed,
                          bucket_bytes=bucket_bytes, wire=args.wire, extra=extra)
    line = BOX.line
    line["config"]["schedule"] = ring.algo
    if os.environ.get("ONO_BENCH_FALLBACK"):  # this headline replaces one that failed (launch_ranks)
        line["headline_fallback"] = json.loads(os.environ["ONO_BENCH_FALLBACK"])
    if world > 1 and ring.algo == "xgmi":
        line["config"]["collective"] = "xGMI peer-access kernels over IPC-mapped peer HBM (no RCCL)"
    if world > 1 and args.wire == "f32" and ring.algo in ("auto", "allreduce"):
        line["config"]["allreduce_segments"] = args.segments or "library default (ONO_AR_SEGMENTS or 4)"
    line["deadline"] = {"s": args.deadline, "skipped": []}
    backstop = start_backstop(budget, rank)

    def leg(path, est_s: float, fn, collective: bool = False):
        """An informational leg: skipped (and recorded) when it would end past the deadline, its failure
        recorded in the line, never fatal to it.  Collective legs are decided by rank 0 for every rank."""
        path = path if isinstance(path, tuple) else (path,)
        name = ":".join(path)
        ok = budget.allow(est_s) if collective else budget.left() >= est_s
        if not ok:
            BOX.put(("deadline", "skipped"), line["deadline"]["skipped"] + [name])
            return None
        BOX.running = name
        try:
            if dry:
                time.sleep(args.dry_leg_s)
                res = {"dry_run": True}
            else:
                res = fn()
        except Exception as e:  # noqa: BLE001
            res = {"error": f"{type(e).__name__}: {e}"[:300]}
        BOX.running = None
        if res is not None:
            BOX.put(path, res)
        return res

    def tcp_legs():
        out = tcp_edge_native(elems, 10) or tcp_edge(ono_amd, elems, 3)
        # BASELINE config 1: the reference's own case — 2 loopback workers, the
        # MLP 784-128-64-10 bucket (109,386 f32) — TCP edge vs CPU ring
        small = {"2_ranks": tcp_edge_native(CONFIG1_ELEMS, 200) or tcp_edge(ono_amd, CONFIG1_ELEMS, 50),
                 "4_ranks": tcp_edge_native(CONFIG1_ELEMS, 200, 4) or tcp_edge(ono_amd, CONFIG1_ELEMS, 50, 4)}
        if not args.no_cpu_baseline:
            from oracle import oracle as O  # noqa: WPS433 (cpu_baseline leg only)
            for k, nr in (("2_ranks", 2), ("4_ranks", 4)):
                cr = O.cpu_ring(nr, CONFIG1_ELEMS, 50, check=False, pin=True, timeout=300)
                small[k]["cpu_ring_ms"] = round(cr["s_per_round"] * 1e3, 4)
        out["config1"] = small
        out["sparse"] = tcp_sparse_legs()
        return out

    if rank == 0 and world == 1:  # estimates: the legs' usual run time on an MI355X box, with margin
        if not args.no_host_fed:
            leg("host_fed", 15, lambda: host_fed(ono_amd, ring, elems, 5))
        if not args.no_tcp_edge:
            leg("tcp_edge", 40, tcp_legs)
        if not args.no_host_fed:
            leg("ps_host_fed", 15, lambda: ps_host_fed(ono_amd, elems))
        if not args.no_local_reduce:
            leg("local_reduce", 15, lambda: local_reduce(torch, ono_amd, max(args.steps, 10), max(args.warmup, 2)))
            leg("path_kernels", 25, lambda: path_kernels(torch, ono_amd, max(args.steps, 10), max(args.warmup, 2)))
            leg("sparse_codec", 25, lambda: sparse_codec(torch, ono_amd))
            leg("copy_ceiling", 15, lambda: copy_ceiling(torch, ono_amd, max(args.steps, 10), max(args.warmup, 2)))
        if not args.no_cpu_baseline:
            leg("cpu_baseline", 80, lambda: cpu_baseline(elems, args.cpu_ranks, args.cpu_rounds))
        with BOX.lock:
            n1_roofline_summary(line["roofline"], line.get("local_reduce"), line.get("copy_ceiling"))

    # Informational: the other exchange schedules at N > 1 (never `value`), each entered by every rank
    # together or skipped by every rank together (rank 0 reads the clock).
    extras = world > 1 or args.alt_at_n1
    alts = [a.split(":") for a in args.alt_schedules.split(",") if a] if extras else []
    if extras:
        BOX.put(("alt_schedules",), {})
        if world > 1 and args.xgmi:  # in child processes: a fault there cannot take the main line down
            def xgmi_leg():
                args.xgmi_timeout = max(30.0, min(args.xgmi_timeout, budget.left() - 60.0))
                for k, v in xgmi_spawn(args, ctl, world, rank, local_rank).items():
                    BOX.put(("alt_schedules", k), v)
            leg(("alt_schedules", "xgmi_children"), 90, xgmi_leg, collective=True)
        rings = {args.wire: ring}
        for alt in alts:
            algo, wire, seg = alt[0], alt[1], int(alt[2]) if len(alt) > 2 else args.segments

            def alt_leg(algo=algo, wire=wire, seg=seg):
                if wire not in rings:
                    rings[wire] = new_ring(wire, "auto")
                r = rings[wire]
                r.set_algo(algo)
                r.set_pipeline(seg)
                el, t = measure(r)
                r.set_pipeline(args.segments)
                return {"value": round(world * bucket_bytes * args.steps / el / GIB, 3),
                        "ms_per_step": round(el / args.steps * 1e3, 4),
                        "roofline": xgmi_roofline(t, bucket_bytes, elems, world, wire, algo, args.steps),
                        "check": run.verify(wire)}
            leg(("alt_schedules", ":".join(alt)), 20, alt_leg, collective=True)
        if world > 1 and not args.no_host_fed:  # the PCIe-inclusive round at N > 1 (north star)
            leg("host_fed", 30, lambda: host_fed_n(ono_amd, new_ring(args.wire, args.algo), elems, ctl, world),
                collective=True)
        if args.sweep_mib:  # BASELINE config 4: the bandwidth-vs-bucket-size curve, main schedule
            def sweep_ring(e):
                r = new_ring(args.wire, args.algo, e)
                r.set_pipeline(args.segments)
                return r
            leg("size_sweep", 45, lambda: size_sweep(torch, ono_amd, ctl, sweep_ring, sweep_sizes(args.sweep_mib),
                                                     world, rank, stream), collective=True)
        if args.ps_mode:  # BASELINE config 5: sharded synchronizer, RS + fused GD + AG
            def ps_leg():
                import numpy as np
                init = np.zeros(elems, np.float32)
                ps = ono_amd.ShardedParamServer(ring, init, ono_amd.GradientDescent(0.1))
                params = torch.empty(elems, dtype=torch.float32, device="cuda")
                run.refill()
                ring.timing(False)
                el, _ = timed_region(lambda i: ps.step(run.residuals[i], params, stream), args.steps, args.warmup,
                                     torch.cuda.synchronize, ctl)
                ps.close()
                del params
                return {"value": round(world * bucket_bytes * args.steps / el / GIB, 3),
                        "ms_per_step": round(el / args.steps * 1e3, 4),
                        "workload": "ShardedParamServer.step: reduce-scatter(sum) -> fused /n + GD on the owned "
                                    "shard -> all-gather(params), 256 MiB gradient per GPU"}
            leg(("alt_schedules", "ps:gd"), 20, ps_leg, collective=True)
        for w, r in rings.items():
            if r is not ring:
                r.close()

    if world == 1 and args.xgmi_coresident > 1:
        leg("xgmi_coresident", 60, lambda: xgmi_spawn(args, ctl, world, rank, local_rank,
                                                      coresident=args.xgmi_coresident))

    backstop.cancel()
    ring.close()
    ctl.close()
    if rank == 0:
        print(BOX.dump(), flush=True)
    return 0


# ------------------------------------------------ xGMI schedule (children)
def xgmi_spawn(args, ctl: Ctl, world: int, rank: int, local_rank: int, coresident: int = 0) -> dict:
    """Measure the xGMI peer-access schedule (ONO_ALGO_XGMI) in child
    processes: each rank starts one child on its GPU (coresident = R: rank 0
    starts R children on its one GPU — a rehearsal with HBM standing in for
    the links).  The children form their own ring (ono_ring_create_xgmi, IPC
    handles over their own gloo group) and time both wires; a child that hangs
    or faults is killed at --xgmi-timeout and recorded, the parent's line
    survives.  Returns {"xgmi:f32": {...}, "xgmi:f16": {...}} from child rank 0."""
    import shutil
    import subprocess
    import tempfile

    n = coresident or world
    rdv_dir = None
    if rank == 0:  # the children's gloo rendezvous: a fresh file on this node (a free port could be taken)
        rdv_dir = tempfile.mkdtemp(prefix="ono_bench_rdv_").encode()
    rdv_dir = ctl.bcast_bytes(rdv_dir).decode()
    import torch
    if torch.cuda.is_available():
        torch.cuda.synchronize()  # nothing of the parent's in flight while the children run
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--xgmi-child", "--gpus", str(n), "--steps",
           str(args.steps), "--warmup", str(args.warmup), "--bucket-mib", str(args.bucket_mib),
           "--sweep-mib", getattr(args, "sweep_mib", "")]
    procs = []
    # The children rendezvous through their own file store: drop torchrun's
    # agent-store settings (TORCHELASTIC_USE_AGENT_STORE=True would make every
    # child a client of a store nobody serves).
    base_env = {k: v for k, v in os.environ.items() if not k.startswith("TORCHELASTIC_")}
    for r in (range(n) if coresident else [rank]):
        env = dict(base_env, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(local_rank), LOCAL_WORLD_SIZE=str(n),
                   ONO_BENCH_RDV="file://" + os.path.join(rdv_dir, "store"))
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    BOX.children.extend(procs)
    deadline = time.time() + args.xgmi_timeout
    outs = []
    for p in procs:
        try:
            out, err = p.communicate(timeout=max(1.0, deadline - time.time()))
        except subprocess.TimeoutExpired:
            p.kill()
            out, err = p.communicate()
            err = f"killed after {args.xgmi_timeout:.0f} s; " + (err or "")
        outs.append((p.returncode, out, err))
    ctl.barrier()
    if rank == 0:
        shutil.rmtree(rdv_dir, ignore_errors=True)
    if rank != 0:
        return {}
    rc, out, err = outs[0]
    try:
        res = json.loads(out.strip().splitlines()[-1])
        if coresident:  # no links here: keep the timings, drop the link roofline
            for v in res.values():
                rl = v.get("roofline") if isinstance(v, dict) else None
                if rl:
                    v["roofline"] = {k: rl[k] for k in ("schedule", "phases_ms_per_step", "kernel_avg_us")
                                     if k in rl}
            res["note"] = (f"co-resident rehearsal: {n} ranks as processes on ONE GPU, peer regions are IPC "
                           "imports of the same HBM (no xGMI links involved; timings only)")
        return res
    except (ValueError, IndexError):
        return {"xgmi": {"error": f"child rank 0 exited {rc}: {(err or '').strip()[-300:]}"}}


def xgmi_child_main(args) -> int:
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    ctl = Ctl(world, rank)  # rendezvous first: a GPU failure below is then reported, not a hang
    try:
        import ono_amd
        torch.cuda.set_device(local_rank)
        elems = args.bucket_mib * (1 << 20) // 4
        run = Runner(torch, ono_amd, args, ctl, world, rank, elems)
    except Exception as e:
        ctl.close()
        if rank == 0:
            print(json.dumps({"xgmi": {"error": f"{type(e).__name__}: {e}"[:300]}}), flush=True)
        return 0
    out = {}
    for gather, wire in (("pull", "f32"), ("pull", "f16"), ("push", "f32"), ("push", "f16")):
        key = f"xgmi:{wire}" if gather == "pull" else f"xgmi-pushgather:{wire}"
        os.environ["ONO_XGMI_GATHER"] = gather  # read when the ring's exchange region is made
        try:
            ring = ono_amd.WorkerRingManager.over_xgmi(rank, world, elems, ctl.allgather_bytes, wire=wire,
                                                       device=local_rank)
            el, t = run.measure(ring)
            out[key] = {"value": round(world * elems * 4 * args.steps / el / GIB, 3),
                        "ms_per_step": round(el / args.steps * 1e3, 4),
                        "roofline": xgmi_roofline(t, elems * 4, elems, world, wire, "xgmi", args.steps),
                        "check": run.verify(wire)}
            if wire == "f32" and gather == "pull":  # BASELINE config 5 over the same regions: push -> sum + GD -> pull
                import numpy as np
                ps = ono_amd.ShardedParamServer(ring, np.zeros(elems, np.float32), ono_amd.GradientDescent(0.1))
                params = torch.empty(elems, dtype=torch.float32, device="cuda")
                run.refill()
                el, _ = timed_region(lambda i: ps.step(run.residuals[i], params, run.stream), args.steps,
                                     args.warmup, torch.cuda.synchronize, ctl)
                out["xgmi-ps:gd"] = {
                    "value": round(world * elems * 4 * args.steps / el / GIB, 3),
                    "ms_per_step": round(el / args.steps * 1e3, 4),
                    "workload": "ShardedParamServer.step over the xGMI exchange regions: push gradient slices -> "
                                "worker-order sum + fused /n + GD on the owned shard -> pull params"}
                ps.close()
                del params
            ring.close()
        except Exception as e:  # recorded
            out[key] = {"error": f"{type(e).__name__}: {e}"[:300]}
    os.environ["ONO_XGMI_GATHER"] = "pull"
    if args.sweep_mib:  # config 4 curve + the config-1 bucket, f32 wire
        out["xgmi:f32_size_sweep"] = size_sweep(
            torch, ono_amd, ctl, lambda e: ono_amd.WorkerRingManager.over_xgmi(
                rank, world, e, ctl.allgather_bytes, wire="f32", device=local_rank),
            sweep_sizes(args.sweep_mib), world, rank, run.stream)
    ctl.close()
    if rank == 0:
        print(json.dumps(out), flush=True)
    return 0


def size_sweep(torch, ono_amd, ctl, make_ring, sizes, world: int, rank: int, stream) -> dict:
    """pull_grads over bucket sizes (10 timed + 3
    warmup steps each, a fresh bucket per step, max over ranks), plus the
    reference's own config-1 bucket (the MLP's 109,386 f32, latency-bound).
    `sizes` = [(label, elems)], `make_ring(elems)` builds the schedule's ring.
    Informational; `value` stays the 256 MiB line."""
    out = {}
    for label, e in sizes:
        try:
            r = make_ring(e)
            k, w = 10, 3
            bufs = [torch.empty(e, dtype=torch.float32, device="cuda") for _ in range(k + w)]
            for i, t in enumerate(bufs):
                ono_amd.kernels.synth(t, SEED + i, rank)
            g = torch.empty(e, dtype=torch.float32, device="cuda")
            torch.cuda.synchronize()
            el, _ = timed_region(lambda i: r.pull_grads_dev(bufs[i], g, stream), k, w, torch.cuda.synchronize, ctl)
            alg = e * 4 * k / el / GIB
            out[label] = {"ms_per_step": round(el / k * 1e3, 4), "algbw_gib_s": round(alg, 3),
                          "busbw_gib_s": round(alg * 2 * (world - 1) / world, 3) if world > 1 else None}
            r.close()
            del bufs, g
            torch.cuda.empty_cache()
        except Exception as ex:  # recorded, never fatal
            out[label] = {"error": f"{type(ex).__name__}: {ex}"[:200]}
    return {"workload": "pull_grads_dev per bucket size (config 4 curve; config1 = the MLP bucket)", "sizes": out}


def sweep_sizes(sweep_mib: str) -> list:
    return [("config1", CONFIG1_ELEMS)] + [(f"{int(m)}MiB", int(m) << 18) for m in sweep_mib.split(",") if m]


def xgmi_link_probe(torch) -> dict | None:
    """calibrate the xGMI denominator with a measured one-link
    copy.  Rank 0 (alone, the other ranks wait at a barrier) copies 256 MiB
    from its GPU to the next one (hipMemcpyPeerAsync under torch), 10 times;
    None when this process sees a single device."""
    try:
        if torch.cuda.device_count() < 2:
            return None
        src_dev = torch.cuda.current_device()
        dst_dev = (src_dev + 1) % torch.cuda.device_count()
        a = torch.ones(1 << 26, dtype=torch.float32, device=f"cuda:{src_dev}")
        b = torch.empty(1 << 26, dtype=torch.float32, device=f"cuda:{dst_dev}")
        for _ in range(2):
            b.copy_(a)
        torch.cuda.synchronize(src_dev)
        torch.cuda.synchronize(dst_dev)
        t0 = time.perf_counter()
        for _ in range(10):
            b.copy_(a)
        torch.cuda.synchronize(src_dev)
        torch.cuda.synchronize(dst_dev)
        t = (time.perf_counter() - t0) / 10
        del a, b
        torch.cuda.empty_cache()
        return {"gbs": round((1 << 28) / t / 1e9, 1), "bytes": 1 << 28,
                "what": f"cuda:{src_dev} -> cuda:{dst_dev} device copy, one direction, 10 x 256 MiB"}
    except Exception as e:  # informational only
        return {"error": f"{type(e).__name__}: {e}"[:200]}


def n1_roofline_summary(roofline: dict, lr: dict | None, cc: dict | None) -> dict:
    """N = 1: the headline kernel's roofline gets, as flat keys (the driver's
    parser keeps scalars, not nested objects), the measured copy ceiling of the
    same size and the BASELINE config-2 reduce kernel's fractions — the
    north_star's single-GPU bar (>= 80 % of HBM) is on sum_scale, not on the
    N = 1 copy + zero fill that `value` measures."""
    lr, cc = lr or {}, cc or {}
    best = cc.get("ceiling_256MiB")
    if isinstance(best, dict) and roofline.get("achieved"):
        roofline["copy_ceiling_gbs"] = best["achieved_gbs"]
        roofline["copy_ceiling_shape"] = best["shape"]
        roofline["frac_of_copy_ceiling"] = round(roofline["achieved"] / best["achieved_gbs"], 4)
    fr = {k: lr[k]["frac_of_hbm_peak"] for k in ("k2", "k4", "k8") if isinstance(lr.get(k), dict)}
    if fr:
        roofline["reduce_kernel"] = {
            "kernel": "sum_scale_f32, 64 MiB, k = 2 / 4 / 8 inputs (BASELINE config 2)",
            "frac": fr, "frac_min": min(fr.values()), "north_star_target_frac": 0.80, "timing": lr.get("timing")}
        roofline["reduce_kernel_frac_min"] = min(fr.values())
        for k, v in fr.items():
            roofline[f"reduce_kernel_frac_{k}"] = v
        c64 = cc.get("ceiling_64MiB")
        if isinstance(c64, dict):
            fc = {k: round(lr[k]["achieved_gbs"] / c64["achieved_gbs"], 4) for k in fr}
            roofline["reduce_kernel"]["frac_of_copy_ceiling_64MiB"] = fc
            roofline["reduce_kernel_frac_of_ceiling_min"] = min(fc.values())
        sp = {k: lr[k]["frac_of_same_pool_copy_zero"] for k in fr if "frac_of_same_pool_copy_zero" in lr[k]}
        if sp:  # the 1R2W copy timed over the same buffers in the same passes (local_reduce)
            roofline["reduce_kernel"]["frac_of_same_pool_copy_zero"] = sp
            roofline["reduce_kernel_frac_of_same_pool_ceiling_min"] = min(sp.values())
    return roofline


def nx_roofline(tim: dict, bucket_bytes: int, elems: int, world: int, wire: str, algo: str, steps: int,
                elapsed: float, link: dict | None = None) -> dict:
    """N > 1: the exchange's roofline (xgmi_roofline) plus the north_star's
    per-GPU bar.  `value` is N x algBW, so it grows with N even if every link
    slows down; the bar (>= 70 % of xGMI algorithmic bandwidth) is per GPU.  An
    all-reduce moves 2(N-1)/N x bucket per rank; over N-1 links of B GB/s per
    direction that takes >= 2 bucket / (N B), i.e. algBW <= N B / 2 (307 GB/s
    at N = 8).  Whole-step time, local kernels included."""
    rl = xgmi_roofline(tim, bucket_bytes, elems, world, wire, algo, steps)
    if link:
        rl["link_probe"] = link
        if rl["achieved"] and link.get("gbs"):
            rl["frac_of_measured_links"] = round(rl["achieved"] / (link["gbs"] * (world - 1)), 4)
    algbw = bucket_bytes * steps / elapsed / 1e9
    peak_alg = world * XGMI_LINK_GBS / 2
    rl.update({
        "per_gpu_algbw_gbs": round(algbw, 2), "xgmi_algbw_peak_gbs": round(peak_alg, 1),
        "frac_of_xgmi_algbw": round(algbw / peak_alg, 4), "north_star_target_frac_of_xgmi_algbw": 0.70,
        "value_note": "value = N x per-GPU algBW (GiB/s, weak scaling); compare frac_of_xgmi_algbw across N"})
    # flat copies of the per-phase split for the driver's parser (it keeps scalars only)
    for ph, ms in (rl.get("phases_ms_per_step") or {}).items():
        rl[f"phase_ms_{ph}"] = ms
    for ph, g in (rl.get("per_link_gbs") or {}).items():
        rl[f"per_link_gbs_{ph}"] = g
    return rl


def xgmi_roofline(tim: dict, bucket_bytes: int, elems: int, world: int, wire: str, algo: str,
                  steps: int) -> dict:
    """N > 1: the exchange is xGMI-bound.  achieved = bytes each rank sends per
    step / the step's collective time (HIP events on the launch stream); peak =
    the N-1 direct links a rank can drive at once, 76.8 GB/s each per direction.
    For the RCCL ring all-reduce the bytes are its busBW bytes 2(N-1)/N x bucket."""
    wb = 2 if wire == "f16" else 4
    if algo == "auto":  # the library's AUTO resolution (ono_ring.cpp resolved_algo)
        algo = "allreduce" if wire == "f32" else "direct"
    if algo == "allreduce" and wire == "f32":
        bytes_out = 2 * (world - 1) / world * bucket_bytes            # ring all-reduce (any segmentation)
    elif algo in ("direct", "xgmi"):
        bytes_out = (world - 1) / world * (bucket_bytes + elems * wb)  # all-to-all f32 + all-gather
    else:
        bytes_out = 2 * (world - 1) / world * elems * wb              # n-1 + n-1 hops
    step_coll_ms = tim["collective_ms"] / max(steps, 1)  # timing is enabled for the K timed steps only
    ach = bytes_out / (step_coll_ms * 1e-3) / 1e9 if step_coll_ms > 0 else None
    peak = XGMI_LINK_GBS * (world - 1)
    kern_ms = tim["kernel_ms"] / max(tim["kernels"], 1)
    phases = {k: round(v[0] / max(steps, 1), 4) for k, v in tim.get("phases", {}).items() if v[1]}
    per_link = {}
    if algo == "xgmi" and world > 1 and phases:
        # one peer segment per link: the scatter moves 4 N/n bytes to each peer, the gather wire N/n
        for ph, b in (("xgmi_scatter", 4 * elems / world), ("xgmi_gather", wb * elems / world)):
            if phases.get(ph):
                per_link[ph] = round(b / (phases[ph] * 1e-3) / 1e9, 1)
    return {
        "bound": "xgmi", "schedule": f"{algo}:{wire}",
        "phases_ms_per_step": phases, "per_link_gbs": per_link or None,
        "achieved": round(ach, 1) if ach else None, "peak": round(peak, 1), "unit": "GB/s",
        "frac": round(ach / peak, 4) if ach else None, "traffic": None,
        # BASELINE.md's primary denominator: one xGMI link (153.6 GB/s, the single-ring per-link bound);
        # `frac` above uses the stricter every-link peak of a fully connected node
        "frac_of_one_link_153gbs": round(ach / (2 * XGMI_LINK_GBS), 4) if ach else None,
        "wire_bytes_per_rank_per_step": int(bytes_out),
        "collective_ms_per_step": round(step_coll_ms, 4),
        "peak_note": "bytes each rank sends per step / collective time, vs (N-1) direct xGMI links x 76.8 GB/s "
                     "per direction (153.6 GB/s bidirectional spec per link)",
        "kernel_avg_us": round(kern_ms * 1e3, 2), "kernel_launches": tim["kernels"],
    }


if __name__ == "__main__":
    sys.exit(main())
