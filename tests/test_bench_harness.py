"""bench.py's multi-rank plumbing on CPU (gloo, world_size 2): the RCCL-id
broadcast, barrier-bracketed timing with max-over-ranks, and the JSON line
contract.  The GPU steps themselves run only on the MI355X (driver's N>1 runs)."""
import json
import os
import socket
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


WORKER = r"""
import json, os, sys, time
sys.path.insert(0, {root!r})
import bench
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
ctl = bench.Ctl(world, rank)
uid = bytes(range(128)) if rank == 0 else None
uid = ctl.bcast_bytes(uid)
assert uid == bytes(range(128))
calls = []
def step(i):
    calls.append(i)
    time.sleep(0.02 if rank == 1 else 0.001)   # rank 1 is the slow one
elapsed, local = bench.timed_region(step, 5, 2, lambda: None, ctl)
print(json.dumps({{"rank": rank, "elapsed": elapsed, "local": local, "calls": calls}}), flush=True)
ctl.close()
"""


def test_two_rank_timing_takes_max_over_ranks():
    port = _free_port()
    procs = []
    for rank in range(2):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK=str(rank),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-c", WORKER.format(root=ROOT)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        out, err = p.communicate(timeout=120)
        assert p.returncode == 0, err
        outs.append(json.loads(out.strip().splitlines()[-1]))
    r0, r1 = sorted(outs, key=lambda d: d["rank"])
    assert r0["calls"] == r1["calls"] == list(range(7))   # W warmup then exactly K timed
    assert r0["elapsed"] == r1["elapsed"]                   # both report the max
    assert r0["elapsed"] >= r1["local"] >= 5 * 0.02 * 0.9
    assert r0["local"] < r1["local"]


def test_single_rank_ctl_is_noop():
    ctl = bench.Ctl(1, 0)
    assert ctl.bcast_bytes(b"x") == b"x"
    assert ctl.max(3.5) == 3.5
    e, loc = bench.timed_region(lambda i: None, 3, 1, lambda: None, ctl)
    assert e == loc >= 0


def test_build_line_contract():
    line = bench.build_line(value=123.0, n_gpus=4, steps=10, warmup=2, elapsed=0.5,
                            bucket_bytes=256 << 20, wire="f32", extra={"roofline": {"bound": "xgmi"}})
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config"):
        assert key in line
    assert line["metric"] == json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
    assert line["scaling"] == "weak" and line["higher_is_better"] is True and line["vs_baseline"] is None
    assert line["ms_per_step"] == pytest.approx(50.0)
    assert line["algbw_gib_s"] == pytest.approx(5.0)
    assert line["busbw_gib_s"] == pytest.approx(5.0 * 2 * 3 / 4)
    assert line["config"]["parallelism"] == "dp4"
    json.dumps(line)


def test_gpus_mismatch_is_an_error(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "1")
    assert bench.main(["--gpus", "2"]) == 2


XGMI_SPAWN = r"""
import json, os, sys, types
sys.path.insert(0, {root!r})
import bench
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
ctl = bench.Ctl(world, rank)
args = types.SimpleNamespace(steps=2, warmup=1, bucket_mib=1, xgmi_timeout=90.0)
res = bench.xgmi_spawn(args, ctl, world, rank, rank)
print(json.dumps({{"rank": rank, "res": res}}), flush=True)
ctl.close()
"""


def test_xgmi_children_under_torchrun_rendezvous_and_report():
    """bench.py's N > 1 xGMI leg runs in child processes.  Launched exactly as
    the driver launches bench.py (torch.distributed.run, whose agent-store
    environment the children must not inherit), the children find each other
    on their own port; when the GPU step then fails (here: no GPU) every parent
    returns and rank 0 records the child's error — no hang, no store timeout."""
    port = _free_port()
    script = os.path.join(ROOT, "tests", "_xgmi_spawn_probe.py")
    with open(script, "w") as f:
        f.write(XGMI_SPAWN.format(root=ROOT))
    try:
        r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                            "--master-addr", "127.0.0.1", "--master-port", str(port), script],
                           capture_output=True, text=True, timeout=240,
                           env=dict(os.environ, HIP_VISIBLE_DEVICES=""))
    finally:
        os.remove(script)
    assert r.returncode == 0, r.stderr[-3000:]
    outs, dec, text, i = [], json.JSONDecoder(), r.stdout, 0  # the two ranks' lines may interleave
    while (i := text.find('{"rank"', i)) >= 0:
        obj, end = dec.raw_decode(text, i)
        outs.append(obj)
        i = end
    r0 = [o for o in outs if o["rank"] == 0][0]["res"]
    r1 = [o for o in outs if o["rank"] == 1][0]["res"]
    assert r1 == {}
    err = r0["xgmi"]["error"]
    assert "killed after" not in err and "exited" not in err, err  # the children rendezvoused and reported


def test_n1_line_carries_reduce_kernel_and_ceiling_as_flat_keys():
    """The driver's parser keeps the roofline's scalar keys only (BENCH_r03.json
    `parsed.roofline` dropped the nested reduce_kernel): the config-2 reduce
    fractions and the copy ceiling must be there as flat keys."""
    rl = {"bound": "hbm", "achieved": 6900.0, "frac": 0.8625}
    lr = {"k2": {"frac_of_hbm_peak": 0.79, "achieved_gbs": 6320.0},
          "k4": {"frac_of_hbm_peak": 0.785, "achieved_gbs": 6280.0},
          "k8": {"frac_of_hbm_peak": 0.80, "achieved_gbs": 6400.0}, "timing": "events"}
    cc = {"ceiling_256MiB": {"shape": "copy_zero", "achieved_gbs": 6950.0},
          "ceiling_64MiB": {"shape": "copy_zero", "achieved_gbs": 6400.0}}
    bench.n1_roofline_summary(rl, lr, cc)
    line = bench.build_line(value=2100.0, n_gpus=1, steps=20, warmup=5, elapsed=0.0024,
                            bucket_bytes=256 << 20, wire="f32", extra={"roofline": rl})
    flat = {k: v for k, v in line["roofline"].items() if not isinstance(v, (dict, list))}
    assert flat["reduce_kernel_frac_min"] == 0.785
    assert flat["reduce_kernel_frac_k2"] == 0.79 and flat["reduce_kernel_frac_k8"] == 0.80
    assert flat["copy_ceiling_gbs"] == 6950.0 and flat["copy_ceiling_shape"] == "copy_zero"
    assert flat["frac_of_copy_ceiling"] == pytest.approx(6900 / 6950, abs=1e-4) and flat["frac_of_copy_ceiling"] <= 1
    assert flat["reduce_kernel_frac_of_ceiling_min"] == pytest.approx(6280 / 6400, abs=1e-4)
    assert "reduce_kernel_frac_of_same_pool_ceiling_min" not in flat  # no same-pool copy timed
    json.dumps(line)


def test_n1_line_carries_the_same_pool_ceiling_of_config2():
    """local_reduce also times the 1R2W copy over k = 2's own buffers in the same
    passes; its fractions travel flat as well."""
    rl = {"bound": "hbm", "achieved": 6900.0, "frac": 0.8625}
    lr = {"k2": {"frac_of_hbm_peak": 0.79, "achieved_gbs": 6320.0, "frac_of_same_pool_copy_zero": 0.991},
          "k4": {"frac_of_hbm_peak": 0.785, "achieved_gbs": 6280.0, "frac_of_same_pool_copy_zero": 0.985},
          "k8": {"frac_of_hbm_peak": 0.80, "achieved_gbs": 6400.0, "frac_of_same_pool_copy_zero": 1.004},
          "copy_zero_same_pool": {"achieved_gbs": 6376.0}, "timing": "events"}
    bench.n1_roofline_summary(rl, lr, {})
    assert rl["reduce_kernel_frac_of_same_pool_ceiling_min"] == 0.985
    assert rl["reduce_kernel"]["frac_of_same_pool_copy_zero"]["k8"] == 1.004
    json.dumps(rl)


@pytest.mark.parametrize("algo,wire", [("xgmi", "f32"), ("xgmi", "f16"), ("allreduce", "f32"), ("direct", "f16")])
def test_nx_line_carries_xgmi_algbw_links_and_phases(algo, wire):
    """The N > 1 line (driver's 8-GPU run): frac_of_xgmi_algbw, per_link_gbs and
    phases_ms_per_step, with flat copies of the per-phase and per-link figures."""
    world, steps, elems = 8, 10, 64 << 20
    phases = {"kernel": (2.0, 10), "rccl": (0.0, 0), "xgmi_scatter": (3.0, 10), "xgmi_barrier": (0.2, 20),
              "xgmi_gather": (2.5, 10)} if algo == "xgmi" else {"kernel": (1.0, 10), "rccl": (9.0, 10)}
    tim = {"kernel_ms": 2.0, "kernels": 10, "collective_ms": 9.0, "collectives": 10, "phases": phases}
    rl = bench.nx_roofline(tim, elems * 4, elems, world, wire, algo, steps, elapsed=0.012,
                           link={"gbs": 70.0})
    line = bench.build_line(value=1.0, n_gpus=world, steps=steps, warmup=2, elapsed=0.012,
                            bucket_bytes=elems * 4, wire=wire, extra={"roofline": rl})
    r = line["roofline"]
    assert r["bound"] == "xgmi" and r["frac_of_xgmi_algbw"] > 0 and r["north_star_target_frac_of_xgmi_algbw"] == 0.7
    assert r["xgmi_algbw_peak_gbs"] == pytest.approx(world * bench.XGMI_LINK_GBS / 2, abs=0.1)
    assert isinstance(r["phases_ms_per_step"], dict) and r["phases_ms_per_step"]
    assert r["frac_of_measured_links"] > 0
    for ph, ms in r["phases_ms_per_step"].items():
        assert r[f"phase_ms_{ph}"] == ms
    if algo == "xgmi":
        assert set(r["per_link_gbs"]) == {"xgmi_scatter", "xgmi_gather"}
        assert r["per_link_gbs_xgmi_scatter"] == pytest.approx(4 * elems / world / 0.3e-3 / 1e9, rel=1e-3)
    else:
        assert r["per_link_gbs"] is None
    json.dumps(line)


def _bench(args, timeout=120, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "ONO_BENCH_DEADLINE")}
    e.update(env, HIP_VISIBLE_DEVICES="")
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--steps", "3", "--warmup", "1",
                        *args], capture_output=True, text=True, timeout=timeout, env=e, cwd=ROOT)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, lines, time.time() - t0


def test_gpus_2_without_a_launcher_starts_its_ranks_and_prints_one_line():
    """`bench.py --gpus 2` with no torch.distributed.run around it starts the two ranks
    itself (one process each, before any GPU call) and relays rank 0's line: exactly one JSON line."""
    r, lines, _ = _bench(["--gpus", "2"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "dp2"
    assert line["check"]["ok"] and "alt_schedules" in line and "size_sweep" in line
    assert line["deadline"]["skipped"] == []


def test_a_leg_that_would_end_past_the_deadline_is_skipped_and_the_line_printed_in_time():
    """With 20 s for the line and 8-s legs: the headline and the first leg are in, every later leg that
    would end past the deadline is recorded as skipped, the line comes out before the deadline."""
    r, lines, took = _bench(["--deadline", "20", "--dry-leg-s", "8"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert line["value"] > 0 and line["check"]["ok"]
    assert line["host_fed"] == {"dry_run": True}
    assert "tcp_edge" in line["deadline"]["skipped"] and "cpu_baseline" in line["deadline"]["skipped"]
    assert took < 20


def test_a_leg_that_overruns_is_cut_and_the_headline_survives():
    """A leg that fits the estimate but runs on past the deadline: at deadline + grace the backstop prints
    the line as it stands (headline, check, the cut leg named) and ends the process."""
    r, lines, took = _bench(["--deadline", "16", "--dry-leg-s", "60"], ONO_BENCH_GRACE_S="2")
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert line["value"] > 0 and line["check"]["ok"]
    assert line["deadline"]["cut"] == "host_fed" and "host_fed" not in line
    assert took < 40


def test_two_self_launched_ranks_cut_together():
    """N = 2, self-launched: the ranks share the launcher's deadline; a collective leg that overruns is cut
    on both, rank 0's line is relayed, nobody is left waiting."""
    r, lines, took = _bench(["--gpus", "2", "--deadline", "25", "--dry-leg-s", "60"], ONO_BENCH_GRACE_S="2")
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["deadline"]["cut"]
    assert took < 60


def test_rccl_failure_falls_back_to_xgmi_in_fresh_ranks():
    """the RCCL ring of the headline cannot be created (dry-run stub of a failing
    ncclCommInitRank): rank 0 reports it, the launcher starts a fresh set of ranks on the xGMI schedule
    (no RCCL) and relays one line that records headline_fallback {from, reason}, within the deadline."""
    r, lines, took = _bench(["--gpus", "2", "--deadline", "60"], ONO_BENCH_DRY_RING_FAIL="1")
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["headline_fallback"]["from"] == "allreduce"
    assert "ncclCommInitRank" in line["headline_fallback"]["reason"]
    assert line["config"]["schedule"] == "xgmi" and line["value"] > 0 and line["check"]["ok"]
    assert line["n_gpus"] == 2 and "headline_error" not in line
    assert took < 60


def test_hung_headline_falls_back_to_xgmi():
    """The headline's ring never comes up (stub: ring creation sleeps): the rank's headline watchdog ends it
    after ONO_BENCH_HEADLINE_TIMEOUT_S with a headline_error, and the xGMI fallback measures the line."""
    r, lines, took = _bench(["--gpus", "2", "--deadline", "60"], ONO_BENCH_DRY_RING_HANG="1",
                            ONO_BENCH_HEADLINE_TIMEOUT_S="4")
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert "did not finish in 4 s" in line["headline_fallback"]["reason"]
    assert line["config"]["schedule"] == "xgmi" and line["value"] > 0
    assert took < 60


@pytest.mark.parametrize("fail", [False, True])
def test_under_torchrun_one_gpu_free_launcher_prints_one_line(fail):
    """Launched the way the driver launches N > 1 (torch.distributed.run --nproc-per-node 2): torchrun's local
    rank 0 becomes the GPU-free launcher of the two ranks, the other torchrun process leaves at once; exactly one
    JSON line comes out, with the xGMI fallback when the RCCL ring fails."""
    port = _free_port()
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "ONO_BENCH_DEADLINE")}
    e.update(HIP_VISIBLE_DEVICES="")
    if fail:
        e["ONO_BENCH_DRY_RING_FAIL"] = "1"
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--dry-run", "--steps", "3", "--warmup", "1", "--deadline", "60"],
                       capture_output=True, text=True, timeout=180, env=e, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["value"] > 0
    assert ("headline_fallback" in line) == fail
