"""The RCCL call mapping of the exchange plans, executed before the 8-GPU node
does.

RCCL refuses two ranks per device, so on a one-GPU box the calls run_plan
(ono_ring.cpp) makes for a plan step — ncclGroupStart / ncclSend / ncclRecv /
ncclGroupEnd, ncclAllReduce, ncclReduceScatter, ncclAllGather — had never run
with the pointers, counts and peers a real rank passes.  Here the product runs
unmodified in one process whose ranks are threads on cuda:0, with a recording
stand-in for those functions preloaded (tests/native/rccl_record.hip, test
infrastructure, never linked into the product).  tests/rccl_record_worker.py
checks that each rank's calls are its plan's communication steps (kind, count,
dtype, peer, grouping, one stream, one base address per plan buffer, the
buckets at their real addresses) and that the results the stand-in produces
by carrying the calls out (matched copies, rank-order sums) equal the oracle
bit for bit: HOPS and DIRECT against the reference hop ring
(worker_ring.rs:112-204), ALLREDUCE (one and four segments) against the
rank-order f32 sum / n, the PS step against the BlockingStore
(blocking/store.rs:84-124).
"""
import json
import os
import subprocess
import sys
import tempfile

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
SHIM = os.path.join(HERE, "native", "librccl_record.so")


def run_case(case: dict, timeout: float = 300.0) -> None:
    assert os.path.exists(SHIM), "build tests/native (make -C tests/native) first"
    with tempfile.TemporaryDirectory(prefix="ono_rccl_rec_") as d:
        rec = os.path.join(d, "calls.jsonl")
        pre = os.environ.get("LD_PRELOAD", "")
        env = dict(os.environ, ONO_RCCL_RECORD=rec, PYTHONUNBUFFERED="1",
                   LD_PRELOAD=(pre + " " + SHIM).strip())
        p = subprocess.run([sys.executable, os.path.join(HERE, "rccl_record_worker.py"), json.dumps(case), rec],
                           env=env, capture_output=True, text=True, timeout=timeout)
        assert p.returncode == 0, p.stderr[-3000:]
        out = json.loads(p.stdout.strip().splitlines()[-1])
        assert out["ok"], out["msg"]


@pytest.mark.parametrize("wire", ["f16", "f32"])
@pytest.mark.parametrize("algo,n,size", [("hops", 2, 109386), ("hops", 3, 40001), ("hops", 4, 4099),
                                         ("direct", 2, 109386), ("direct", 3, 40001), ("direct", 5, 65539)])
def test_p2p_schedules_call_mapping(algo, n, size, wire):
    run_case({"algo": algo, "n": n, "size": size, "wire": wire, "rounds": 2})


@pytest.mark.parametrize("n,size,segments", [(2, 109386, 1), (3, 40001, 1), (2, (1 << 24) + 5, 4),
                                             (3, (1 << 24) + 7, 4)])
def test_allreduce_call_mapping(n, size, segments):
    """The N > 1 headline schedule (AUTO = ALLREDUCE for f32), segmented: the
    finaliser of segment j on the side stream beside the all-reduce of j+1."""
    run_case({"algo": "allreduce", "n": n, "size": size, "wire": "f32", "segments": segments, "rounds": 2})


@pytest.mark.parametrize("algo,wire", [("hops", "f16"), ("direct", "f16"), ("direct", "f32")])
def test_host_fed_sub_rounds_over_rccl_calls(algo, wire, monkeypatch):
    """pull_grads_host: the sub-round plans issued on the ring's compute
    stream while H2D / D2H run beside them; bit-exact with the whole round."""
    monkeypatch.setenv("ONO_HOST_CHUNK_MIB", "1")
    run_case({"algo": algo, "n": 3, "size": (1 << 20) + 3, "wire": wire, "rounds": 1, "host": True})


@pytest.mark.parametrize("opt", ["gd", "momentum", "adam"])
@pytest.mark.parametrize("n", [2, 3])
def test_ps_step_call_mapping(n, opt):
    """ono_ps_step over RCCL: reduce-scatter of the padded gradients, the
    fused shard update, all-gather of the parameters (BASELINE config 5)."""
    run_case({"mode": "ps", "n": n, "size": 100003, "opt": opt, "steps": 3})
