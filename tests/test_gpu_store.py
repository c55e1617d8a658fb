"""GPU parity of the parameter-server store / synchronizers (device resident)
against the oracle and the reference's own unit tests.

Reference tests restated here on the HBM store:
  blocking/shard.rs:131-185  accumulation/update, double buffering, averaging
  blocking/store.rs:175-243  ragged shards, buffer swap, CAS lock, flow, ragged edge
"""
import threading

import numpy as np
import pytest
import torch

import ono_amd
from ono_amd import AddOptimizer, Adam, GradientDescent, GradientDescentWithMomentum
from conftest import SEED, assert_bitexact
from oracle import oracle as O
from oracle import oracle_np as N

pytestmark = pytest.mark.gpu


def test_accumulation_and_update():
    s = ono_amd.BlockingStore(3, 1, np.zeros(3), AddOptimizer())
    s.accumulate([1.0, 2.0, 3.0])
    s.accumulate([1.0, 1.0, 1.0])
    s.update_params()
    assert list(s.pull_params()) == [2.0, 3.0, 4.0]


def test_gradient_is_averaged_across_workers():
    s = ono_amd.BlockingStore(2, 2, np.zeros(2), AddOptimizer())
    s.accumulate([2.0, 4.0])
    s.accumulate([2.0, 4.0])
    s.update_params()
    assert list(s.pull_params()) == [2.0, 4.0]


def test_handle_ragged_shards():
    s = ono_amd.BlockingStore(8, 1, np.zeros(15), AddOptimizer())
    s.accumulate(np.ones(15))
    s.update_params()
    assert list(s.pull_params()) == [1.0] * 15


def test_handle_buffer_swap():
    s = ono_amd.BlockingStore(1, 1, np.zeros(10), AddOptimizer())
    s.accumulate(np.ones(10))
    s.update_params()
    assert s.active_idx == 1
    s.accumulate(np.full(10, 5.0))
    assert list(s.pull_params()) == [1.0] * 10
    s.update_params()
    assert list(s.pull_params()) == [6.0] * 10


def test_update_locking_mechanism():
    s = ono_amd.BlockingStore(1, 1, np.zeros(10), AddOptimizer())
    s.set_updating(True)
    before = s.active_idx
    s.update_params()
    assert s.active_idx == before
    s.set_updating(False)
    s.update_params()
    assert s.active_idx != before


@pytest.mark.parametrize("params,shard", [(100, 25), (105, 10)])
def test_store_initialization_and_flow(params, shard):
    s = ono_amd.BlockingStore(shard, 1, np.zeros(params), AddOptimizer())
    s.accumulate(np.ones(params))
    s.update_params()
    out = s.pull_params()
    assert out.size == params and np.all(out == 1.0)


def test_size_mismatch():
    s = ono_amd.BlockingStore(2, 1, np.zeros(4), GradientDescent(0.1))
    with pytest.raises(ono_amd.SizeMismatch):
        s.accumulate(np.ones(5))
    with pytest.raises(ono_amd.SizeMismatch):
        s.pull_params(np.zeros(3, np.float32))


OPTS = {
    "gd": GradientDescent(0.1),
    "momentum": GradientDescentWithMomentum(0.1, 0.9),
    "adam": Adam(0.1, 0.9, 0.999, 1e-8),
}


def test_store_golden(golden):
    g = golden("store")
    for kind, opt in OPTS.items():
        for nworkers in (1, 3):
            s = ono_amd.BlockingStore(100, nworkers, g[f"{kind}_w{nworkers}_init"], opt)
            for rnd in range(4):
                for w in range(nworkers):
                    s.accumulate(N.synth(1031, SEED + 1000 * rnd + w, w + 1))
                s.update_params()
                assert_bitexact(s.pull_params(), g[f"{kind}_w{nworkers}_traj"][rnd], f"{kind} w{nworkers} r{rnd}")


@pytest.mark.parametrize("kind", ["gd", "momentum", "adam"])
@pytest.mark.parametrize("nparams", [1, 4099, 1 << 20])
def test_store_vs_oracle_many_rounds(kind, nparams):
    init = O.synth(nparams, SEED + 1, 9)
    opt = OPTS[kind]
    s = ono_amd.BlockingStore(ono_amd.shard_size_for(nparams), 2, init, opt)
    ref = O.Store(init, 7, 2, kind, lr=0.1, momentum=0.9, beta1=0.9, beta2=0.999, eps=1e-8)
    for rnd in range(6):
        for w in range(2):
            g = O.synth(nparams, SEED + rnd, w)
            s.accumulate(g)
            ref.accumulate(g)
        s.update_params()
        ref.update_params()
    assert_bitexact(s.pull_params(), ref.pull_params(), kind)


@pytest.mark.parametrize("kind", ["gd", "adam"])
def test_wild_store_single_worker(kind):
    init = O.synth(5000, SEED, 2)
    s = ono_amd.WildStore(100, init, OPTS[kind])
    ref = O.WildStore(init, 100, kind, lr=0.1, momentum=0.9, beta1=0.9, beta2=0.999, eps=1e-8)
    for rnd in range(5):
        g = O.synth(5000, SEED + rnd, 1)
        s.accumulate(g)
        ref.accumulate(g)
        s.update_params()
    assert_bitexact(s.pull_params(), ref.pull_params())


def test_barrier_sync_three_workers():
    """Three worker tasks step through BarrierSync; the leader applies the
    averaged update once per round; every worker pulls the same params.
    Gradients are integer-valued so the arrival order cannot change sums."""
    nparams, nworkers, rounds = 1031, 3, 5
    init = O.synth(nparams, SEED, 0)
    s = ono_amd.BlockingStore(64, nworkers, init, GradientDescent(0.1))
    sync = ono_amd.BarrierSync(nworkers)
    clones = [sync.clone() for _ in range(nworkers - 1)] + [sync]
    outs = [[None] * rounds for _ in range(nworkers)]
    grads = [[np.round(O.synth(nparams, SEED + r, w) * 64).astype(np.float32) for r in range(rounds)]
             for w in range(nworkers)]
    errors = []

    def worker(w):
        try:
            p = np.empty(nparams, np.float32)
            for r in range(rounds):
                clones[w].step(s, grads[w][r], p)
                outs[w][r] = p.copy()
        except Exception as e:  # pragma: no cover
            errors.append(e)

    ts = [threading.Thread(target=worker, args=(w,)) for w in range(nworkers)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert not errors and all(not t.is_alive() for t in ts)
    ref = O.Store(init, 64, nworkers, "gd", lr=0.1)
    for r in range(rounds):
        for w in range(nworkers):
            ref.accumulate(grads[w][r])
        ref.update_params()
        e = ref.pull_params()
        for w in range(nworkers):
            assert_bitexact(outs[w][r], e, f"round {r} worker {w}")
    for c in clones:
        c.drop()


def test_no_blocking_sync_single_worker():
    init = O.synth(777, SEED, 3)
    s = ono_amd.BlockingStore(50, 1, init, GradientDescentWithMomentum(0.1, 0.9))
    sync = ono_amd.NoBlockingSync()
    ref = O.Store(init, 50, 1, "momentum", lr=0.1, momentum=0.9)
    p = np.empty(777, np.float32)
    for r in range(4):
        g = O.synth(777, SEED + r, 1)
        sync.step(s, g, p)
        ref.accumulate(g)
        ref.update_params()
        assert_bitexact(p, ref.pull_params())
    sync.drop()


def test_lineal_convergence():
    """parameter_server/src/test.rs:85-126 on the device store."""
    s = ono_amd.BlockingStore(1, 1, np.full(2, 0.5, np.float32), GradientDescent(0.1))
    sync = ono_amd.BarrierSync(1)
    p = s.pull_params()
    for _ in range(100):
        g = N.quantize_f16((p - np.float32(1.0)).astype(np.float32))
        sync.step(s, g, p)
    assert np.all(np.abs(p - 1.0) < 1e-3)


@pytest.mark.parametrize("kind", ["gd", "momentum", "adam"])
def test_sharded_ps_single_gpu(kind):
    """ono_ps at nranks = 1: reduce-scatter/all-gather degenerate to copies;
    the fused shard update equals the store oracle with nworkers = 1."""
    nparams = 100003
    ring = ono_amd.WorkerRingManager(0, 1, nparams)
    init = O.synth(nparams, SEED, 4)
    ps = ono_amd.ShardedParamServer(ring, init, OPTS[kind])
    ref = O.Store(init, 1000, 1, kind, lr=0.1, momentum=0.9, beta1=0.9, beta2=0.999, eps=1e-8)
    params = torch.empty(nparams, device="cuda:0")
    for r in range(3):
        g = O.synth(nparams, SEED + r, 1)
        ps.step(torch.from_numpy(g).cuda(), params)
        ref.accumulate(g)
        ref.update_params()
        torch.cuda.synchronize()
        assert_bitexact(params.cpu().numpy(), ref.pull_params(), f"round {r}")
    ps.close()
    ring.close()


@pytest.mark.parametrize("kind", ["gd", "momentum", "adam"])
@pytest.mark.parametrize("nparams", [1, 4099, 1 << 20])
def test_store_accumulate_f16_wire(kind, nparams):
    """The PS server's receive path fused: the worker's f16 payload
    (ParamServerHandle::push_grad) is decoded inside the accumulate kernel.
    Equal to the oracle fed the CPU decode of the same payload (worker.rs:
    82-101), host and device payloads, specials included."""
    init = O.synth(nparams, SEED + 1, 9)
    s = ono_amd.BlockingStore(ono_amd.shard_size_for(nparams), 2, init, OPTS[kind])
    ref = O.Store(init, 7, 2, kind, lr=0.1, momentum=0.9, beta1=0.9, beta2=0.999, eps=1e-8)
    for rnd in range(4):
        for w in range(2):
            h = O.f16_encode(O.synth_special(nparams, SEED + rnd, w) if nparams > 200 else
                             O.synth(nparams, SEED + rnd, w))
            if w == 0:
                s.accumulate_f16(h)
            else:
                s.accumulate_f16(torch.from_numpy(h.view(np.int16)).cuda())
            ref.accumulate(O.f16_decode(h))
        s.update_params()
        ref.update_params()
        ok = O.same_or_both_nan(s.pull_params(), ref.pull_params())
        assert ok.all(), f"{kind} round {rnd}: {np.count_nonzero(~ok)} differ"


def test_wild_store_and_sync_step_f16():
    init = O.synth(5000, SEED, 2)
    s = ono_amd.WildStore(100, init, OPTS["adam"])
    ref = O.WildStore(init, 100, "adam", lr=0.1, momentum=0.9, beta1=0.9, beta2=0.999, eps=1e-8)
    for rnd in range(4):
        h = O.f16_encode(O.synth(5000, SEED + rnd, 1))
        s.accumulate_f16(h)
        ref.accumulate(O.f16_decode(h))
    assert_bitexact(s.pull_params(), ref.pull_params(), "wild f16")
    b = ono_amd.BlockingStore(50, 1, init, GradientDescentWithMomentum(0.1, 0.9))
    sync = ono_amd.NoBlockingSync()
    rb = O.Store(init, 50, 1, "momentum", lr=0.1, momentum=0.9)
    p = np.empty(5000, np.float32)
    for r in range(3):
        h = O.f16_encode(O.synth(5000, SEED + r, 4))
        sync.step_f16(b, h, p)
        rb.accumulate(O.f16_decode(h))
        rb.update_params()
        assert_bitexact(p, rb.pull_params(), f"sync f16 round {r}")
    sync.drop()
