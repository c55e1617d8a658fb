"""The N > 1 exchange plans run on the GPU (ono_plan_run_local*): every rank's
plan, built by the same host code the RCCL interpreter executes, run by
co-resident ranks on one device in lockstep — kernels through the
interpreter's own launcher (plan_kernel), sends matched with receives as
device copies, collectives as the sum over ranks in rank order.  RCCL refuses
two ranks per device, so this is how the DIRECT / HOPS / ALLREDUCE / PS plans'
device work is checked on a one-GPU box before the driver's 8-GPU run.

Oracle: the ring restatement (worker_ring.rs:112-204) for HOPS and DIRECT,
bit-exact for both wires; the all-reduce against the f32 sum in rank order
then / n, bit-exact (the emulation fixes RCCL's order; the RCCL tolerance is
DESIGN §5's); the PS step against the BlockingStore oracle fed in rank order
(store.rs:84-124, shard.rs:74-92), bit-exact, three steps.
"""
import numpy as np
import pytest
import torch

import ono_amd
from ono_amd import plan as P
from conftest import SEED, assert_bitexact
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.parametrize("algo", ["hops", "direct"])
@pytest.mark.parametrize("wire", ["f16", "f32"])
@pytest.mark.parametrize("n,length", [(2, 109386), (3, 2 ** 18 + 5), (5, 65541), (8, 1000003), (16, 4099)])
def test_exact_plans_vs_oracle(algo, wire, n, length):
    ins = [O.synth(length, SEED + 17, r) for r in range(n)]
    res = [dev(x) for x in ins]
    grads = [torch.full_like(r, 7.0) for r in res]
    P.run_local(algo, wire, res, grads)
    torch.cuda.synchronize()
    want, _ = O.ring_pull_grads(ins, wire)
    for r in range(n):
        assert_bitexact(grads[r].cpu().numpy(), want[r], f"{algo}/{wire} rank {r}")
        assert not res[r].cpu().numpy().view(np.uint32).any(), f"rank {r}: residual not zeroed"


@pytest.mark.parametrize("algo", ["hops", "direct"])
@pytest.mark.parametrize("wire", ["f16", "f32"])
@pytest.mark.parametrize("n,length,sub", [(2, 109386, 4096), (3, 2 ** 18 + 5, 1 << 14), (5, 65541, 64),
                                          (8, 1000003, 1 << 16)])
def test_host_fed_sub_rounds_vs_oracle(algo, wire, n, length, sub):
    """The host-fed HOPS / DIRECT round's sub-rounds (ono_ring_pull_grads_host cuts the round into a
    slice of every chunk each) run on the device one after another: bit-exact with the whole round."""
    ins = [O.synth(length, SEED + 31, r) for r in range(n)]
    res = [dev(x) for x in ins]
    grads = [torch.full_like(r, 7.0) for r in res]
    P.run_local_sub(algo, wire, res, grads, sub)
    torch.cuda.synchronize()
    want, _ = O.ring_pull_grads(ins, wire)
    for r in range(n):
        assert_bitexact(grads[r].cpu().numpy(), want[r], f"{algo}/{wire} rank {r}")
        assert not res[r].cpu().numpy().view(np.uint32).any(), f"rank {r}: residual not zeroed"


@pytest.mark.parametrize("segments", [1, 4])
@pytest.mark.parametrize("n,length", [(2, (1 << 22) + 5), (3, 1000003), (8, (1 << 22) + 7)])
def test_allreduce_plan_segments(segments, n, length):
    """the main N > 1 line's plan (ALLREDUCE + the fused finaliser, segmented
    as the library runs it by default)"""
    ins = [O.synth(length, SEED + 19, r) for r in range(n)]
    res = [dev(x) for x in ins]
    grads = [torch.full_like(r, 7.0) for r in res]
    P.run_local("allreduce", "f32", res, grads, segments=segments)
    torch.cuda.synchronize()
    acc = ins[0].copy()
    for x in ins[1:]:
        acc = (acc + x).astype(np.float32)
    want = (acc / np.float32(n)).astype(np.float32)
    for r in range(n):
        assert_bitexact(grads[r].cpu().numpy(), want, f"rank {r}")
        assert not res[r].cpu().numpy().view(np.uint32).any()


@pytest.mark.parametrize("kind", ["gd", "momentum", "adam"])
@pytest.mark.parametrize("n,nparams", [(2, 4099), (3, 100003), (5, 65536)])
def test_ps_plan_vs_store_oracle(kind, n, nparams):
    lr, mu, b1, b2, eps = 0.1, 0.9, 0.9, 0.999, 1e-8
    opt = {"gd": ono_amd.GradientDescent(lr), "momentum": ono_amd.GradientDescentWithMomentum(lr, mu),
           "adam": ono_amd.Adam(lr, b1, b2, eps)}[kind]
    init = O.synth(nparams, SEED, 99)
    ref = O.Store(init, 1000, n, kind, lr=lr, momentum=mu, beta1=b1, beta2=b2, eps=eps)
    C = -(-nparams // n)
    shards = [dev(init[min(nparams, r * C):min(nparams, (r + 1) * C)].copy()) if r * C < nparams
              else torch.zeros(1, device="cuda") for r in range(n)]
    v = [torch.zeros(C, device="cuda") for _ in range(n)]
    s = [torch.zeros(C, device="cuda") for _ in range(n)]
    params = [torch.empty(nparams, device="cuda") for _ in range(n)]
    b1t = b2t = np.float32(1.0)
    for st in range(3):
        gs = [O.synth(nparams, SEED + 10 * st, w) for w in range(n)]
        grads = [dev(g) for g in gs]
        step = 0.0
        if kind == "adam":  # ono_ps_step's f32 host arithmetic (adam.rs:76-80)
            b1t, b2t = np.float32(b1t * np.float32(b1)), np.float32(b2t * np.float32(b2))
            step = float(np.float32(lr) * (np.sqrt(np.float32(1) - b2t) / (np.float32(1) - b1t)))
        P.run_local_ps(grads, params, shards, opt, step, v=v, s=s)
        torch.cuda.synchronize()
        for w in range(n):
            ref.accumulate(gs[w])
        ref.update_params()
        want = ref.pull_params()
        for r in range(n):
            assert_bitexact(params[r].cpu().numpy(), want, f"step {st} rank {r}")
            assert_bitexact(grads[r].cpu().numpy(), gs[r], "the workers' gradients must stay untouched")
