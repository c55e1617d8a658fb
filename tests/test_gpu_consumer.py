"""GPU parity of the all-reduce consumer: the fused
ParamManager::optimize + zero_grad + optimization_params copy of
worker/src/workers/all_reduce.rs:126-132, against the oracle's optimizers
(machine_learning/src/optimization/*.rs restated in oracle/)."""
import numpy as np
import pytest
import torch

import ono_amd
from conftest import SEED, assert_bitexact
from oracle import oracle as O
from oracle import oracle_np as N

pytestmark = pytest.mark.gpu

OPTS = {
    "gd": (ono_amd.GradientDescent(0.1), dict(lr=0.1)),
    "momentum": (ono_amd.GradientDescentWithMomentum(0.05, 0.9), dict(lr=0.05, momentum=0.9)),
    "adam": (ono_amd.Adam(0.01, 0.9, 0.999, 1e-8), dict(lr=0.01, beta1=0.9, beta2=0.999, eps=1e-8)),
}


@pytest.mark.parametrize("kind", ["gd", "momentum", "adam"])
@pytest.mark.parametrize("n", [1, 4099, (1 << 20) + 3])
def test_optimizer_consumer_vs_oracle(kind, n):
    spec, hp = OPTS[kind]
    params0 = O.synth(n, SEED, 11)
    ref = N.Optimizer(kind, n, **hp)
    w_ref = params0.copy()
    params = torch.from_numpy(params0.copy()).cuda()
    copy = torch.empty_like(params)
    opt = ono_amd.DeviceOptimizer(spec, n)
    for rnd in range(5):
        g = O.synth(n, SEED + rnd, 3)   # includes signed zeros: no +0 canonicalisation here
        grad = torch.from_numpy(g).cuda()
        pm = ono_amd.ParamManager(params, grad, None)
        pm.optimize(opt, params_copy=copy)
        ref.update(g.copy(), w_ref)
        torch.cuda.synchronize()
        assert_bitexact(params.cpu().numpy(), w_ref, f"{kind} round {rnd}")
        assert_bitexact(copy.cpu().numpy(), w_ref, "optimization_params copy")
        assert not grad.cpu().numpy().view(np.uint32).any(), "zero_grad"
    opt.close()


def test_optimizer_consumer_size_mismatch():
    opt = ono_amd.DeviceOptimizer(ono_amd.GradientDescent(0.1), 10)
    p = torch.zeros(11, device="cuda")
    with pytest.raises(ono_amd.SizeMismatch):
        opt.step(p, torch.zeros(11, device="cuda"))
    opt.close()


def test_worker_round_end_to_end():
    """One AllReduceWorker round on the device, n = 1 (all_reduce.rs:114-132):
    acc_residual per batch -> pull_grads -> optimize + zero_grad + copy."""
    n = 100003
    ring = ono_amd.WorkerRingManager(0, 1, n)
    params = torch.from_numpy(O.synth(n, SEED, 5)).cuda()
    opt_params = params.clone()
    opt = ono_amd.DeviceOptimizer(ono_amd.GradientDescent(0.1), n)
    batches = [O.synth(n, SEED + b, 9) for b in range(3)]
    for b in batches:
        ring.acc_residual(torch.from_numpy(b).cuda())
    pm = ring.pull_grads(params)
    pm.optimize(opt, params_copy=opt_params)
    torch.cuda.synchronize()
    res = np.zeros(n, np.float32)
    for b in batches:
        res = (res + b).astype(np.float32)
    w = O.synth(n, SEED, 5)
    N.Optimizer("gd", n, lr=0.1).update(res, w)
    assert_bitexact(params.cpu().numpy(), w)
    assert_bitexact(opt_params.cpu().numpy(), w)
    assert not ring.grad.cpu().numpy().view(np.uint32).any()
    assert not ring.residual.cpu().numpy().view(np.uint32).any()
    opt.close()
    ring.close()
