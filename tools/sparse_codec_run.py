"""K drops + K device lifts of the bench's sparse workload (64 MiB gradient, 90th
percentile threshold), K times — a short program for rocprofv3 kernel stats."""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oxidized-neural-orchestra_amd"))
import ono_amd  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
n = 16 << 20
g = ono_amd.kernels.synth(torch.empty(n, dtype=torch.float32, device="cuda"), 1234, 7)
t = float(torch.quantile(g[: 1 << 20].abs().float(), 0.9).item())
L = ono_amd.lib()
import time  # noqa: E402
wire = ono_amd.sparse.grad_drop_dev(g, t)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(K):
    wire = ono_amd.sparse.grad_drop_dev(g, t)
print(f"drop {(time.perf_counter() - t0) / K * 1e6:.1f} us per blocking call")
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
for _ in range(K):
    wire = ono_amd.sparse.grad_drop_dev(g, t)
ev1.record()
torch.cuda.synchronize()
print(f"drop {ev0.elapsed_time(ev1) / K * 1e3:.1f} us per call between events on the stream")
buf = torch.empty(L.ono_sparse_max_bytes(n), dtype=torch.uint8, device="cuda")
nbd = torch.zeros(1, dtype=torch.int64, device="cuda")
ev0.record()
for _ in range(K):
    ono_amd.sparse.grad_drop_async(g, t, buf, nbd)
ev1.record()
torch.cuda.synchronize()
print(f"drop {ev0.elapsed_time(ev1) / K * 1e3:.1f} us per stream-ordered drop, back to back")
assert int(nbd.item()) == wire.numel() and torch.equal(buf[: wire.numel()], wire)
# the same, over 6 different gradients in turn (384 MiB > the 256 MiB Infinity Cache): every drop
# reads its gradient from HBM, as a fresh bucket would be
G = [ono_amd.kernels.synth(torch.empty(n, dtype=torch.float32, device="cuda"), 1234 + j, 7) for j in range(6)]
T = [float(torch.quantile(x[: 1 << 20].abs().float(), 0.9).item()) for x in G]
for j in range(6):
    ono_amd.sparse.grad_drop_async(G[j], T[j], buf, nbd)
torch.cuda.synchronize()
ev0.record()
for i in range(K):
    ono_amd.sparse.grad_drop_async(G[i % 6], T[i % 6], buf, nbd)
ev1.record()
torch.cuda.synchronize()
print(f"drop {ev0.elapsed_time(ev1) / K * 1e3:.1f} us per stream-ordered drop, back to back, 6 rotating gradients")
del G
out = torch.empty(n, dtype=torch.float32, device="cuda")
ln = C.c_size_t(0)
s = torch.cuda.current_stream().cuda_stream
KL = K if not os.environ.get("ONO_SP_VARIANT") else 0  # variants write garbage
ono_amd._lib.call("ono_sparse_lift_dev", out.data_ptr(), n, C.byref(ln), wire.data_ptr(), wire.numel(), s)
torch.cuda.synchronize()
t0 = time.perf_counter()
ev0.record()
for _ in range(KL):
    ono_amd._lib.call("ono_sparse_lift_dev", out.data_ptr(), n, C.byref(ln), wire.data_ptr(), wire.numel(), s)
ev1.record()
torch.cuda.synchronize()
if KL:
    print(f"lift_dev {(time.perf_counter() - t0) / KL * 1e6:.1f} us per blocking call, "
          f"{ev0.elapsed_time(ev1) / KL * 1e3:.1f} us between events")
    ref = ono_amd.sparse.grad_lift(bytes(wire.cpu().numpy()), n)
    print("lift_dev equals the host-stream lift:", bool(torch.equal(out.view(torch.int32), ref.view(torch.int32))))
if KL:  # stream-ordered lifts back to back (ono_sparse_lift_dev_async): the device's own time per lift
    st = torch.zeros(1, dtype=torch.int64, device="cuda")
    for _ in range(3):
        ono_amd.sparse.grad_lift_dev_async(wire, out, st)
    torch.cuda.synchronize()
    ev0.record()
    tks = [ono_amd.sparse.grad_lift_dev_async(wire, out, st) for _ in range(KL)]
    ev1.record()
    torch.cuda.synchronize()
    print(f"lift_dev {ev0.elapsed_time(ev1) / KL * 1e3:.1f} us per stream-ordered lift, back to back "
          f"(refused: {int(st.item()) in tks})")
print("lift fallbacks", L.ono_sparse_lift_fallbacks(), "wire", wire.numel())
# the config-1 chunk (54,693 values, 27 tiles: the one-launch encoder sp_drop1) K times, stream-ordered
gc = ono_amd.kernels.synth(torch.empty(54_693, dtype=torch.float32, device="cuda"), 99, 7)
tc = float(torch.quantile(gc.abs().float(), 0.9).item())
bc = torch.empty(L.ono_sparse_max_bytes(gc.numel()), dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
ev0.record()
for _ in range(K):
    ono_amd.sparse.grad_drop_async(gc, tc, bc, nbd)
ev1.record()
torch.cuda.synchronize()
print(f"drop (config-1 chunk) {ev0.elapsed_time(ev1) / K * 1e3:.1f} us per stream-ordered drop")
