import ctypes as C, os, sys
ROOT = os.getcwd()
sys.path[:0] = [ROOT, os.path.join(ROOT, "oxidized-neural-orchestra_amd")]
import numpy as np, torch, ono_amd
from ono_amd import kernels
L = ono_amd.lib()
torch.cuda.set_device(0)
sh = torch.cuda.current_stream().cuda_stream
for n in (16384, 54693, 1 << 25):
    g = torch.empty(n, dtype=torch.float32, device="cuda"); kernels.synth(g, 1, 0)
    m = min(n, 16384)
    st = C.c_uint64(3); idx = np.zeros(m, np.uint32)
    if n > 16384: L.ono_sparse_sample_default(C.byref(st), n, idx.ctypes.data, m)
    t = C.c_float(0)
    for _ in range(100):
        L.ono_sparse_threshold(C.byref(t), kernels.f32_ptr(g), n, idx.ctypes.data if n > 16384 else None, m, 0.1, sh)
    print(n, t.value)
