"""Run one GEMM engine on one shape a few times (PMC passes: rocprofv3 --pmc over this program).

    python bench/x5_one.py qkv x5 [reps]       engines: x5, x5:<shape code>, x4, lib
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench.gemm_r6_probe import SHAPES  # noqa: E402
from rocket_amd.ops import _lib  # noqa: E402

name, eng = sys.argv[1], sys.argv[2]
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
m, n, k = SHAPES[name]
dev = torch.device("cuda")
x = (torch.rand(m, k, device=dev) * 2 - 1).to(torch.bfloat16)
w = (torch.rand(n, k, device=dev) * 2 - 1).to(torch.bfloat16)
bias = torch.randn(n, device=dev)
y = torch.empty(m, n, dtype=torch.bfloat16, device=dev)
lib = _lib.kernels()
if eng.startswith("x5:"):  # x5:<rk_xgemm5_set_shape code>
    lib.rk_xgemm5_set_shape(int(eng[3:]))
    eng = "x5"
for _ in range(reps):
    if eng == "x5":
        lib.rk_xgemm5(x.data_ptr(), k, w.data_ptr(), k, y.data_ptr(), n, 1, bias.data_ptr(), m, n, k, _lib.stream_ptr(dev))
    elif eng == "x4":
        lib.rk_xgemm4_set_dbg(32)
        lib.rk_xgemm4(x.data_ptr(), k, w.data_ptr(), k, y.data_ptr(), n, 1, bias.data_ptr(), m, n, k, _lib.stream_ptr(dev))
    else:
        torch.addmm(bias.to(torch.bfloat16), x, w.t(), out=y)
torch.cuda.synchronize()
