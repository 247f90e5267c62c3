"""Diagnostic: is the fused LeNet backward's conv-gradient slab bitwise repeatable?
Runs rk_lenet_bwd repeatedly on identical inputs and reports differing slab rows/columns."""
import ctypes
import sys

import torch

from rocket_amd.models import LeNet
from rocket_amd.ops import _lib
from rocket_amd.ops.lenet import lenet_forward

lib = _lib.kernels()
W = int(lib.rk_lenet_slab_width())
for N in (256, 1024, 64, 512):
    torch.manual_seed(5)
    net = LeNet(fused=False).cuda()
    x = torch.rand(N, 1, 28, 28, device="cuda")
    g = torch.randn(N, 10, device="cuda")
    y = lenet_forward(x, net.conv1, net.conv2, net.fc1, net.fc2, net.fc3)
    xs, a1, c1, c2, a2T, h1T, h2T, frag, w2c, logits = y.grad_fn.saved_tensors
    bf = dict(dtype=torch.bfloat16, device="cuda")
    outs = []
    for rep in range(40):
        dyT, d2T, d1T = torch.empty(10, N, **bf), torch.empty(84, N, **bf), torch.empty(120, N, **bf)
        slab = torch.full((N // 4, W), float("nan"), device="cuda")
        _lib.check(lib.rk_lenet_bwd(xs.data_ptr(), a1.data_ptr(), c1.data_ptr(), c2.data_ptr(), w2c.data_ptr(),
                                    frag.data_ptr(), g.data_ptr(), h1T.data_ptr(), h2T.data_ptr(), dyT.data_ptr(),
                                    d2T.data_ptr(), d1T.data_ptr(), slab.data_ptr(), N, 1, None,
                                    _lib.stream_ptr(x.device)), "bwd")
        outs.append((slab.clone(), dyT.clone(), d2T.clone(), d1T.clone()))
    torch.cuda.synchronize()
    cols = int(lib.rk_lenet_slab_cols())
    ref = outs[0]
    nbad = 0
    for i, o in enumerate(outs[1:], 1):
        s0, s1 = ref[0][:, :cols], o[0][:, :cols]
        same = (s0 == s1) | (s0.isnan() & s1.isnan())
        if not bool(same.all()):
            nbad += 1
            bad = (~same).nonzero()
            print(f"N={N} rep{i}: slab differs at {bad.shape[0]} entries; rows {sorted(set(bad[:, 0].tolist()))[:10]} "
                  f"cols {sorted(set(bad[:, 1].tolist()))[:20]} max {float((s0 - s1).abs().nan_to_num(1e9).max())}")
        for k, nm in ((1, "dyT"), (2, "d2T"), (3, "d1T")):
            if not torch.equal(ref[k], o[k]):
                print(f"N={N} rep{i}: {nm} differs")
    print(f"N={N}: {nbad}/39 runs differ; nan in slab cols: {int(ref[0][:, :cols].isnan().sum())}", flush=True)


# part 2: forward + full backward repeated, as the test does
names = ["x", "a1", "c1", "c2", "a2T", "h1T", "h2T", "frag", "w2c", "logits"]
for N in (1024, 256):
    torch.manual_seed(5)
    net = LeNet(fused=False).cuda()
    x = torch.rand(N, 1, 28, 28, device="cuda")
    g = torch.randn(N, 10, device="cuda")
    ref = None
    for rep in range(30):
        net.zero_grad(set_to_none=True)
        y = lenet_forward(x, net.conv1, net.conv2, net.fc1, net.fc2, net.fc3)
        saved = [t.clone() for t in y.grad_fn.saved_tensors]
        y.backward(g)
        grads = [p.grad.clone() for p in net.parameters()]
        if ref is None:
            ref = (saved, grads)
            continue
        for nm, a, b in zip(names, ref[0], saved):
            if not torch.equal(a, b):
                d = (a != b).nonzero()
                print(f"N={N} rep{rep}: saved {nm} differs at {d.shape[0]} entries, first {d[:4].tolist()}")
        for (nm, _), a, b in zip(net.named_parameters(), ref[1], grads):
            if not torch.equal(a, b):
                print(f"N={N} rep{rep}: grad {nm} differs max {float((a - b).abs().max())}")
    print(f"N={N} part2 done", flush=True)
