"""Per-parameter gradient error of the fused LeNet fp16 build vs the fp32 reference (debug)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import torch.nn.functional as F
from rocket_amd.models import LeNet
from rocket_amd.ops.lenet import lenet_forward

def _h(t): return t.to(torch.float16).float()
def _b(t): return t.to(torch.bfloat16).float()
def ref(x, net, q):
    h = q(F.max_pool2d(F.relu(F.conv2d(q(x), q(net.conv1.weight), net.conv1.bias, padding=2)), 2))
    h = F.max_pool2d(F.relu(F.conv2d(h, q(net.conv2.weight), net.conv2.bias)), 2)
    a2 = q(h.flatten(1))
    h1 = q(F.relu(F.linear(a2, q(net.fc1.weight), net.fc1.bias)))
    h2 = q(F.relu(F.linear(h1, q(net.fc2.weight), net.fc2.bias)))
    return F.linear(h2, q(net.fc3.weight), net.fc3.bias)
rel = lambda a, b: ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()
for dt, q in ((torch.float16, _h), (torch.bfloat16, _b)):
    for N in (64, 1024):
        torch.manual_seed(2)
        net = LeNet(fused=False).cuda(); r = LeNet(fused=False).cuda(); r.load_state_dict(net.state_dict())
        x = torch.rand(N, 1, 28, 28, device="cuda")
        with torch.autocast("cuda", dtype=dt):
            y = lenet_forward(x, net.conv1, net.conv2, net.fc1, net.fc2, net.fc3)
        yr = ref(x, r, q)
        g = torch.randn_like(y)
        y.backward(g); yr.backward(g)
        print(dt, N, "y", round(rel(y, yr), 5), {n: round(rel(p.grad, pr.grad), 4) for (n, p), pr in zip(net.named_parameters(), r.parameters())})
        print("   fc1.bias", net.fc1.bias.grad[:6].tolist(), r.fc1.bias.grad[:6].tolist())
