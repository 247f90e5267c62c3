"""Run one pipeline on either framework and dump what a user can observe (used by
``test_reference_diff.py``; runs in its own process).

    python _driver.py {reference|rocket_amd} {train|eval} OUT.json WORKDIR [REFERENCE_DIR]

Observables: the (capsule, event) trace, per-iteration loss/lr as published on
``attrs.looper.state``, the final parameters, and the checkpoint directory listing.
"""

import json
import os
import sys
import types


def _shim_reference(ref_dir):
    """The reference needs two tiny third-party packages that are not installed: ``adict``
    (attribute dict whose missing attributes read as None) and ``termcolor.colored``."""
    class adict(dict):
        def __getattr__(self, k):
            return self.get(k)

        def __setattr__(self, k, v):
            self[k] = v

        def __delattr__(self, k):
            self.pop(k, None)

    m = types.ModuleType("adict")
    m.adict = adict
    sys.modules["adict"] = m
    t = types.ModuleType("termcolor")
    t.colored = lambda text, *a, **k: text
    sys.modules["termcolor"] = t
    sys.path.insert(0, ref_dir)


def main():
    which, scenario, out, work = sys.argv[1:5]
    os.environ["ACCELERATE_USE_CPU"] = "1"
    import torch

    if which == "reference":
        _shim_reference(sys.argv[5])
        import rocket as fw
        from rocket.core.capsule import Capsule
    else:
        import rocket_amd as fw
        from rocket_amd.core.capsule import Capsule

    trace = []
    orig = Capsule.dispatch

    def spy(self, event, attrs=None):
        trace.append([type(self).__name__, event.value])
        return orig(self, event, attrs)

    Capsule.dispatch = spy

    torch.manual_seed(0)
    x, y = torch.randn(12, 4), torch.randint(0, 3, (12,))
    data = [(x[i], y[i]) for i in range(12)]

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.lin = torch.nn.Linear(4, 3)

        def forward(self, batch):
            return (batch[0], batch[1], self.lin(batch[0]))

    class Objective(torch.nn.Module):
        def forward(self, batch):
            return torch.nn.functional.cross_entropy(batch[2], batch[1])

    seen = []

    class Probe(Capsule):
        def __init__(self):
            super().__init__(priority=50)

        def launch(self, attrs=None):
            st = attrs.looper.state
            loss = st.loss
            lr = st.lr
            seen.append([None if loss is None else float(loss), None if lr is None else [float(v) for v in lr]])

    net = Net()
    opt = torch.optim.SGD(net.parameters(), lr=0.1)
    sched = torch.optim.lr_scheduler.StepLR(opt, 2, gamma=0.5)
    metrics = []
    if scenario == "train":
        loopers = [fw.Looper([fw.Dataset(data, batch_size=2),
                              fw.Module(net, [fw.Loss(Objective()), fw.Optimizer(opt), fw.Scheduler(sched)]),
                              fw.Checkpointer(save_every=4), Probe()])]
        kw = dict(num_epochs=2, gradient_accumulation_steps=2)
    else:
        class Acc(fw.Metric):
            def __init__(self):
                super().__init__()
                self.hits, self.n = 0, 0

            def launch(self, attrs=None):
                logits, target = attrs.batch[2], attrs.batch[1]
                self.hits += int((logits.argmax(1) == target).sum())
                self.n += int(target.shape[0])

            def reset(self, attrs=None):
                metrics.append([self.hits, self.n])
                self.hits, self.n = 0, 0

        ev = [(x[i] * 0.5, y[(i + 1) % 12]) for i in range(7)]
        loopers = [fw.Looper([fw.Dataset(data, batch_size=4, shuffle=False),
                              fw.Module(net, [fw.Loss(Objective()), fw.Optimizer(opt)]), Probe()]),
                   fw.Looper([fw.Dataset(ev, batch_size=2), fw.Module(net), fw.Meter([Acc()], keys=[1, 2])],
                             grad_enabled=False, run_every=2, tag="eval")]
        kw = dict(num_epochs=3)
    launcher = fw.Launcher(loopers, tag="diff", logging_dir=work, destroy_process_group_after_launch=False, **kw)
    error = None
    try:
        launcher.launch()
    except RuntimeError as e:  # reference quirk Q1: the default Checkpointer breaks destroy
        error = str(e)
    weights = os.path.join(work, "diff", "v0", "weights")
    ckpts = {d: sorted(os.listdir(os.path.join(weights, d))) for d in sorted(os.listdir(weights))} \
        if os.path.isdir(weights) else {}
    with open(out, "w") as fh:
        json.dump(dict(trace=trace, seen=seen, params=[p.detach().tolist() for p in net.parameters()],
                       ckpts=ckpts, metrics=metrics, error=error), fh)


if __name__ == "__main__":
    main()
