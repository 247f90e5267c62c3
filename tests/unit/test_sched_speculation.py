"""EngineScheduler under the fp16 device-resident scaler: the scheduler steps speculatively when
the step's skip flag has not landed yet, and a mispredicted (skipped) step is rolled back when the
flag is read (runtime/engine.py EngineScheduler.SPECULATE)."""

import torch

from rocket_amd.runtime.engine import EngineOptimizer, EngineScheduler


class _Flags:
    """Stands in for FusedGradScaler's published skip flags (handle = (scaler, update number))."""

    def __init__(self, skipped: bool):
        self.skipped = skipped
        self.done = False  # published yet

    def _entry(self, seq):
        return self.skipped if self.done else None

    def _resolve(self, seq):
        self.done = True  # (the real one waits for the update)
        return self.skipped


class _Eng:
    sync_gradients = True
    num_processes = 1
    scaler = None


def _flag(skipped: bool):
    return (_Flags(skipped), 1)


def test_speculated_step_kept_and_mispredicted_step_rolled_back():
    p = torch.nn.Parameter(torch.zeros(2))
    opt = torch.optim.SGD([p], lr=1.0, momentum=0.9)
    eo = EngineOptimizer(opt, _Eng())
    sch = EngineScheduler(torch.optim.lr_scheduler.StepLR(opt, step_size=1, gamma=0.5), [eo], _Eng())

    eo._skip_lazy, eo._lazy_handle = True, _flag(False)
    sch.step()  # flag not landed: speculate
    assert opt.param_groups[0]["lr"] == 0.5 and sch._pending is not None

    eo._skip_lazy, eo._lazy_handle = True, _flag(True)
    sch.step()  # resolves step 1 (kept), speculates step 2
    assert opt.param_groups[0]["lr"] == 0.25 and sch.mispredicted == 0

    assert sch.get_last_lr() == [0.5]  # step 2 was skipped: rolled back on the read
    assert opt.param_groups[0]["lr"] == 0.5 and sch.mispredicted == 1
    assert sch.scheduler.last_epoch == 1


def test_landed_flag_takes_the_exact_path():
    p = torch.nn.Parameter(torch.zeros(2))
    opt = torch.optim.SGD([p], lr=1.0)
    eo = EngineOptimizer(opt, _Eng())
    sch = EngineScheduler(torch.optim.lr_scheduler.StepLR(opt, step_size=1, gamma=0.5), [eo], _Eng())
    h = _flag(True)
    h[0].done = True
    eo._skip_lazy, eo._lazy_handle = True, h
    sch.step()  # flag available: the skipped step does not advance the schedule
    assert opt.param_groups[0]["lr"] == 1.0 and sch._pending is None
