"""EngineScheduler under the fp16 device-resident scaler.

Default (exact form): a skipped step never advances the schedule, as in accelerate
(``accelerate@1.14.0:scheduler.py:54-83``; reference ``rocket/core/scheduler.py:94-113``); a step
whose skip flag has not landed is taken provisionally only when it leaves the hyperparameters
unchanged (then no update can see the difference), else the flag is waited for.
Opt-in speculation (ROCKET_SCHED_SPECULATE=1, runtime/engine.py EngineScheduler.SPECULATE): the
scheduler steps when the step's skip flag has not landed yet and a mispredicted (skipped) step is
rolled back when the flag is read; checkpoints settle the speculation first."""

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
    sch.SPECULATE = True

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


def test_exact_form_is_the_default():
    assert EngineScheduler.SPECULATE is False


def _run_lrs(skips, speculate):
    """lr seen by every update of a run whose steps ``skips`` flags as inf/NaN-skipped."""
    p = torch.nn.Parameter(torch.zeros(2))
    opt = torch.optim.SGD([p], lr=1.0)
    eo = EngineOptimizer(opt, _Eng())
    sch = EngineScheduler(torch.optim.lr_scheduler.StepLR(opt, step_size=1, gamma=0.5), [eo], _Eng())
    sch.SPECULATE = speculate
    seen = []
    for sk in skips:
        seen.append(opt.param_groups[0]["lr"])  # the lr this update runs with
        eo._skip_lazy, eo._lazy_handle = True, _flag(sk)
        sch.step()
    sch.get_last_lr()
    return seen, opt.param_groups[0]["lr"]


def test_exact_lr_sequence_matches_accelerate_with_skipped_steps():
    skips = [True, True, False, True, False, False, True, False]
    # accelerate: the scheduler steps only after a non-skipped optimizer step
    lr, want = 1.0, []
    for sk in skips:
        want.append(lr)
        if not sk:
            lr *= 0.5
    seen, final = _run_lrs(skips, speculate=False)
    assert seen == want and final == lr
    # the speculative form differs exactly on the update that follows a skipped step
    seen_spec, final_spec = _run_lrs(skips, speculate=True)
    assert final_spec == lr and seen_spec != want


def test_checkpoint_settles_a_mispredicted_speculation(tmp_path):
    from rocket_amd.runtime import checkpoint_io

    p = torch.nn.Parameter(torch.zeros(2))
    opt = torch.optim.SGD([p], lr=1.0)

    class _E(_Eng):
        _models, _custom_objects, step, process_index = [], [], 0, 0

    eng = _E()
    eo = EngineOptimizer(opt, eng)
    sch = EngineScheduler(torch.optim.lr_scheduler.StepLR(opt, step_size=1, gamma=0.5), [eo], eng)
    sch.SPECULATE = True
    eng._optimizers, eng._schedulers = [eo], [sch]
    eo._skip_lazy, eo._lazy_handle = True, _flag(True)
    sch.step()  # speculated; the step was in fact skipped
    assert opt.param_groups[0]["lr"] == 0.5
    checkpoint_io.save_state(eng, str(tmp_path / "ck"))
    osd = torch.load(tmp_path / "ck" / "optimizer.bin", weights_only=True)
    ssd = torch.load(tmp_path / "ck" / "scheduler.bin", weights_only=True)
    assert osd["param_groups"][0]["lr"] == 1.0 and ssd["last_epoch"] == 0

    # and the optimizer's own state_dict settles it too
    eo._skip_lazy, eo._lazy_handle = True, _flag(True)
    sch.step()
    assert eo.state_dict()["param_groups"][0]["lr"] == 1.0


def test_exact_form_defers_hyperparameter_neutral_steps():
    """StepLR(step_size=3): steps that do not cross a milestone leave lr unchanged, so the exact form
    takes them without waiting for the flag; the milestone step waits.  The lr sequence still
    equals accelerate's, including across skipped steps."""
    skips = [False, True, False, False, True, False, False, False, True, False]

    def run():
        p = torch.nn.Parameter(torch.zeros(2))
        opt = torch.optim.SGD([p], lr=1.0)
        eo = EngineOptimizer(opt, _Eng())
        sch = EngineScheduler(torch.optim.lr_scheduler.StepLR(opt, step_size=3, gamma=0.5), [eo], _Eng())
        seen = []
        for sk in skips:
            seen.append(opt.param_groups[0]["lr"])
            eo._skip_lazy, eo._lazy_handle = True, _flag(sk)
            sch.step()
        sch.get_last_lr()
        return seen, opt.param_groups[0]["lr"], sch

    lr, n, want = 1.0, 0, []
    for sk in skips:
        want.append(lr)
        if not sk:
            n += 1
            if n % 3 == 0:
                lr *= 0.5
    seen, final, sch = run()
    assert seen == want and final == lr
    assert sch.provisional >= 5  # the non-milestone steps never waited
    assert sch.mispredicted >= 1  # and the skipped ones among them were rolled back


def test_steplr_fast_path_matches_torch():
    """EngineScheduler's StepLR fast path (between milestones) leaves exactly torch's state."""
    import copy

    def make():
        p = torch.nn.Parameter(torch.zeros(2))
        opt = torch.optim.SGD([p], lr=1.0)
        opt.step()
        return opt, torch.optim.lr_scheduler.StepLR(opt, step_size=3, gamma=0.5)

    opt_a, ref = make()
    opt_b, s = make()
    sch = EngineScheduler(s, [EngineOptimizer(opt_b, _Eng())], _Eng())
    for _ in range(10):
        ref.step()
        sch.step()
        assert opt_a.param_groups[0]["lr"] == opt_b.param_groups[0]["lr"]
        assert ref.state_dict() == s.state_dict()
    assert copy.deepcopy(s.get_last_lr()) == ref.get_last_lr()


def test_light_provisional_step_rolls_back_exactly():
    """Between StepLR milestones the provisional step keeps a three-field snapshot (no
    state_dict); a skipped step restores exactly the state of a scheduler that never took it."""
    p = torch.nn.Parameter(torch.zeros(2))
    opt = torch.optim.SGD([p], lr=1.0)
    eo = EngineOptimizer(opt, _Eng())
    sch = EngineScheduler(torch.optim.lr_scheduler.StepLR(opt, step_size=10, gamma=0.5), [eo], _Eng())
    sch.LIGHT = True
    ref_opt = torch.optim.SGD([torch.nn.Parameter(torch.zeros(2))], lr=1.0)
    ref = torch.optim.lr_scheduler.StepLR(ref_opt, step_size=10, gamma=0.5)
    skips = [False, False, True, False, True, True, False, False, False, False, False, False, True, False]
    for i, sk in enumerate(skips):
        eo._skip_lazy, eo._lazy_handle = True, _flag(sk)
        sch.step()
        if i + 1 < len(skips) and 1 < sch.scheduler._step_count and (sch.scheduler.last_epoch % 10):
            assert sch._pending is None or sch._pending[1][0] in ("light", "full")
        if not sk:
            ref_opt.step()
            ref.step()
    sch._resolve()
    assert sch.scheduler.last_epoch == ref.last_epoch
    assert sch.scheduler._step_count == ref._step_count
    assert sch.scheduler.get_last_lr() == ref.get_last_lr()
    assert opt.param_groups[0]["lr"] == ref_opt.param_groups[0]["lr"]
    assert sch.provisional > 0


class _LagFlags:
    """A skip flag that lands ``lag`` scheduler steps after its update (the device running behind
    the host); reading it before then waits (counted)."""

    clock = [0]
    waits = [0]

    def __init__(self, skipped: bool, lag: int):
        self.skipped, self.at = skipped, _LagFlags.clock[0] + lag

    def _entry(self, seq):
        return self.skipped if _LagFlags.clock[0] >= self.at else None

    def _resolve(self, seq):
        if _LagFlags.clock[0] < self.at:
            _LagFlags.waits[0] += 1
        return self.skipped


def test_queued_provisional_steps_with_lagging_flags_match_accelerate():
    """Exact form with the device several steps behind: provisional steps queue up (no wait per
    step), flags settle in order as they land, a skipped one is undone and the later ones re-taken;
    the lr every update runs with and the final scheduler state equal accelerate's, and only the
    milestone steps wait."""
    for light in (False, True):
        skips = [False, True, False, False, True, True, False, False, False, True, False, False, False, True,
                 False, False, False, False, True, False, False, False, False, False, False]
        p = torch.nn.Parameter(torch.zeros(2))
        opt = torch.optim.SGD([p], lr=1.0)
        eo = EngineOptimizer(opt, _Eng())
        sch = EngineScheduler(torch.optim.lr_scheduler.StepLR(opt, step_size=4, gamma=0.5), [eo], _Eng())
        sch.LIGHT = light
        ref_opt = torch.optim.SGD([torch.nn.Parameter(torch.zeros(2))], lr=1.0)
        ref = torch.optim.lr_scheduler.StepLR(ref_opt, step_size=4, gamma=0.5)
        _LagFlags.clock[0], _LagFlags.waits[0] = 0, 0
        seen, want = [], []
        for sk in skips:
            seen.append(opt.param_groups[0]["lr"])
            want.append(ref_opt.param_groups[0]["lr"])
            eo._skip_lazy, eo._lazy_handle = True, (_LagFlags(sk, lag=3), 1)
            milestone = (sch.scheduler.last_epoch + 1) % 4 == 0  # this step would change the lr
            w0 = _LagFlags.waits[0]
            sch.step()
            assert milestone or _LagFlags.waits[0] == w0  # only a milestone step waits for flags
            _LagFlags.clock[0] += 1
            if not sk:
                ref_opt.step()
                ref.step()
            assert len(sch._queue) <= sch.MAXQ
        sch._resolve()
        assert seen == want
        assert sch.scheduler.last_epoch == ref.last_epoch and sch.scheduler._step_count == ref._step_count
        assert sch.scheduler.get_last_lr() == ref.get_last_lr()
        assert opt.param_groups[0]["lr"] == ref_opt.param_groups[0]["lr"]
        assert sch.mispredicted >= 3 and sch.provisional >= 10


class _RingScaler:
    """FusedGradScaler's flag ring (runtime/amp.py): update ``seq``'s flag is readable from the time the
    device publishes it until RING later updates have overwritten its slot; ``_resolve`` waits for the
    device and, for an overwritten slot, falls back to the LATEST update's flag (the real fallback)."""

    def __init__(self):
        from rocket_amd.runtime.amp import RING

        self.ring = RING
        self._seq = 0  # updates launched
        self.published = 0  # updates the device has finished
        self.flags = {}
        self.syncs = 0

    def launch(self, skipped: bool):
        self._seq += 1
        self.flags[self._seq] = skipped
        self.published = self._seq - 1  # the device runs one update behind the host

    def _entry(self, seq):
        if seq > self.published or self.published - seq >= self.ring:
            return None
        return self.flags[seq]

    def _resolve(self, seq):
        f = self._entry(seq)
        if f is not None:
            return f
        self.syncs += 1
        self.published = self._seq
        f = self._entry(seq)
        return f if f is not None else self.flags[self._seq]


def test_per_epoch_scheduler_never_reads_an_overwritten_flag():
    """a scheduler stepped once per epoch (100 updates per step) must not queue provisional
    steps whose flags leave the 64-update ring before they are read: the lr sequence equals
    accelerate's although every epoch's LAST update (the one the scheduler step follows) alternates
    between kept and skipped."""
    p = torch.nn.Parameter(torch.zeros(2))
    opt = torch.optim.SGD([p], lr=1.0)
    eo = EngineOptimizer(opt, _Eng())
    sch = EngineScheduler(torch.optim.lr_scheduler.StepLR(opt, step_size=3, gamma=0.5), [eo], _Eng())
    ref_opt = torch.optim.SGD([torch.nn.Parameter(torch.zeros(2))], lr=1.0)
    ref = torch.optim.lr_scheduler.StepLR(ref_opt, step_size=3, gamma=0.5)
    sc = _RingScaler()
    last_skipped = [False, True, False, False, True, False, True, True, False, False, False, True]
    for epoch, sk in enumerate(last_skipped):
        for i in range(100):
            sc.launch(sk if i == 99 else False)
        eo._skip_lazy, eo._lazy_handle = True, (sc, sc._seq)
        sch.step()
        if not sk:
            ref.step()
        assert opt.param_groups[0]["lr"] == ref_opt.param_groups[0]["lr"], epoch
        assert len(sch._queue) <= 1
    sch._resolve()
    assert sch.scheduler.last_epoch == ref.last_epoch and sch.scheduler.get_last_lr() == ref.get_last_lr()


def test_fast_cadence_settles_a_step_before_its_flag_ages_out():
    """Per-iteration cadence with the device far behind: a queued step whose flag would be overwritten
    before the next scheduler step is settled (waited for) instead of left to the stale fallback."""
    p = torch.nn.Parameter(torch.zeros(2))
    opt = torch.optim.SGD([p], lr=1.0)
    eo = EngineOptimizer(opt, _Eng())
    sch = EngineScheduler(torch.optim.lr_scheduler.StepLR(opt, step_size=1000, gamma=0.5), [eo], _Eng())
    sch.MAXQ = 32
    sc = _RingScaler()
    for it in range(200):
        for _ in range(3):  # three updates per scheduler step (e.g. three optimizers' worth)
            sc.launch(False)
        sc.published = max(0, sc._seq - 60)  # the device lags 60 updates: flags land late
        eo._skip_lazy, eo._lazy_handle = True, (sc, sc._seq)
        sch.step()
        for h, _ in sch._queue:
            assert sc._seq - h[0][1] < sc.ring  # every queued flag is still in the ring
    sch._resolve()
    assert sch.scheduler.last_epoch == 200 and sch.mispredicted == 0
