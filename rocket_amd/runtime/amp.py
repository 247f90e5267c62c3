"""Device-resident fp16 dynamic loss scaling (the GradScaler that accelerate's fp16
mode wraps around ``optimizer.step``, reference ``rocket/core/optimizer.py:128-130``).

``torch.amp.GradScaler`` costs, per step: a ``_amp_foreach_non_finite_check_and_unscale_`` launch
over every gradient, a host read of ``found_inf`` (to decide whether to call ``step``), an
``_amp_update_scale_`` launch, and accelerate adds a ``get_scale()`` host read before and after.

:class:`FusedGradScaler` keeps the whole state on the device (``native/kernels/optim_common.h``
``AmpSlot`` layout: scale, 1/scale, found flag, growth tracker, growth / backoff factors,
interval, last found flag) and, for the fused multi-tensor optimizers, turns a scaled step into
two launches with no host synchronisation:

1. ``rk_amp_check`` flags any non-finite gradient;
2. ``rk_optim_mt`` unscales inside the update (gradient × 1/scale), skips the whole update —
   step counter included — when the flag is set, and its last block applies the growth/backoff
   rule of ``torch._amp_update_scale_`` and clears the flag.

Whether a step was skipped is only needed by the LR scheduler wrapper (accelerate does not step
the scheduler after a skipped optimizer step); that value is copied to pinned memory behind the
update and read lazily.  The two launches are graph-capturable (``step_device``): fp16 steps are
captured like bf16 ones, the flag copy being enqueued after each replay.  Optimizers that are not fused fall back to the torch primitives on the
same device state.  ``state_dict`` uses ``torch.amp.GradScaler``'s format (``scaler.pt``
checkpoints are interchangeable).
"""

from __future__ import annotations

from typing import Optional

import torch

SCALE, INV, FOUND, TRACKER, GROWTH, BACKOFF, INTERVAL, LAST = range(8)


class FusedGradScaler:
    def __init__(self, device, init_scale: float = 2.0 ** 16, growth_factor: float = 2.0,
                 backoff_factor: float = 0.5, growth_interval: int = 2000, enabled: bool = True):
        self.device = torch.device(device)
        self._enabled = enabled
        self._growth_factor = float(growth_factor)
        self._backoff_factor = float(backoff_factor)
        self._growth_interval = int(growth_interval)
        self.state = torch.tensor([init_scale, 1.0 / init_scale, 0.0, 0.0, growth_factor, backoff_factor,
                                   float(growth_interval), 0.0], dtype=torch.float32, device=self.device)
        # the skip flag of recent steps: a small ring of pinned copies + their events, so a caller can
        # hold the handle of step k while step k+1 records its own (EngineScheduler speculation)
        pin = self.device.type == "cuda"
        self._ring = [torch.zeros(1, dtype=torch.float32, pin_memory=pin) for _ in range(4)]
        self._ring_ev = [torch.cuda.Event() for _ in range(4)] if pin else [None] * 4  # reused: no per-step event
        self._ring_i = 0
        self._last_host = self._ring[0]
        self._last_event = None
        self._unscaled = set()  # id(optimizer) unscaled this step (clip_grad_norm_ path)

    # ------------------------------------------------------------------ API
    def is_enabled(self) -> bool:
        return self._enabled

    def scale(self, outputs):
        if not self._enabled:
            return outputs
        if isinstance(outputs, torch.Tensor):
            # the fp32 0-dim scale promotes a 0-dim fp16 loss to fp32 (as torch's GradScaler):
            # 65536 cast to fp16 would be inf and skip every growth step
            return outputs * self.state[SCALE]
        return type(outputs)(self.scale(o) for o in outputs)

    def _grads(self, optimizer):
        return [p.grad for g in optimizer.param_groups for p in g["params"] if p.grad is not None]

    def unscale_(self, optimizer) -> None:
        """Unscale the gradients in place now (before clipping); the step then uses scale 1."""
        if not self._enabled or id(optimizer) in self._unscaled:
            return
        grads = self._grads(optimizer)
        if grads:
            found = self.state[FOUND : FOUND + 1]
            torch._amp_foreach_non_finite_check_and_unscale_(grads, found, self.state[INV : INV + 1])
        self._unscaled.add(id(optimizer))

    def step(self, optimizer, *args, zero_grads: bool = False, **kwargs):
        """Scaled optimizer step.  Fused optimizers: two launches, no host read; others: torch's
        unscale + one host read of the flag + the scale update."""
        if not self._enabled:
            return optimizer.step(*args, **kwargs)
        from rocket_amd.ops.optim import _FusedBase

        unscaled = id(optimizer) in self._unscaled
        if isinstance(optimizer, _FusedBase) and not args and not kwargs:
            if not optimizer.prepare():
                # no gradient to update: torch.amp.GradScaler.step asserts here ("No inf checks
                # were recorded for this optimizer") without touching the scale or the growth
                # tracker; same here, after dropping this step's unscaled mark
                self._unscaled.discard(id(optimizer))
                raise AssertionError("No inf checks were recorded for this optimizer.")
            if not unscaled:
                optimizer.amp_check(self.state)
            else:  # unscaled in place (and checked) already: unscale by 1 this time; the last
                self.state[INV] = 1.0  # block restores 1/scale with the scale update
            optimizer.amp = self.state
            try:
                optimizer.launch(zero_grads=zero_grads)
            finally:
                optimizer.amp = None
            self._record_last()
            return None
        # generic optimizer: torch's primitives on the device state, one host read of the flag
        if not unscaled:
            self.unscale_(optimizer)
        skip = bool(self.state[FOUND].item())
        out = None if skip else optimizer.step(*args, **kwargs)
        self._update_host_side()
        self._record_last()
        return out

    def step_device(self, optimizer, zero_grads: bool = False) -> None:
        """The device part of a fused scaled step (flag check + update with in-kernel unscale and
        scale rule): graph-capturable; ``record_last`` after the replay publishes the skip flag."""
        if id(optimizer) not in self._unscaled:
            optimizer.amp_check(self.state)
        else:
            self.state[INV] = 1.0
        optimizer.amp = self.state
        try:
            optimizer.launch(zero_grads=zero_grads)
        finally:
            optimizer.amp = None
        self._unscaled.clear()

    def record_last(self) -> None:
        self._record_last()

    def _update_host_side(self) -> None:
        """The scale update for a step that did not run through the fused optimizer kernel."""
        scale = self.state[SCALE : SCALE + 1]
        tracker = torch.zeros(1, dtype=torch.int32, device=self.device)
        tracker.copy_(self.state[TRACKER : TRACKER + 1])
        found = self.state[FOUND : FOUND + 1]
        torch._amp_update_scale_(scale, tracker, found, self._growth_factor, self._backoff_factor,
                                 self._growth_interval)
        self.state[TRACKER : TRACKER + 1].copy_(tracker)
        self.state[INV] = 1.0 / self.state[SCALE]
        self.state[LAST] = self.state[FOUND]
        self.state[FOUND] = 0.0

    def _record_last(self) -> None:
        self._unscaled.clear()
        self._ring_i = (self._ring_i + 1) % len(self._ring)
        self._last_host = self._ring[self._ring_i]
        self._last_host.copy_(self.state[LAST : LAST + 1], non_blocking=True)
        self._last_event = self._ring_ev[self._ring_i]
        if self._last_event is not None:
            self._last_event.record()

    def last_handle(self):
        """(pinned flag copy, event) of the last recorded step: resolve with :func:`handle_skipped`."""
        return (self._last_host, self._last_event)

    @staticmethod
    def handle_ready(h) -> bool:
        return h[1] is None or h[1].query()

    @staticmethod
    def handle_skipped(h) -> bool:
        if h[1] is not None:
            h[1].synchronize()
        return bool(h[0][0] != 0)

    def update(self, new_scale=None) -> None:
        """The scale update already ran on the device; ``new_scale`` overrides it."""
        if new_scale is not None:
            v = float(new_scale)
            self.state[SCALE] = v
            self.state[INV] = 1.0 / v

    def last_step_skipped(self) -> bool:
        """Whether the last scaled step found inf/NaN gradients (waits for that step only)."""
        if self._last_event is not None:
            self._last_event.synchronize()
        return bool(self._last_host[0] != 0)

    def get_scale(self) -> float:
        return float(self.state[SCALE].item()) if self._enabled else 1.0

    def get_growth_factor(self) -> float:
        return self._growth_factor

    def get_backoff_factor(self) -> float:
        return self._backoff_factor

    def get_growth_interval(self) -> int:
        return self._growth_interval

    # ------------------------------------------------------------ checkpoint
    def state_dict(self) -> dict:
        if not self._enabled:
            return {}
        return {"scale": self.get_scale(), "growth_factor": self._growth_factor,
                "backoff_factor": self._backoff_factor, "growth_interval": self._growth_interval,
                "_growth_tracker": int(self.state[TRACKER].item())}

    def load_state_dict(self, sd: dict) -> None:
        if not sd:
            return
        self._growth_factor = float(sd["growth_factor"])
        self._backoff_factor = float(sd["backoff_factor"])
        self._growth_interval = int(sd["growth_interval"])
        s = float(sd["scale"])
        self.state.copy_(torch.tensor([s, 1.0 / s, 0.0, float(sd.get("_growth_tracker", 0)), self._growth_factor,
                                       self._backoff_factor, float(self._growth_interval), 0.0]))


def make_scaler(device) -> Optional[object]:
    """The fp16 scaler of the engine: fused on a HIP device, torch's GradScaler elsewhere."""
    device = torch.device(device)
    if device.type == "cuda":
        return FusedGradScaler(device)
    return torch.amp.GradScaler(device.type)
