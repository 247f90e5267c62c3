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
the scheduler after a skipped optimizer step); the update's last block publishes it into a
host-mapped ring (``(n << 1) | skipped`` at slot ``n % 64`` for update number ``n``), which the host
reads lazily with a plain load — no copy and no event on the stream (those cost the launch-bound
fp16 LeNet step ~40 us of host time).  The two launches are graph-capturable (``step_device``):
fp16 steps are captured like bf16 ones.  Optimizers that are not fused fall back to the torch primitives on the
same device state.  ``state_dict`` uses ``torch.amp.GradScaler``'s format (``scaler.pt``
checkpoints are interchangeable).
"""

from __future__ import annotations

from typing import Optional

import ctypes
import weakref

import torch

SCALE, INV, FOUND, TRACKER, GROWTH, BACKOFF, INTERVAL, LAST, SEQ = range(9)
HOST = 10   # slots 10..11: device address of the host-mapped flag ring (int64 bits)
SLOTS = 12  # optim_common.h kAmpSlots
RING = 64   # optim_common.h kAmpRing


_ACTIVE = {}  # device -> weakref of the last enabled FusedGradScaler created on it


def active_loss_scale(device) -> Optional[torch.Tensor]:
    """The live loss-scale tensor of the last enabled FusedGradScaler on ``device`` (or None): what a
    kernel that folds the loss scale into the gradient it seeds should assume before its loss says
    otherwise (the fused LeNet's speculative whole-step launch)."""
    ref = _ACTIVE.get(torch.device(device))
    sc = ref() if ref is not None else None
    return sc.scale_tensor if sc is not None else None


class FusedGradScaler:
    def __init__(self, device, init_scale: float = 2.0 ** 16, growth_factor: float = 2.0,
                 backoff_factor: float = 0.5, growth_interval: int = 2000, enabled: bool = True):
        self.device = torch.device(device)
        self._enabled = enabled
        self._growth_factor = float(growth_factor)
        self._backoff_factor = float(backoff_factor)
        self._growth_interval = int(growth_interval)
        self.state = torch.zeros(SLOTS, dtype=torch.float32, device=self.device)
        self.state[:8].copy_(torch.tensor([init_scale, 1.0 / init_scale, 0.0, 0.0, growth_factor, backoff_factor,
                                           float(growth_interval), 0.0]))
        # the live scale as a fixed 1-element view (state is only ever updated in place): kernels
        # that fold the loss scale into the gradient they seed read it from here
        self.scale_tensor = self.state[SCALE : SCALE + 1] if enabled else None
        if self.scale_tensor is not None:
            self.scale_tensor._rocket_amp_state = self.state  # consumers that also flag found-inf
            if self.device.type == "cuda":
                idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
                _ACTIVE[torch.device("cuda", idx)] = weakref.ref(self)
        # the skip flags of recent updates (a caller may hold the handle of update n while n+1
        # publishes its own: EngineScheduler speculation): host-mapped on a HIP device, written by
        # the update kernel; plain host memory elsewhere
        self._ring_h = None
        if self.device.type == "cuda":
            from rocket_amd.ops import _lib

            lib = _lib.kernels()
            dev = ctypes.c_void_p()
            with torch.cuda.device(self.device):
                h = lib.rk_host_mapped_alloc(RING * 4, ctypes.byref(dev))
            if not h:
                raise RuntimeError("FusedGradScaler: rk_host_mapped_alloc failed")
            self._ring_h = h
            self._free = lib.rk_host_mapped_free
            self._ring = (ctypes.c_int32 * RING).from_address(h)
            self.state.view(torch.int64)[HOST // 2] = int(dev.value)
        else:
            self._ring = (ctypes.c_int32 * RING)()
        self._seq = 0  # updates launched (host count; the device counts its own in state[SEQ])
        self._unscaled = set()  # id(optimizer) unscaled this step (clip_grad_norm_ path)

    def __del__(self):
        h, self._ring_h = getattr(self, "_ring_h", None), None
        if h:
            try:
                torch.cuda.synchronize(self.device)  # no update may still write the ring
                self._free(h)
            except Exception:
                pass

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
            # consume the producer's mark on every step (also the unscale_ path), so a stale mark
            # can never skip the check of a later step whose producer did not fold it
            checked = self._producer_checked(optimizer)
            if not unscaled:
                if not checked:
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
        self._record_last(host_flag=skip)
        return out

    def step_device(self, optimizer, zero_grads: bool = False) -> None:
        """The device part of a fused scaled step (flag check + update with in-kernel unscale and
        scale rule): graph-capturable; ``record_last`` after the replay publishes the skip flag."""
        checked = self._producer_checked(optimizer)  # consumed on every step (see step)
        if id(optimizer) not in self._unscaled:
            if not checked:
                optimizer.amp_check(self.state)
        else:
            self.state[INV] = 1.0
        optimizer.amp = self.state
        try:
            optimizer.launch(zero_grads=zero_grads)
        finally:
            optimizer.amp = None
        self._unscaled.clear()

    @staticmethod
    def _producer_checked(optimizer) -> bool:
        """The gradients' producer already flagged non-finite values into state[FOUND] (the fused
        LeNet weight-gradient launch: _FusedBase.amp_fold_target); consumes the mark."""
        done = getattr(optimizer, "amp_checked", False)
        if done:
            optimizer.amp_checked = False
        return done

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

    def _record_last(self, host_flag=None) -> None:
        """One update was launched (its kernel publishes the flag), or ran host side (``host_flag``:
        its skip flag, published here, and the device count advanced to match)."""
        self._unscaled.clear()
        self._seq += 1
        if host_flag is not None:
            u = ((self._seq << 1) | int(bool(host_flag))) & 0xFFFFFFFF  # as the kernel stores it
            self._ring[self._seq % RING] = u - (1 << 32) if u >= (1 << 31) else u
            self.state.view(torch.int32)[SEQ] += 1

    def _entry(self, seq: int):
        """The published skip flag of update ``seq``, or None (not yet written / overwritten)."""
        u = self._ring[seq % RING] & 0xFFFFFFFF
        return bool(u & 1) if (u >> 1) == (seq & 0x7FFFFFFF) else None

    def _resolve(self, seq: int) -> bool:
        f = self._entry(seq)
        if f is not None:
            return f
        torch.cuda.synchronize(self.device)  # the update is enqueued: wait for it
        f = self._entry(seq)
        if f is not None:
            return f
        # the host and device counts disagree (an update ran outside record_last, or this handle
        # is over RING updates old): realign on the device's count, answer with its latest flag
        self._seq = int(self.state.view(torch.int32)[SEQ].item())
        return bool(self.state[LAST].item() != 0)

    def last_handle(self):
        """Handle of the last launched update's skip flag: resolve with :func:`handle_skipped`."""
        return (self, self._seq)

    @staticmethod
    def handle_ready(h) -> bool:
        return h[1] == 0 or h[0]._entry(h[1]) is not None

    @staticmethod
    def handle_seq(h):
        """The update number a handle names (None for the null handle or a stand-in without one)."""
        return h[1] if h[1] != 0 and isinstance(h[1], int) else None

    @staticmethod
    def handle_age(h) -> int:
        """Updates launched on the handle's scaler since the one it names (the flag ring keeps RING)."""
        seq = getattr(h[0], "_seq", None)
        return 0 if h[1] == 0 or not isinstance(seq, int) else seq - h[1]

    @staticmethod
    def handle_skipped(h) -> bool:
        return False if h[1] == 0 else h[0]._resolve(h[1])

    def update(self, new_scale=None) -> None:
        """The scale update already ran on the device; ``new_scale`` overrides it."""
        if new_scale is not None:
            v = float(new_scale)
            self.state[SCALE] = v
            self.state[INV] = 1.0 / v

    def last_step_skipped(self) -> bool:
        """Whether the last scaled step found inf/NaN gradients (waits only if it has not run yet)."""
        return self.handle_skipped(self.last_handle())

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
        self.state[:8].copy_(torch.tensor([s, 1.0 / s, 0.0, float(sd.get("_growth_tracker", 0)), self._growth_factor,
                                           self._backoff_factor, float(self._growth_interval), 0.0]))


def make_scaler(device) -> Optional[object]:
    """The fp16 scaler of the engine: fused on a HIP device, torch's GradScaler elsewhere."""
    device = torch.device(device)
    if device.type == "cuda":
        return FusedGradScaler(device)
    return torch.amp.GradScaler(device.type)
