"""Fused multi-tensor optimizers on the HIP kernel ``native/kernels/optim.hip``.

:class:`FusedAdamW` / :class:`FusedAdam` / :class:`FusedSGD` are drop-in
``torch.optim.Optimizer`` subclasses (same constructor arguments and the same
``state_dict`` format as ``torch.optim.AdamW``/``Adam``/``SGD``, so
``optimizer.bin`` checkpoints stay interchangeable).

Per ``step()`` exactly one kernel launch updates every parameter (10 tensors /
61,706 elements for LeNet; hundreds of tensors for ResNet/ViT).  The launch
reads device-resident tables: tensor pointers (re-uploaded only when a pointer
changes), per-group hyper-parameters (re-uploaded only when a scheduler changes
them) and the step counter (advanced on the device).  ``step()`` is therefore
HIP-graph capturable: :meth:`prepare` does the host bookkeeping outside the
graph, :meth:`launch` is the captured part.
"""

from __future__ import annotations

from typing import List, Optional

import operator

import torch

from rocket_amd.ops import _lib


def _same_layout(a: torch.Tensor, b: torch.Tensor) -> bool:
    """Same memory walk: strides agree on every dim of size > 1."""
    return a.shape == b.shape and all(sa == sb for sa, sb, n in zip(a.stride(), b.stride(), a.shape) if n > 1)


class _FusedBase(torch.optim.Optimizer):
    KIND = 0
    STATE_KEYS: tuple = ()

    def __init__(self, params, defaults):
        super().__init__(params, defaults)
        self._key = None
        self._tables = None
        self._hyper_host = None
        self._hyper_list = None
        self._hyper_dev = None
        self._hyper_get = None
        self._hyper_raw = None
        self._step_dev = None
        self._device = None
        self._gdtype = 0
        self._nblocks = 0
        self._chunk = 0
        self.version = 0  # bumped whenever a device table/state pointer changes (captured graphs go stale)
        # fp16 AMP: the device loss-scaling state of a FusedGradScaler (optim_common.h AmpSlot
        # layout), set for the launches of a scaled step.  torch.amp.GradScaler instead drives the
        # ``_step_supports_amp_scaling`` protocol below (grad_scale / found_inf tensors).
        self.amp: Optional[torch.Tensor] = None
        self._torch_amp = None
        # data parallel over the P2P kernel: an identity AmpSlot block whose found flag a timed-out
        # reduction raises (parallel/p2p.py), read by unscaled launches so they skip that update
        self.guard: Optional[torch.Tensor] = None

    # ----------------------------------------------------------- host side
    def _active(self) -> List[tuple]:
        out = []
        for gi, group in enumerate(self.param_groups):
            for p in group["params"]:
                if p.grad is not None:
                    out.append((gi, p))
        return out

    def _hyper_row(self, group) -> List[float]:
        raise NotImplementedError

    def _init_state(self, p) -> None:
        st = self.state[p]
        for k in self.STATE_KEYS:
            if k not in st:
                st[k] = torch.zeros_like(p, memory_format=torch.preserve_format)
        if "step" not in st:
            st["step"] = torch.tensor(0.0)

    def _ensure_device_state(self, device) -> None:
        if self._step_dev is None or self._device != device:
            self._device = device
            steps = [float(st["step"]) for st in self.state.values() if "step" in st]
            self._step_dev = torch.tensor([max(steps) if steps else 0.0], dtype=torch.float32, device=device)
            self.version += 1

    def prepare(self) -> bool:
        """Host-side bookkeeping; returns False when there is nothing to update."""
        active = self._active()
        if not active:
            return False
        device = active[0][1].device
        if device.type != "cuda":
            raise RuntimeError(f"{type(self).__name__} needs parameters on a HIP device")
        self._ensure_device_state(device)
        for _, p in active:
            if p.dtype != torch.float32:
                raise RuntimeError(f"{type(self).__name__}: parameters must be fp32 master weights, got {p.dtype}")
            if not _same_layout(p.grad, p):
                # the kernel walks param/grad/state memory linearly: layouts must agree
                raise RuntimeError(f"{type(self).__name__}: gradient layout {p.grad.stride()} differs from the "
                                   f"parameter layout {p.stride()}")
            self._init_state(p)
        gd = {p.grad.dtype for _, p in active}
        if len(gd) != 1 or next(iter(gd)) not in (torch.float32, torch.bfloat16):
            raise RuntimeError(f"{type(self).__name__}: unsupported gradient dtypes {gd}")
        self._gdtype = 0 if torch.float32 in gd else 1
        key = tuple((gi, p.data_ptr(), p.grad.data_ptr()) + self._shadow_ptrs(p) for gi, p in active)
        if key != self._key:
            self._build_tables(active, device)
            self._key = key
        self.refresh_hyper()
        self._opt_called = True  # what torch's LR schedulers check for "optimizer.step() ran first"
        return True

    #: the param-group entries _hyper_row reads (raw values: an unchanged step is one tuple compare)
    HYPER_KEYS: tuple = ()

    def refresh_hyper(self) -> None:
        """Upload the per-group hyper-parameters if a scheduler/user changed them (cheap when unchanged)."""
        if self.HYPER_KEYS:
            get = self._hyper_get
            if get is None:
                get = self._hyper_get = operator.itemgetter(*self.HYPER_KEYS)
            raw = [get(g) for g in self.param_groups]
            if raw == self._hyper_raw:
                return  # (never cached while any entry is a tensor: those change in place)
            # tuple entries too (betas=(Tensor, Tensor) is valid torch Adam/AdamW input)
            self._hyper_raw = None if any(isinstance(x, torch.Tensor) for r in raw for v in r
                                          for x in (v if isinstance(v, (tuple, list)) else (v,))) else raw
        flat = [x for g in self.param_groups for x in self._hyper_row(g)]
        if flat != self._hyper_list:
            self._hyper_list = flat
            if self._hyper_dev is None or self._hyper_dev.numel() != len(flat):
                self.version += 1
            host = torch.tensor(flat, dtype=torch.float32).pin_memory()
            if self._hyper_dev is None or self._hyper_dev.numel() != len(flat):
                self._hyper_dev = torch.empty(len(flat), dtype=torch.float32, device=self._device)
            self._hyper_dev.copy_(host, non_blocking=True)
            self._hyper_host = host  # keep the pinned source alive until the copy has run

    def _build_tables(self, active, device) -> None:
        chunk = int(_lib.kernels().rk_optim_chunk_for(sum(p.numel() for _, p in active)))
        self._chunk = chunk
        recs, blocks = [], []
        for ti, (gi, p) in enumerate(active):
            st = self.state[p]
            s = [st[k].data_ptr() for k in self.STATE_KEYS] + [0] * (2 - len(self.STATE_KEYS))
            rec = [p.data_ptr(), p.grad.data_ptr(), s[0], s[1], p.numel(), gi, *self._shadow_ptrs(p)]
            for c in range((p.numel() + chunk - 1) // chunk):
                recs += rec  # one record per block: the kernel loads it without a dependent table walk
                blocks += [ti, c]
        t_host = torch.tensor(recs, dtype=torch.int64).pin_memory()
        b_host = torch.tensor(blocks, dtype=torch.int32).pin_memory()
        self._tables = (t_host.to(device, non_blocking=True), b_host.to(device, non_blocking=True))
        self._nblocks = len(blocks) // 2
        for _, p in active:  # the kernel now keeps these parameters' bf16 shadows current
            if self._shadow_ptrs(p)[0]:
                p._rocket_shadow_live = True
        self.version += 1

    @staticmethod
    def _shadow_ptrs(p) -> tuple:
        """(index-map, bf16 buffer) pointers of a parameter's registered bf16 shadow, or (0, 0).

        A consumer registers ``p._rocket_bf16_shadow = (index int32 [numel, 2], bf16 buffer)``;
        every update then also writes bf16(p[i]) to ``buffer[index[i, 0/1]]`` (-1 = skip).  With
        ``index = None`` the shadow is dense: ``buffer`` is a bf16 (or fp16) tensor laid out like ``p``."""
        sh = getattr(p, "_rocket_bf16_shadow", None)
        if sh is None:
            return (0, 0)
        idx, buf = sh
        if idx is None and buf.dtype == torch.float16:  # dense fp16 copy (fp16 autocast compute)
            if buf.shape != p.shape or buf.stride() != p.stride() or buf.device != p.device:
                raise RuntimeError("dense fp16 shadow: buffer must have the parameter's shape, layout and device")
            return (2, buf.data_ptr())
        if buf.dtype not in (torch.bfloat16, torch.float16) or buf.device != p.device:
            raise RuntimeError("shadow: expected a bf16 / fp16 buffer on the parameter's device")
        if idx is None:
            if buf.dtype != torch.bfloat16:
                raise RuntimeError("dense shadow: unexpected dtype")
            if buf.shape != p.shape or buf.stride() != p.stride():
                raise RuntimeError("dense bf16 shadow: buffer must have the parameter's shape and layout")
            return (1, buf.data_ptr())
        if idx.dtype != torch.int32 or idx.shape != (p.numel(), 2) or idx.device != p.device:
            raise RuntimeError("bf16 shadow: expected an int32 [numel, 2] index map on the device")
        if not idx.is_contiguous() or idx.data_ptr() % 16:
            # the kernel fetches 4 elements' entries as two 16-byte loads: keep an aligned copy
            idx = idx.contiguous().clone()
            p._rocket_bf16_shadow = (idx, buf)
        # bit 0 of the (16-byte aligned) map pointer: fp16 buffer (optim_common.h shadow_cvt)
        return (idx.data_ptr() | int(buf.dtype == torch.float16), buf.data_ptr())

    # --------------------------------------------------------- device side
    def amp_check(self, amp: torch.Tensor) -> None:
        """Flag non-finite gradients into ``amp`` (one launch over the same block tables)."""
        _lib.check(_lib.kernels().rk_amp_check(self._gdtype, self._tables[0].data_ptr(), self._tables[1].data_ptr(),
                                               self._nblocks, amp.data_ptr(), self._chunk,
                                               _lib.stream_ptr(self._device)), "rk_amp_check")

    def launch(self, zero_grads: bool = False) -> None:
        """Enqueue the fused update (graph-capturable); ``zero_grads`` also clears the consumed gradients."""
        lib = _lib.kernels()
        dev = self._device
        amp = self.amp if self.amp is not None else self._torch_amp if self._torch_amp is not None else self.guard
        _lib.check(
            lib.rk_optim_mt(self.KIND, self._gdtype, self._tables[0].data_ptr(), self._tables[1].data_ptr(),
                            self._nblocks, self._hyper_dev.data_ptr(), self._step_dev.data_ptr(), _lib.ptr(amp),
                            _lib.Workspace.get(dev).counter(f"optim_{id(self)}"), int(zero_grads), self._chunk,
                            _lib.stream_ptr(dev)),
            "rk_optim_mt",
        )

    # torch.amp.GradScaler protocol: with this flag GradScaler.step() skips its own unscale and
    # hands over `grad_scale` (the scale, or None when already unscaled) and `found_inf` tensors
    _step_supports_amp_scaling = True

    def _torch_amp_state(self) -> Optional[torch.Tensor]:
        gs, fi = getattr(self, "grad_scale", None), getattr(self, "found_inf", None)
        if gs is None and fi is None:
            return None
        # a private AmpSlot block: unscale by grad_scale, skip on found_inf; GradScaler.update()
        # (host side) keeps owning the scale, so growth/backoff here are inert
        amp = torch.zeros(12, dtype=torch.float32, device=self._device)  # optim_common.h kAmpSlots
        amp[1] = 1.0
        amp[6] = float("inf")
        if gs is not None:  # torch hands over the scale itself (its fused kernels divide by it)
            amp[1:2].copy_(1.0 / gs.reshape(1).float())
        if fi is not None:
            amp[2:3].copy_(fi.reshape(1).float())
        return amp

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if self.epilogue_done:  # the gradient producer already applied this step's update
            self.epilogue_done = False
            return loss
        if self.prepare():
            self._torch_amp = self._torch_amp_state()
            try:
                self.launch()
            finally:
                self._torch_amp = None
        return loss

    # ------------------------------------------------------------- state
    def _sync_step_to_state(self) -> None:
        if self._step_dev is not None:
            s = float(self._step_dev.item())
            for st in self.state.values():
                if "step" in st:
                    st["step"] = torch.tensor(s)

    def state_dict(self):
        self._sync_step_to_state()
        return super().state_dict()

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        for p, st in self.state.items():
            for k in self.STATE_KEYS:
                if k in st:
                    v = st[k].float()
                    if v.shape == p.shape and not _same_layout(v, p):  # same memory walk as the param
                        v = torch.empty_like(p, dtype=torch.float32).copy_(v)
                    st[k] = v
            if "step" in st and isinstance(st["step"], torch.Tensor):
                st["step"] = st["step"].detach().to("cpu", torch.float32)
        self._key = None
        self._step_dev = None

    @property
    def device_step(self) -> Optional[torch.Tensor]:
        return self._step_dev

    # ------------------------------------------------- update epilogue
    # A kernel that produces parameters' FINAL gradients can apply the update itself (the fused
    # LeNet weight-gradient launch does): the Optimizer capsule arms it for one step when that is
    # exact (single replica, gradient-sync step, no AMP scaler); the producer asks for the records
    # with ``epilogue(params)``, reports ``epilogue_done``, and the step's own launch is skipped.
    epilogue_armed = False
    epilogue_done = False
    # fp16 AMP: a producer of ALL the active parameters' final (fp32) gradients may flag non-finite
    # values into the scaler's found slot itself when armed (``amp_fold_target``); it then sets
    # ``amp_checked`` and the scaler skips this step's check launch
    amp_fold_armed = False
    amp_checked = False

    def amp_fold_target(self, params) -> bool:
        """True when the fold is armed and ``params`` are exactly the active parameters (fp32 grads)."""
        if not (self.amp_fold_armed and self._tables is not None and self._gdtype == 0):
            return False
        active = self._active()
        return len(active) == len(params) and {id(p) for _, p in active} == {id(p) for p in params}

    # The same fusion one stage later, for data parallelism: the P2P all-reduce of the gradient
    # buckets applies the update in its write-back (parallel/p2p.py ``all_reduce_adam_``).  Armed by
    # the Optimizer capsule on a gradient-sync step of a W > 1 run without an AMP scaler.
    reduce_epilogue_armed = False

    def reduce_plan(self, flat: torch.Tensor, params) -> Optional[tuple]:
        """``(segments, ngroups, hyper_ptr, step_ptr, counter_ptr, amp_ptr)`` for a P2P reduce of
        ``flat`` whose ``params`` (their ``.grad`` are views into ``flat``) are updated in its
        write-back; None when that is not exact or not supported.  ``segments``: device int64
        [n, 10] (tensor record, element offset in ``flat``, 0), cached per (flat, table version)."""
        if not (self.reduce_epilogue_armed and self.KIND == 0 and self._tables is not None and self._gdtype == 0):
            return None
        if len(self.param_groups) > 4 or self.amp is not None or self._torch_amp is not None:
            return None
        key = (flat.data_ptr(), flat.numel(), self.version, tuple(id(p) for p in params))
        cache = getattr(self, "_reduce_plans", None)
        if cache is None:
            cache = self._reduce_plans = {}
        hit = cache.get(key)
        if hit is not None:
            return hit
        gidx = {id(p): gi for gi, p in self._active()}
        base = flat.data_ptr()
        rows = []
        for p in params:
            if id(p) not in gidx or p.grad is None:
                return None
            off, rem = divmod(p.grad.data_ptr() - base, 4)
            if rem or off < 0 or off + p.numel() > flat.numel() or not _same_layout(p.grad, p):
                return None
            st = self.state[p]
            s = [st[k].data_ptr() for k in self.STATE_KEYS]
            rows.append([p.data_ptr(), p.grad.data_ptr(), s[0], s[1], p.numel(), gidx[id(p)], *self._shadow_ptrs(p),
                         off, 0])
        if not rows or len(rows) > 32:
            return None
        segs = torch.tensor(rows, dtype=torch.int64).to(self._device)
        dev = self._device
        amp = self.guard
        plan = (segs, len(self.param_groups), self._hyper_dev.data_ptr(), self._step_dev.data_ptr(),
                _lib.Workspace.get(dev).counter(f"optim_{id(self)}"), _lib.ptr(amp))
        if len(cache) > 8:
            cache.clear()
        cache[key] = plan
        return plan

    def epilogue(self, params) -> Optional[tuple]:
        """``(ngroups, hyper_ptr, step_ptr, counter_ptr, records)`` when ``params`` are exactly this
        optimizer's active parameters and the epilogue is armed; ``records[i]`` is the 8-int64 tensor
        record of ``params[i]`` (p, grad, state0, state1, numel, group, shadow map, shadow buffer)."""
        if not (self.epilogue_armed and self.KIND == 0 and self._tables is not None and self._gdtype == 0):
            return None
        active = self._active()
        if len(active) != len(params) or {id(p) for _, p in active} != {id(p) for p in params}:
            return None
        if len(self.param_groups) > 4 or self.amp is not None:
            return None
        gidx = {id(p): gi for gi, p in active}
        recs = []
        for p in params:
            st = self.state[p]
            s = [st[k].data_ptr() for k in self.STATE_KEYS]
            recs.append((p.data_ptr(), p.grad.data_ptr(), s[0], s[1], p.numel(), gidx[id(p)], *self._shadow_ptrs(p)))
        dev = self._device
        return (len(self.param_groups), self._hyper_dev.data_ptr(), self._step_dev.data_ptr(),
                _lib.Workspace.get(dev).counter(f"optim_{id(self)}"), recs)


class FusedAdamW(_FusedBase):
    """AdamW with decoupled weight decay (``torch.optim.AdamW`` semantics, no amsgrad)."""

    KIND = 0
    STATE_KEYS = ("exp_avg", "exp_avg_sq")
    DECOUPLED = True

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, amsgrad=False,
                 *, maximize=False, foreach=None, capturable=False, differentiable=False, fused=None):
        if amsgrad:
            raise NotImplementedError("amsgrad is not supported by the fused kernel")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False, maximize=maximize,
                        foreach=foreach, capturable=capturable, differentiable=differentiable, fused=fused)
        super().__init__(params, defaults)

    HYPER_KEYS = ("lr", "betas", "eps", "weight_decay", "maximize")

    def _hyper_row(self, g):
        lr = float(g["lr"])
        b1, b2 = g["betas"]
        return [lr, float(b1), float(b2), float(g["eps"]), float(g["weight_decay"]),
                1.0 if self.DECOUPLED else 0.0, 1.0 if g.get("maximize") else 0.0, 0.0]


class FusedAdam(FusedAdamW):
    """Adam with L2 weight decay (``torch.optim.Adam`` semantics)."""

    DECOUPLED = False

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=False, **kw):
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=amsgrad, **kw)


class FusedSGD(_FusedBase):
    """SGD with momentum / dampening / nesterov / weight decay (``torch.optim.SGD`` semantics)."""

    KIND = 1
    STATE_KEYS = ("momentum_buffer",)

    def __init__(self, params, lr=1e-3, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False, *,
                 maximize=False, foreach=None, differentiable=False, fused=None):
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                        nesterov=nesterov, maximize=maximize, foreach=foreach, differentiable=differentiable,
                        fused=fused)
        super().__init__(params, defaults)

    HYPER_KEYS = ("lr", "momentum", "dampening", "weight_decay", "nesterov", "maximize")

    def _hyper_row(self, g):
        return [float(g["lr"]), float(g["momentum"]), float(g["dampening"]), float(g["weight_decay"]),
                1.0 if g["nesterov"] else 0.0, 1.0 if g.get("maximize") else 0.0, 0.0, 0.0]

    def _init_state(self, p) -> None:
        st = self.state[p]
        if self.param_groups and any(g["momentum"] != 0 for g in self.param_groups):
            if "momentum_buffer" not in st:
                st["momentum_buffer"] = torch.zeros_like(p)
        if "step" not in st:
            st["step"] = torch.tensor(0.0)

    def _build_tables(self, active, device) -> None:
        for _, p in active:
            self.state[p].setdefault("momentum_buffer", torch.zeros_like(p))
        super()._build_tables(active, device)
