"""The runtime engine: everything the reference delegates to ``accelerate.Accelerator``.

Every capsule of the reference reaches the device/precision/distribution layer
through ``self._accelerator`` (SURVEY §2.3 lists the 25 call sites).  This class
provides that surface natively on PyTorch-ROCm so the capsule code keeps its
shape while the hot path is ours:

==========================  ===================================================
accelerate surface           here
==========================  ===================================================
``Accelerator(...)``         ``Engine(mixed_precision, gradient_accumulation_steps,
                             project_dir, cpu, seed, …)`` — comm initialised first
``prepare(model)``           device move, :class:`~rocket_amd.parallel.ddp.DataParallel`
                             when W>1, autocast+fp32-output forward patch
``prepare(optimizer)``       :class:`EngineOptimizer` (sync-gated step/zero_grad, fp16 scaler)
``prepare(scheduler)``       :class:`EngineScheduler` (steps ×W on sync steps)
``prepare(dataloader)``      :class:`~rocket_amd.runtime.data.ShardedLoader` /
                             :class:`~rocket_amd.runtime.data.DeviceLoader`
``accumulate``/``no_sync``   GA state machine (``_do_sync``) + replica ``no_sync``
``backward``                 ``loss / GA`` (+ GradScaler)
``gather``/``gather_for_metrics``/``reduce``  RCCL collectives, remainder truncation
``save_state``/``load_state``  :mod:`rocket_amd.runtime.checkpoint_io` (same layout)
trackers                     :mod:`rocket_amd.runtime.trackers`
==========================  ===================================================
"""

from __future__ import annotations

import contextlib
import math
import os
from typing import Any, Callable, List, Optional

import torch
from torch import nn

from rocket_amd.parallel.ddp import DataParallel, unwrap
from rocket_amd.runtime import comm as _comm
from rocket_amd.runtime import checkpoint_io
from rocket_amd.runtime.amp import RING as _AMP_RING, FusedGradScaler, make_scaler
from rocket_amd.runtime.host_data import HostLoader, HostTensorDataset
from rocket_amd.runtime.data import (
    DeviceLoader,
    DeviceTensorDataset,
    GradientState,
    ShardedLoader,
    _LoaderBase,
)
from rocket_amd.runtime.trackers import GeneralTracker, make_tracker
from rocket_amd.utils.collections import apply_to_collection, is_collection
from rocket_amd.utils.logging import get_logger

logger = get_logger(__name__)

_MP = {None: None, "no": None, "fp32": None, "bf16": torch.bfloat16, "fp16": torch.float16}


def _to_fp32(x):
    if isinstance(x, torch.Tensor):
        return x.float() if x.dtype in (torch.float16, torch.bfloat16) else x
    if is_collection(x) and not isinstance(x, (str, bytes)):
        return apply_to_collection(x, lambda v, key=None: _to_fp32(v))
    return x


class EngineOptimizer:
    """Optimizer wrapper: steps and zeroes only on gradient-sync micro-steps.

    Parity: ``accelerate.optimizer.AcceleratedOptimizer`` (reached from
    ``rocket/core/optimizer.py:109,128-130``).
    """

    def __init__(self, optimizer: torch.optim.Optimizer, engine: "Engine"):
        self.optimizer = optimizer
        self.engine = engine
        self._skipped = False
        self._skip_lazy = False  # fp16 fused scaler: the flag lives on the device until asked for
        self._lazy_handle = None  # (pinned copy, event) of that flag (FusedGradScaler.last_handle)

    @property
    def step_was_skipped(self) -> bool:
        """accelerate's ``step_was_skipped``.  With the device-resident scaler it is read back only
        here (waiting for that step's update), not on every step."""
        if self._skip_lazy:
            h = self._lazy_handle
            self._skipped = (FusedGradScaler.handle_skipped(h) if h is not None
                             else self.engine.scaler.last_step_skipped())
            self._skip_lazy = False
        return self._skipped

    def step_was_skipped_lazy(self) -> None:
        """A scaled update ran on the device (e.g. in a replayed graph): resolve the flag on demand."""
        self._skip_lazy = True
        scaler = self.engine.scaler
        self._lazy_handle = scaler.last_handle() if isinstance(scaler, FusedGradScaler) else None

    @step_was_skipped.setter
    def step_was_skipped(self, v: bool) -> None:
        self._skipped, self._skip_lazy = bool(v), False

    @property
    def param_groups(self):
        return self.optimizer.param_groups

    @property
    def state(self):
        return self.optimizer.state

    @property
    def defaults(self):
        return self.optimizer.defaults

    def state_dict(self):
        # a speculated scheduler step may still hold this optimizer's param-group hyperparameters:
        # settle it first, so the saved lr is the one accelerate would hold
        for s in getattr(self.engine, "_schedulers", ()):
            if any(o is self for o in s.optimizers):
                s._resolve()
        return self.optimizer.state_dict()

    def load_state_dict(self, sd):
        self.optimizer.load_state_dict(sd)

    def _params(self):
        return [p for g in self.optimizer.param_groups for p in g["params"]]

    def zero_grad(self, set_to_none: Optional[bool] = None) -> None:
        if not self.engine.sync_gradients:
            return
        self.engine.zero_grads(self._params(), set_to_none)

    def step(self, closure: Callable | None = None):
        if not self.engine.sync_gradients:
            return None
        scaler = self.engine.scaler
        if isinstance(scaler, FusedGradScaler):
            out = scaler.step(self.optimizer, closure) if closure else scaler.step(self.optimizer)
            self.step_was_skipped_lazy()
            return out
        if scaler is not None:
            scale_before = scaler.get_scale()
            scaler.step(self.optimizer, closure) if closure else scaler.step(self.optimizer)
            scaler.update()
            self.step_was_skipped = scaler.get_scale() < scale_before
            return None
        self.step_was_skipped = False
        return self.optimizer.step(closure) if closure else self.optimizer.step()

    def fused_zero_ok(self) -> bool:
        """True when the fused update kernel may clear the gradients itself (same result as zero_grad)."""
        opt = self.optimizer
        return (
            (self.engine.scaler is None or isinstance(self.engine.scaler, FusedGradScaler))
            and hasattr(opt, "launch")
            and all(getattr(p, "_rocket_direct_grad", False) for p in self._params() if p.requires_grad)
        )

    def step_and_zero_grad(self, set_to_none: Optional[bool] = None) -> None:
        """``step(); zero_grad()`` — one kernel for the fused optimizers over persistent gradients."""
        if not self.engine.sync_gradients:
            return
        if self.fused_zero_ok():
            if isinstance(self.engine.scaler, FusedGradScaler):
                self.engine.scaler.step(self.optimizer, zero_grads=True)
                self.step_was_skipped_lazy()
                return
            self.step_was_skipped = False
            if self.optimizer.prepare():
                self.optimizer.launch(zero_grads=True)
            return
        self.step()
        self.zero_grad(set_to_none)

    def __getattr__(self, name):
        return getattr(self.optimizer, name)


class EngineScheduler:
    """Scheduler wrapper (parity: ``accelerate.scheduler.AcceleratedScheduler``).

    On sync steps it steps once per process (the global batch grew ×W); on
    accumulation micro-steps it only advances ``_step_count``.
    """

    #: fp16 device-resident scaler: the step's skip flag is on the device when the scheduler steps.
    #: Exact form (default): step the scheduler provisionally and keep it undecided only when that
    #: leaves every param-group hyperparameter unchanged (StepLR / MultiStepLR between milestones,
    #: warmup plateaus...) — the next update then runs with the same lr whichever way the flag reads,
    #: so the lr sequence is accelerate's, and the flag is read at the next scheduler step (a
    #: skipped step rolls the scheduler state back).  A step that would change a hyperparameter
    #: waits for the flag (a host sync on those steps only).
    #: Opt-in (ROCKET_SCHED_SPECULATE=1): provisional steps also when the hyperparameters change;
    #: after a skipped step one update then runs with the next lr, which accelerate never does.
    SPECULATE = os.environ.get("ROCKET_SCHED_SPECULATE", "0") == "1"
    #: ROCKET_SCHED_LIGHT=1: provisional steps between StepLR milestones keep a three-field snapshot
    #: instead of a state_dict copy.  Off: it cut host time per step but the fp16 LeNet step measured
    #: slower with it (19.7-19.8 M vs 21.1-21.3 M samples/s, same box, scripts/archive/r5/gpu_fp.sh; the GPU
    #: step p50 rose 0.043 -> 0.046 ms — the faster host polls the device's skip-flag ring sooner)
    LIGHT = os.environ.get("ROCKET_SCHED_LIGHT", "0") == "1"
    #: provisional steps kept undecided at once (exact form): a step does not wait for the previous
    #: steps' flags, it settles the ones that have landed (the flag ring holds 64 updates).
    #: ROCKET_SCHED_QUEUE=1: one at a time (every step first waits for the previous step's flag)
    MAXQ = max(1, min(32, int(os.environ.get("ROCKET_SCHED_QUEUE", "16"))))

    def __init__(self, scheduler, optimizers: List[EngineOptimizer], engine: "Engine"):
        self.scheduler = scheduler
        self.optimizers = optimizers
        self.engine = engine
        self._queue = []  # [(flag handles, snapshot)] of provisional steps, oldest first
        self.mispredicted = 0  # provisional steps rolled back (their update was skipped)
        self.provisional = 0  # steps taken before their skip flag was read
        self._seen_seq = {}  # id(scaler) -> its update count at the previous scheduler step

    def _groups(self):
        return [g for o in self.optimizers for g in o.optimizer.param_groups]

    def _snapshot(self):
        sd = {k: (list(v) if isinstance(v, list) else v) for k, v in self.scheduler.state_dict().items()}
        return "full", sd, [{k: v for k, v in g.items() if k != "params"} for g in self._groups()]

    @property
    def _pending(self):
        """The newest provisional step (flag handles, snapshot), or None."""
        return self._queue[-1] if self._queue else None

    def _restore(self, snap) -> None:
        if snap[0] == "light":  # fast StepLR steps: only these three fields moved
            s = self.scheduler
            _, s._step_count, s.last_epoch, s._last_lr = snap
            return
        _, sd, groups = snap
        self.scheduler.load_state_dict(sd)
        for g, saved in zip(self._groups(), groups):
            g.update(saved)

    def _resolve(self, wait: bool = True) -> None:
        """Settle the provisional steps in order: a kept one is dropped from the queue; a skipped one
        is undone (its snapshot restored) and the later, still undecided ones are taken again from
        there.  They left every hyperparameter unchanged, and re-taken one epoch earlier they stay
        inside the same constant stretch of the schedule, so no update sees a different lr.
        ``wait=False``: stop at the first step whose flag has not landed (no host sync)."""
        while self._queue:
            handles, snap = self._queue[0]
            if not wait and not all(FusedGradScaler.handle_ready(h) for h in handles):
                return
            if not any(FusedGradScaler.handle_skipped(h) for h in handles):
                self._queue.pop(0)
                continue
            self.mispredicted += 1
            later = self._queue[1:]
            self._restore(snap)
            self._queue = []
            for h2, old in later:
                light = old[0] == "light"
                s = self.scheduler
                self._queue.append((h2, ("light", s._step_count, s.last_epoch, s._last_lr) if light
                                    else self._snapshot()))
                self._do_step()

    def _cadence(self, handles) -> int:
        """Scaler updates since the previous scheduler step (the largest over the handles' scalers);
        remembers the current counts for the next call."""
        seen = self._seen_seq
        cadence = 0
        for h in handles:
            seq = FusedGradScaler.handle_seq(h)
            if seq is None:
                continue
            cadence = max(cadence, seq - seen.get(id(h[0]), 0))  # first step: updates since the start
            seen[id(h[0])] = seq
        return cadence

    def _ages_out(self, cadence: int) -> bool:
        """Whether the oldest provisional step's flag would be overwritten in the scaler's flag ring
        (``amp.RING`` updates) before the next scheduler step: then it is settled now."""
        if not self._queue:
            return False
        age = max((FusedGradScaler.handle_age(h) for h in self._queue[0][0]), default=0)
        return age + cadence + len(self.optimizers) >= _AMP_RING

    def _light_ok(self) -> bool:
        """The next scheduler step(s) of this sync step are all ``_fast_step``s (StepLR between
        milestones): they move only ``_step_count`` / ``last_epoch`` / ``_last_lr`` and leave every
        hyperparameter, so the provisional step needs no state_dict snapshot nor group compare."""
        s = self.scheduler
        if type(s) is not torch.optim.lr_scheduler.StepLR or s._step_count == 1:
            return False
        for i in range(1, self.engine.num_processes + 1):
            e = s.last_epoch + i
            if e == 0 or e % s.step_size == 0:
                return False
        return all(type(g["lr"]) is float for g in s.optimizer.param_groups)

    def _do_step(self, *args, **kwargs) -> None:
        for _ in range(self.engine.num_processes):
            total = getattr(self.scheduler, "total_steps", None)
            if total is not None and self.scheduler._step_count > total:
                continue
            if args or kwargs or not self._fast_step():
                self.scheduler.step(*args, **kwargs)

    def _fast_step(self) -> bool:
        """``StepLR.step()`` between milestones without torch's generic machinery (~4 us of host
        time per iteration): exactly what it does there — ``_step_count`` and ``last_epoch`` advance,
        the param groups' lr stay, ``_last_lr`` is re-read.  Only for the exact class with float lrs
        and off its first call (where torch checks the optimizer-order warnings)."""
        s = self.scheduler
        if type(s) is not torch.optim.lr_scheduler.StepLR or s._step_count == 1:
            return False
        e = s.last_epoch + 1
        if e != 0 and e % s.step_size == 0:
            return False  # a milestone: the lr changes
        lrs = [g["lr"] for g in s.optimizer.param_groups]
        if not all(type(v) is float for v in lrs):
            return False
        s._step_count += 1
        s.last_epoch = e
        s._last_lr = lrs
        return True

    def step(self, *args, **kwargs):
        if not self.engine.sync_gradients:
            self.scheduler._step_count += 1
            return
        # exact form: settle the provisional steps whose flags have landed, without waiting for the
        # rest (a host sync here would drain the device queue every step); speculation / explicit
        # scheduler arguments keep one undecided step at a time
        queued = not (self.SPECULATE or args or kwargs)
        lazy = [o for o in self.optimizers if o._skip_lazy and o._lazy_handle is not None]
        handles = [o._lazy_handle for o in lazy]
        cadence = self._cadence(handles)
        self._resolve(wait=not queued or len(self._queue) >= self.MAXQ or self._ages_out(cadence))
        # a flag must still be in the scaler's ring when the NEXT scheduler step reads it: at a slow
        # cadence (a scheduler stepped once per epoch, several optimizers on one scaler) the step
        # waits for its own flag instead of queueing (one host sync per scheduler step)
        slow = 2 * cadence + len(self.optimizers) >= _AMP_RING
        if lazy and len(lazy) == len(self.optimizers) and not slow and \
                not all(FusedGradScaler.handle_ready(h) for h in handles):
            if self.LIGHT and not args and not kwargs and self._light_ok():
                s = self.scheduler
                snap = ("light", s._step_count, s.last_epoch, s._last_lr)
                self._do_step()
                self.provisional += 1
                self._queue.append((handles, snap))
                return
            snap = self._snapshot()
            self._do_step(*args, **kwargs)
            if self.SPECULATE or all(
                    {k: v for k, v in g.items() if k != "params"} == saved for g, saved in zip(self._groups(), snap[2])):
                self.provisional += 1
                self._queue.append((handles, snap))
                return
            # this step moves a hyperparameter: undo it, settle every earlier provisional step, then
            # decide on this step's own flag
            self._restore(snap)
            self._resolve()
        if any(o.step_was_skipped for o in self.optimizers):
            return
        self._do_step(*args, **kwargs)

    def get_last_lr(self):
        self._resolve()
        return self.scheduler.get_last_lr()

    def state_dict(self):
        self._resolve()
        return self.scheduler.state_dict()

    def load_state_dict(self, sd):
        self._queue = []
        self.scheduler.load_state_dict(sd)

    def __getattr__(self, name):
        return getattr(self.scheduler, name)


class Engine:
    """Native replacement of the accelerate runtime used by the capsules."""

    def __init__(
        self,
        device_placement: bool = True,
        mixed_precision: str | None = None,
        gradient_accumulation_steps: int = 1,
        project_dir: str | None = None,
        cpu: bool | None = None,
        seed: int | None = None,
        bucket_cap_mb: float | None = None,
        even_batches: bool = True,
        log_with: List[str] | None = None,
        flat_grads: bool | None = None,
        comm: str | None = None,
        **unused: Any,
    ):
        env_mp = os.environ.get("ROCKET_MIXED_PRECISION", os.environ.get("ACCELERATE_MIXED_PRECISION"))
        mixed_precision = mixed_precision if mixed_precision is not None else env_mp
        if mixed_precision not in _MP:
            raise ValueError(f"unsupported mixed_precision {mixed_precision!r}")
        self.ctx = _comm.init(cpu=cpu)
        if self.ctx.device.type == "cuda":
            from rocket_amd.runtime.tuning import use_tuned_gemms

            use_tuned_gemms()  # measured hipBLASLt solutions for the library GEMMs
        self.device_placement = device_placement
        self.mixed_precision = mixed_precision or "no"
        self._amp_dtype = _MP[mixed_precision]
        self.gradient_accumulation_steps = max(1, int(gradient_accumulation_steps))
        self.gradient_state = GradientState(self.gradient_accumulation_steps)
        self.project_dir = project_dir
        self.logging_dir = project_dir
        self.seed = 0 if seed is None else int(seed)
        self.even_batches = even_batches
        self.bucket_cap_mb = bucket_cap_mb or float(os.environ.get("ROCKET_BUCKET_MB", 32.0))
        self.step = 0
        self.scaler = None
        if self.mixed_precision == "fp16":
            self.scaler = make_scaler(self.device)
        self._models: List[nn.Module] = []
        self._wrapped: dict = {}
        self._grad_owners: list = []  # FlatGrads / DataParallel owning persistent .grad storage
        self.flat_grads = self.device.type == "cuda" if flat_grads is None else bool(flat_grads)
        # data-parallel transport: "native" (own RCCL communicator + side-stream bucket reducer; the
        # default on GPUs: graph-capturable, so a captured DP step overlaps its all-reduce with
        # backward) or "torch" (ProcessGroupNCCL = RCCL; ROCKET_NATIVE_COMM=0)
        self.comm_backend = comm or ("torch" if os.environ.get("ROCKET_NATIVE_COMM", "1") == "0" else "native")
        self._native_comm = None
        self._optimizers: List[EngineOptimizer] = []
        self._schedulers: List[EngineScheduler] = []
        self._dataloaders: List[_LoaderBase] = []
        self._custom_objects: List[Any] = []
        self.trackers: List[GeneralTracker] = []
        self.log_with: List[str] = list(log_with or [])

    # ------------------------------------------------------------ topology
    @property
    def device(self) -> torch.device:
        return self.ctx.device

    @property
    def num_processes(self) -> int:
        return self.ctx.world_size

    @property
    def process_index(self) -> int:
        return self.ctx.rank

    @property
    def local_process_index(self) -> int:
        return self.ctx.local_rank

    @property
    def num_nodes(self) -> int:
        return self.ctx.num_nodes

    @property
    def is_main_process(self) -> bool:
        return self.ctx.is_main_process

    @property
    def is_local_main_process(self) -> bool:
        return self.ctx.is_local_main_process

    @property
    def distributed(self) -> bool:
        return self.ctx.distributed

    def wait_for_everyone(self) -> None:
        _comm.barrier()

    def print(self, *args, **kwargs) -> None:
        if self.is_local_main_process:
            print(*args, **kwargs)

    # ------------------------------------------------------------- prepare
    def prepare(self, *objs, device_placement: Optional[List[bool]] = None):
        placement = device_placement or [self.device_placement] * len(objs)
        out = []
        for obj, place in zip(objs, placement):
            if isinstance(obj, nn.Module):
                out.append(self.prepare_model(obj, device_placement=place))
            elif isinstance(obj, torch.optim.Optimizer):
                out.append(self.prepare_optimizer(obj))
            elif isinstance(obj, torch.optim.lr_scheduler.LRScheduler) or hasattr(obj, "get_last_lr"):
                out.append(self.prepare_scheduler(obj))
            elif isinstance(obj, (torch.utils.data.DataLoader, _LoaderBase)):
                out.append(self.prepare_data_loader(obj, device_placement=place))
            else:
                out.append(obj)
        return out[0] if len(out) == 1 else tuple(out)

    def prepare_model(self, model: nn.Module, device_placement: bool = True) -> nn.Module:
        if device_placement:
            model = model.to(self.device)
        if self._amp_dtype is not None and not getattr(model.forward, "_rocket_amp", False):
            orig = model.forward
            dtype, dev = self._amp_dtype, self.device.type

            def forward(*args, **kwargs):
                with torch.autocast(device_type=dev, dtype=dtype):
                    out = orig(*args, **kwargs)
                return _to_fp32(out)

            forward._rocket_amp = True
            forward.__wrapped__ = orig
            model.forward = forward
        self._models.append(model)
        if self.distributed and any(p.requires_grad for p in model.parameters()):
            wrapped = DataParallel(model, bucket_cap_mb=self.bucket_cap_mb, comm=self._dp_comm())
            self._wrapped[id(model)] = wrapped
            self._grad_owners.append(wrapped)
            self._wire_fault_guards()
            return wrapped
        if self.flat_grads and any(p.requires_grad for p in model.parameters()):
            from rocket_amd.parallel.flat_grads import FlatGrads

            self._grad_owners.append(FlatGrads([p for p in model.parameters()]))
        return model

    def _dp_comm(self):
        if os.environ.get("ROCKET_DP_COMM") == "p2p" and self.device.type == "cuda":
            # P2P-kernel transport (parallel/p2p.py P2PComm): overlapped + capturable like the native
            # reducer, and it runs with several ranks on one device (single-GPU rehearsals)
            if self._native_comm is None:
                from rocket_amd.parallel.p2p import P2PComm

                cap = int(os.environ.get("ROCKET_P2P_COMM_CAP", str(16 << 20)))
                self._native_comm = P2PComm.create(cap, group=_comm.context().host_group, device=self.device)
            return self._native_comm
        if self.comm_backend != "native" or self.device.type != "cuda" or _comm.context().backend != "nccl":
            return None  # DataParallel's default: the torch.distributed RCCL/gloo group
        if self._native_comm is None:
            from rocket_amd.parallel.rccl import RcclComm

            comm, err = None, None
            try:
                comm = RcclComm(self.device)
            except Exception as e:
                err = e
            # a failure can be rank-local (hipSetDevice, an allocation, a watchdog): the ranks agree
            # over the host group, and ALL fall back together if any rank failed — a rank that fell
            # back alone would issue different collectives from its peers and hang them
            if not _comm.all_ranks_agree(err is None):
                if comm is not None:
                    comm.close()
                logger.warning(f"native RCCL communicator unavailable on some rank ({err or 'peer failed'}); "
                               "every rank uses the torch.distributed group")
                self.comm_backend = "torch"
                return None
            self._native_comm = comm
        return self._native_comm

    def grad_owner(self, p):
        for o in self._grad_owners:
            if o.owns(p):
                return o
        return None

    def zero_grads(self, params, set_to_none: Optional[bool] = None) -> None:
        """Zero gradients: one memset per persistent buffer fully covered, views otherwise."""
        params = list(params)
        ids = {id(p) for p in params}
        loose = []
        done = set()
        for o in self._grad_owners:
            mine = [p for p in o.params if id(p) in ids]
            if not mine:
                continue
            if len(mine) == len(o.params):
                o.zero_()
            else:
                with torch.no_grad():
                    for p in mine:
                        p.grad.zero_()
            done.update(id(p) for p in mine)
        for p in params:
            if id(p) not in done:
                loose.append(p)
        for p in loose:
            if p.grad is None:
                continue
            if set_to_none is False:
                with torch.no_grad():
                    p.grad.zero_()
            else:
                p.grad = None

    def prepare_optimizer(self, optimizer: torch.optim.Optimizer) -> EngineOptimizer:
        if self.device_placement:
            for state in optimizer.state.values():
                for k, v in state.items():
                    if isinstance(v, torch.Tensor) and k != "step":
                        state[k] = v.to(self.device)
        wrapped = EngineOptimizer(optimizer, self)
        self._optimizers.append(wrapped)
        self._wire_fault_guards()
        return wrapped

    def _wire_fault_guards(self) -> None:
        """Fused optimizers of a model reduced by the P2P kernel read its fault guard (a peer
        timeout then skips the update that would apply un-reduced gradients); with the fp16
        scaler the kernel also raises the scaler's found flag (parallel/p2p.py)."""
        for o in self._grad_owners:
            p2p = getattr(o, "_p2p", None)
            if p2p is None:
                continue
            if isinstance(self.scaler, FusedGradScaler):
                p2p.guard_scaler(self.scaler.state)
            for eo in self._optimizers:
                opt = eo.optimizer
                if hasattr(opt, "guard") and any(o.owns(p) for g in opt.param_groups for p in g["params"]):
                    opt.guard = p2p.fault

    def prepare_scheduler(self, scheduler) -> EngineScheduler:
        opts = [o for o in self._optimizers if o.optimizer is getattr(scheduler, "optimizer", None)]
        wrapped = EngineScheduler(scheduler, opts or list(self._optimizers), self)
        self._schedulers.append(wrapped)
        return wrapped

    def make_loader(self, dataset, device_placement: bool = False, **kwargs) -> _LoaderBase:
        """Build the sharded loader for a dataset (what ``Dataset.setup`` uses)."""
        common = dict(
            num_replicas=self.num_processes,
            rank=self.process_index,
            even_batches=self.even_batches,
            seed=kwargs.pop("seed", self.seed),
            gradient_state=self.gradient_state,
        )
        if isinstance(dataset, DeviceTensorDataset):
            loader = DeviceLoader(dataset, **kwargs, **common)
        elif isinstance(dataset, HostTensorDataset):
            loader = HostLoader(dataset, device=self.device if device_placement else None, **kwargs, **common)
        else:
            kwargs.setdefault("pin_memory", self.device.type == "cuda")
            loader = ShardedLoader(dataset, device=self.device if device_placement else None, **kwargs, **common)
        self._dataloaders.append(loader)
        return loader

    def prepare_data_loader(self, dl, device_placement: bool = False) -> _LoaderBase:
        if isinstance(dl, _LoaderBase):
            if dl not in self._dataloaders:
                self._dataloaders.append(dl)
            return dl
        kw = dict(
            batch_size=dl.batch_size,
            drop_last=dl.drop_last,
            num_workers=dl.num_workers,
            collate_fn=dl.collate_fn,
            pin_memory=dl.pin_memory,
        )
        if dl.batch_size is None:
            kw = dict(batch_sampler=dl.batch_sampler, num_workers=dl.num_workers, collate_fn=dl.collate_fn)
        else:
            kw["sampler"] = dl.sampler
        return self.make_loader(dl.dataset, device_placement=device_placement, **kw)

    def skip_first_batches(self, dataloader: _LoaderBase, num_batches: int = 0) -> _LoaderBase:
        return dataloader.with_skip(num_batches)

    def unwrap_model(self, model: nn.Module) -> nn.Module:
        model = unwrap(model)
        fwd = model.__dict__.get("forward")
        if fwd is not None and getattr(fwd, "_rocket_amp", False):
            pass  # keep the patched forward on the live model; state_dict is unaffected
        return model

    def replica(self, model: nn.Module) -> nn.Module:
        """Return the data-parallel wrapper of a prepared model (or the model itself)."""
        return self._wrapped.get(id(unwrap(model)), model)

    # ---------------------------------------------------- mixed precision / GA
    def autocast(self):
        if self._amp_dtype is None:
            return contextlib.nullcontext()
        return torch.autocast(device_type=self.device.type, dtype=self._amp_dtype)

    @property
    def sync_gradients(self) -> bool:
        return self.gradient_state.sync_gradients

    @sync_gradients.setter
    def sync_gradients(self, value: bool) -> None:
        self.gradient_state.sync_gradients = bool(value)

    @property
    def end_of_dataloader(self) -> bool:
        return self.gradient_state.end_of_dataloader

    def _do_sync(self) -> None:
        if self.gradient_state.end_of_dataloader:
            self.step = 0
            self.sync_gradients = True
        else:
            self.step += 1
            self.sync_gradients = (self.step % self.gradient_accumulation_steps) == 0

    @contextlib.contextmanager
    def no_sync(self, model: nn.Module):
        rep = self.replica(model)
        ctx = rep.no_sync() if isinstance(rep, DataParallel) else contextlib.nullcontext()
        with ctx:
            yield

    @contextlib.contextmanager
    def accumulate(self, *models: nn.Module):
        self._do_sync()
        with contextlib.ExitStack() as stack:
            if not self.sync_gradients:
                for m in models:
                    stack.enter_context(self.no_sync(m))
            yield

    def backward(self, loss: torch.Tensor, **kwargs) -> None:
        if self.gradient_accumulation_steps > 1:
            loss = loss / self.gradient_accumulation_steps
        if self.scaler is not None:
            self.scaler.scale(loss).backward(**kwargs)
        else:
            loss.backward(**kwargs)

    def clip_grad_norm_(self, parameters, max_norm: float, norm_type: float = 2.0):
        if self.scaler is not None:
            for o in self._optimizers:
                self.scaler.unscale_(o.optimizer)
        return torch.nn.utils.clip_grad_norm_(parameters, max_norm, norm_type=norm_type)

    # --------------------------------------------------------- collectives
    def gather(self, tensor):
        if isinstance(tensor, torch.Tensor):
            return _comm.all_gather_tensor(tensor)
        return apply_to_collection(tensor, lambda v, key=None: self.gather(v))

    def gather_for_metrics(self, input_data, use_gather_object: bool = False):
        def all_tensors(x):
            if isinstance(x, torch.Tensor):
                return True
            if is_collection(x) and not isinstance(x, (str, bytes)):
                vals = x.values() if isinstance(x, dict) else x
                return all(all_tensors(v) for v in vals)
            return False

        as_object = use_gather_object or not all_tensors(input_data)
        if as_object:
            parts = _comm.all_gather_object(input_data)
            data = [v for part in parts for v in (part if isinstance(part, list) else [part])]
        else:
            data = self.gather(input_data)
        gs = self.gradient_state
        if gs.end_of_dataloader and gs.remainder > 0 and self.num_processes > 1:
            r = gs.remainder
            if as_object:
                return data[:r]
            return apply_to_collection(data, lambda v, key=None: v[:r]) if not isinstance(data, torch.Tensor) else data[:r]
        return data

    def reduce(self, tensor, reduction: str = "sum", scale: float = 1.0):
        if isinstance(tensor, torch.Tensor):
            out = tensor.clone()
            _comm.all_reduce_(out, "mean" if reduction == "mean" else "sum")
            return out * scale if scale != 1.0 else out
        return apply_to_collection(tensor, lambda v, key=None: self.reduce(v, reduction, scale))

    # ------------------------------------------------------------ checkpoints
    def register_for_checkpointing(self, *objects) -> None:
        bad = [o for o in objects if not (hasattr(o, "state_dict") and hasattr(o, "load_state_dict"))]
        if bad:
            raise ValueError(f"objects without state_dict/load_state_dict: {bad}")
        self._custom_objects.extend(objects)

    def save_state(self, output_dir: str | None = None, **kwargs):
        if output_dir is None:
            if self.project_dir is None:
                raise ValueError("save_state needs output_dir or a project_dir")
            output_dir = os.path.join(self.project_dir, "checkpoints", f"checkpoint_{len(os.listdir(self.project_dir))}")
        return checkpoint_io.save_state(self, output_dir)

    def load_state(self, input_dir: str, load_custom: bool = True, **kwargs) -> None:
        checkpoint_io.load_state(self, input_dir, load_custom=load_custom)

    # ---------------------------------------------------------------- trackers
    def get_tracker(self, name: str, unwrap: bool = False):
        for t in self.trackers:
            if t.name == name:
                return t.tracker if unwrap else t
        return GeneralTracker(_blank=True)

    def init_trackers(self, project_name: str = "", config: dict | None = None, init_kwargs: dict | None = None):
        if not self.is_main_process:
            return
        have = {t.name for t in self.trackers}
        for name in self.log_with:
            if isinstance(name, GeneralTracker):
                if name not in self.trackers:
                    self.trackers.append(name)
                continue
            if name in have:
                continue
            t = make_tracker(name, project_name, self.logging_dir or ".")
            if config is not None:
                t.store_init_configuration(config)
            self.trackers.append(t)

    def log(self, values: dict, step: int | None = None, log_kwargs: dict | None = None) -> None:
        if self.is_main_process:
            for t in self.trackers:
                t.log(values, step=step, **(log_kwargs or {}).get(t.name, {}))

    def end_training(self) -> None:
        for t in self.trackers:
            try:
                t.finish()
            except Exception as e:  # pragma: no cover
                logger.warning(f"tracker {t.name} finish failed: {e}")
        self.trackers = []
