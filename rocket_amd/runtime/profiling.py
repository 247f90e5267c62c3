"""Step timing and trace markers (SURVEY §5 "Tracing / profiling": absent in the reference).

* :class:`StepTimer` — a capsule placed last in a Looper (priority 1).  It
  records a HIP event at every iteration boundary (no host sync inside the
  loop) and can bracket a measurement window with a barrier + device sync on
  both sides, which is the protocol ``bench.py`` reports.  After the loop the
  per-step device times give p50/p90 without perturbing the steady state.
* :func:`range_push`/:func:`range_pop` — roctx ranges (``libroctx64``) around
  step phases so ``rocprofv3 --marker-trace`` timelines are readable; no-ops
  when the library is unavailable.
"""

from __future__ import annotations

import ctypes
import statistics
import time
from typing import List, Optional

import torch

from rocket_amd.core.attributes import Attributes
from rocket_amd.core.capsule import Capsule
from rocket_amd.runtime import comm as _comm

_roctx = None


def _load_roctx():
    global _roctx
    if _roctx is None:
        try:
            _roctx = ctypes.CDLL("libroctx64.so")
            _roctx.roctxRangePushA.argtypes = [ctypes.c_char_p]
        except OSError:
            _roctx = False
    return _roctx


def range_push(name: str) -> None:
    lib = _load_roctx()
    if lib:
        lib.roctxRangePushA(name.encode())


def range_pop() -> None:
    lib = _load_roctx()
    if lib:
        lib.roctxRangePop()


def sync_all(device: torch.device) -> None:
    """Barrier over ranks with device idle on both sides."""
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    _comm.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize(device)


class StepTimer(Capsule):
    """Measure a window of ``steps`` iterations after ``warmup`` iterations.

    ``stride``: record a timing event every ``stride`` iterations (step times are then the
    per-iteration means of stride-long groups).  A timing event is not free on ROCm (≈5 µs of
    queue time next to a graph replay), which matters for ~80 µs LeNet steps.
    """

    def __init__(self, warmup: int = 0, steps: Optional[int] = None, priority: int = 1, stride: int = 1):
        super().__init__(priority=priority)
        self.warmup = warmup
        self.steps = steps
        self.stride = max(1, int(stride))
        self._i = 0
        self._events: List = []
        self._host: List[float] = []
        self._pool = None
        self.t_start: Optional[float] = None
        self.t_end: Optional[float] = None

    def _mark(self) -> None:
        if self._pool is not None:
            ev = self._pool[len(self._events)] if len(self._events) < len(self._pool) else torch.cuda.Event(
                enable_timing=True)
            ev.record()
            self._events.append(ev)
        self._host.append(time.perf_counter())

    def setup(self, attrs: Attributes | None = None) -> None:
        Capsule.setup(self, attrs)
        # timing events are created up front: constructing one costs more than recording it
        self._pool = None
        if self._accelerator.device.type == "cuda":
            n = (self.steps // self.stride + 2) if self.steps is not None else 1024
            self._pool = [torch.cuda.Event(enable_timing=True) for _ in range(n)]

    def set(self, attrs: Attributes | None = None) -> None:
        if self.warmup == 0 and self.t_start is None:
            self.start_now()

    def launch(self, attrs: Attributes | None = None) -> None:
        self._i += 1
        dev = self._accelerator.device
        if self._i == self.warmup:
            sync_all(dev)
            self.t_start = time.perf_counter()
            self._mark()
        elif self._i > self.warmup and (self.steps is None or self._i <= self.warmup + self.steps):
            last = self.steps is not None and self._i == self.warmup + self.steps
            if (self._i - self.warmup) % self.stride == 0 or last:
                self._mark()
            if last:
                sync_all(dev)
                self.t_end = time.perf_counter()

    def start_now(self) -> None:
        """Start the window before the first iteration (warmup == 0)."""
        sync_all(self._accelerator.device)
        self.t_start = time.perf_counter()
        self._mark()

    @property
    def elapsed(self) -> float:
        return (self.t_end or time.perf_counter()) - (self.t_start or 0.0)

    def _group_sizes(self) -> List[int]:
        """Iterations between consecutive marks (``stride``, the last group possibly shorter)."""
        n = len(self._host) - 1
        if self.steps is None:
            return [self.stride] * n
        sizes = [self.stride] * (self.steps // self.stride)
        if self.steps % self.stride:
            sizes.append(self.steps % self.stride)
        return sizes[:n] + [self.stride] * max(0, n - len(sizes))

    def step_times_ms(self) -> List[float]:
        """Per-iteration times (ms): one value per mark interval, divided by its iteration count."""
        sizes = self._group_sizes()
        if self._events:
            torch.cuda.synchronize()
            return [a.elapsed_time(b) / k for a, b, k in zip(self._events[:-1], self._events[1:], sizes)]
        return [(b - a) * 1e3 / k for a, b, k in zip(self._host[:-1], self._host[1:], sizes)]

    def host_ms_p50(self) -> float:
        """Median host-side time per iteration between marks: how fast the host enqueues.  When the
        GPU is the bottleneck the host runs ahead until the device queue is full and is then paced by
        the GPU (each enqueue waits for queue space), so this approaches the step time; it measures
        host cost only when it is well below the step time.  :meth:`host_issue_ms` is the unpaced
        cost."""
        h = [(b - a) * 1e3 / k for a, b, k in zip(self._host[:-1], self._host[1:], self._group_sizes())]
        return statistics.median(h) if h else 0.0

    def host_issue_ms(self) -> float:
        """Host time per iteration of the first timed group, which starts right after the warmup's
        device synchronisation (an empty queue): the host's own cost to issue a step, before any
        queue back-pressure (per-iteration mean over the group)."""
        if len(self._host) < 2:
            return 0.0
        return (self._host[1] - self._host[0]) * 1e3 / self._group_sizes()[0]

    def summary(self) -> dict:
        t = self.step_times_ms()
        if not t:
            return {}
        t_sorted = sorted(t)
        return {
            "host_ms_p50": self.host_ms_p50(),
            "host_issue_ms": self.host_issue_ms(),
            "step_ms_p50": statistics.median(t),
            "step_ms_p90": t_sorted[min(len(t) - 1, int(0.9 * len(t)))],
            "step_ms_min": t_sorted[0],
            "step_ms_mean": sum(t) / len(t),
            "step_ms_max": t_sorted[-1],
            "step_ms_max_at": t.index(t_sorted[-1]) * self.stride,  # iteration (within the timed run)
        }
