"""Host-resident datasets batched by the native C++ gather pool (``native/runtime/loader.cpp``).

:class:`HostTensorDataset` holds aligned row-major host tensors (e.g. a uint8/bf16 image array
too large for HBM, or any dataset on a CPU-only run).  :class:`HostLoader` replaces the
reference's ``DataLoader`` workers + ``collate`` + blocking ``.to(device)``:

* batch ``k+1`` (and ``k+2``) are gathered by C++ threads into PINNED staging slots while
  batch ``k`` is copied and consumed — no Python per sample, no worker processes;
* each staged batch is copied to the device with one ``non_blocking`` copy per tensor on a
  dedicated copy stream; the compute stream waits on an event (no host sync); device batches
  live in a small ring of persistent buffers (``_rocket_persistent``) so a captured training
  step reads them in place;
* sharding, epoch-seeded shuffling, ``even_batches`` padding, one-ahead ``end_of_dataloader``
  and ``skip`` are the shared semantics of :class:`~rocket_amd.runtime.data._LoaderBase`.
"""

from __future__ import annotations

import ctypes
import os
from typing import List

import torch
from torch.utils.data import BatchSampler

from rocket_amd.runtime.data import EpochSampler, GradientState, ShardedBatchSampler, _LoaderBase, mark_ring


class HostTensorDataset(torch.utils.data.Dataset):
    def __init__(self, *tensors: torch.Tensor):
        if not tensors:
            raise ValueError("HostTensorDataset needs at least one tensor")
        n = tensors[0].shape[0]
        if any(t.shape[0] != n for t in tensors):
            raise ValueError("all tensors must share their first dimension")
        if any(t.device.type != "cpu" for t in tensors):
            raise ValueError("HostTensorDataset tensors live in host memory")
        self.tensors = tuple(t.contiguous() for t in tensors)

    def __len__(self) -> int:
        return self.tensors[0].shape[0]

    def __getitem__(self, i):
        return tuple(t[i] for t in self.tensors)


class _NativeGather:
    def __init__(self, tensors, nthreads: int, nslots: int):
        from rocket_amd.runtime.native import check, runtime

        self.rt = runtime()
        self.tensors = tensors
        k = len(tensors)
        self._bases = (ctypes.c_void_p * k)(*[t.data_ptr() for t in tensors])
        self._rb = (ctypes.c_int64 * k)(*[t[0].numel() * t.element_size() if t.shape[0] else 0 for t in tensors])
        h = ctypes.c_void_p()
        check(self.rt.rkl_create(ctypes.byref(h), k, self._bases, self._rb, tensors[0].shape[0], nthreads, nslots),
              "rkl_create")
        self.h = h

    def submit(self, slot: int, idx: torch.Tensor, outs: List[torch.Tensor]) -> None:
        from rocket_amd.runtime.native import check

        dst = (ctypes.c_void_p * len(outs))(*[o.data_ptr() for o in outs])
        check(self.rt.rkl_submit(self.h, slot, idx.data_ptr(), idx.numel(), dst), "rkl_submit")

    def wait(self, slot: int) -> None:
        self.rt.rkl_wait(self.h, slot)

    def close(self) -> None:
        if self.h is not None:
            self.rt.rkl_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HostLoader(_LoaderBase):
    RING = 4      # device batch buffers (a yielded batch stays valid for RING - 1 more batches)
    AHEAD = 2     # batches staged ahead of the one being consumed

    def __init__(self, dataset: HostTensorDataset, batch_size: int = 1, shuffle: bool = False,
                 drop_last: bool = False, num_replicas: int = 1, rank: int = 0, even_batches: bool = True,
                 seed: int = 0, skip: int = 0, gradient_state: GradientState | None = None,
                 device: torch.device | None = None, num_threads: int | None = None, **unused):
        sampler = EpochSampler(len(dataset), shuffle=shuffle, seed=seed)
        bs = BatchSampler(sampler, batch_size, drop_last)
        super().__init__(dataset, ShardedBatchSampler(bs, num_replicas, rank, even_batches, skip), gradient_state)
        self._ctor = dict(batch_size=batch_size, shuffle=shuffle, drop_last=drop_last, num_replicas=num_replicas,
                          rank=rank, even_batches=even_batches, seed=seed, gradient_state=gradient_state,
                          device=device, num_threads=num_threads)
        self.device = device if device is not None else torch.device("cpu")
        self.device_resident = device is not None
        self._threads = num_threads or max(1, min(8, (os.cpu_count() or 2) // 2))
        self._gather = None
        self._staging: dict = {}
        self._ring: dict = {}
        self._ring_pos: dict = {}
        self._copy_stream = None

    # ------------------------------------------------------------------ buffers
    def _native(self) -> _NativeGather:
        if self._gather is None:
            self._gather = _NativeGather(self.dataset.tensors, self._threads, self.AHEAD + 1)
        return self._gather

    def _stage(self, slot: int, n: int) -> List[torch.Tensor]:
        key = (slot, n)
        bufs = self._staging.get(key)
        if bufs is None:
            pin = self.device.type == "cuda"
            bufs = [torch.empty((n,) + tuple(t.shape[1:]), dtype=t.dtype, pin_memory=pin) for t in self.dataset.tensors]
            self._staging[key] = bufs
        return bufs

    def _device_buffers(self, n: int):
        ring = self._ring.get(n)
        if ring is None:
            ring = []
            for _ in range(self.RING):
                bufs = tuple(torch.empty((n,) + tuple(t.shape[1:]), dtype=t.dtype, device=self.device)
                             for t in self.dataset.tensors)
                ring.append(bufs)
            mark_ring(ring)
            self._ring[n] = ring
        k = self._ring_pos.get(n, 0)
        self._ring_pos[n] = (k + 1) % self.RING
        return ring[k]

    # ------------------------------------------------------------------ iteration
    def _batches(self):
        batches = self.batch_sampler.local_batches()
        if not batches:
            return
        g = self._native()
        idx = [torch.tensor(b, dtype=torch.int64) for b in batches]
        nslots = self.AHEAD + 1
        events = [None] * nslots
        for k in range(min(nslots, len(idx))):
            g.submit(k, idx[k], self._stage(k, idx[k].numel()))
        cuda = self.device.type == "cuda"
        if cuda and self._copy_stream is None:
            self._copy_stream = torch.cuda.Stream(device=self.device)
        for k in range(len(idx)):
            slot = k % nslots
            n = idx[k].numel()
            g.wait(slot)
            staged = self._stage(slot, n)
            if cuda:
                out = self._device_buffers(n)
                cs = self._copy_stream
                cur = torch.cuda.current_stream(self.device)
                cs.wait_stream(cur)  # the ring buffer's previous reader has been enqueued before
                with torch.cuda.stream(cs):
                    for o, s in zip(out, staged):
                        o.copy_(s, non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(cs)
                cur.wait_event(ev)
                events[slot] = ev
            else:
                out = tuple(s.clone() for s in staged)
            nxt = k + nslots
            if nxt < len(idx):
                if events[slot] is not None:
                    events[slot].synchronize()  # staging slot is free once its H2D copy ran
                g.submit(slot, idx[nxt], self._stage(slot, idx[nxt].numel()))
            yield out

    def with_skip(self, num_batches: int) -> "HostLoader":
        out = HostLoader(self.dataset, skip=num_batches, **self._ctor)
        out.set_epoch(self.iteration)
        out._gather, out._staging, out._ring, out._ring_pos = self._gather, self._staging, self._ring, self._ring_pos
        out._copy_stream = self._copy_stream
        return out
