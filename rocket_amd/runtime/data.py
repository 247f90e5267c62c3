"""Data-parallel data path: sharded batch sampling, one-ahead loading, device datasets.

Replaces ``accelerate``'s ``BatchSamplerShard``/``DataLoaderShard``/
``skip_first_batches`` that the reference reaches via ``Dataset.setup``
(``rocket/core/dataset.py:175-180, 205-210``).

Semantics kept (they are observable through metrics and checkpoints):

* **round-robin batch sharding** – global batch *k* goes to rank ``k mod W``;
  with ``even_batches`` (default) the epoch is padded by wrapping around to the
  first indices of the epoch so every rank sees the same number of full batches
  (verified oracle: 40 samples, bs 6, W 2 → rank-0 last batch ``[36..39, 0, 1]``);
* the loader iterates **one batch ahead** so ``end_of_dataloader`` is known
  while the last batch is being consumed (GA forced sync, metric truncation);
* ``remainder = len(dataset) % (batch_size * W)`` is published for
  ``gather_for_metrics``.

MI355X-first differences:

* shuffling is **epoch-seeded** (``seed + epoch``) and identical on every rank
  by construction — no per-epoch RNG broadcast, and mid-epoch resume
  replays exactly the same permutation (fixes Q5);
* host batches are pinned and moved ``non_blocking`` while the previous step
  computes (the one-ahead slot doubles as the prefetch slot);
* :class:`DeviceTensorDataset` keeps a whole dataset resident in HBM (288 GB per
  GPU makes this the common case for vision datasets) and batches are gathered
  on-device by a precomputed per-epoch index table: no worker processes, no
  collate, no H2D copy in the hot loop.
"""

from __future__ import annotations

import math
import os
from typing import Any, Iterator, List, Optional, Sequence

import torch
from torch.utils.data import BatchSampler, DataLoader, RandomSampler, Sampler, SequentialSampler


class EpochSampler(Sampler[int]):
    """Sequential or shuffled sampler whose permutation depends only on ``(seed, epoch)``."""

    def __init__(self, data_len: int, shuffle: bool = False, seed: int = 0):
        self.data_len = int(data_len)
        self.shuffle = shuffle
        self.seed = int(seed)
        self.epoch = 0

    def set_epoch(self, epoch: int) -> None:
        self.epoch = int(epoch)

    def order(self) -> torch.Tensor:
        if not self.shuffle:
            return torch.arange(self.data_len)
        g = torch.Generator()
        g.manual_seed(self.seed * 1_000_003 + self.epoch)
        return torch.randperm(self.data_len, generator=g)

    def __iter__(self) -> Iterator[int]:
        return iter(self.order().tolist())

    def __len__(self) -> int:
        return self.data_len


def shard_batches(
    batches: List[List[int]],
    batch_size: int,
    num_replicas: int,
    rank: int,
    drop_last: bool,
    even_batches: bool = True,
) -> List[List[int]]:
    """Return the list of batches rank ``rank`` consumes in one epoch."""
    W = num_replicas
    if W == 1:
        return batches
    n = len(batches)
    if n == 0:
        return []
    if drop_last:
        return batches[: (n // W) * W][rank::W]
    if not even_batches:
        return batches[rank::W]
    full_last = len(batches[-1]) == batch_size
    if n % W == 0 and full_last:
        return batches[rank::W]
    seed_pool: List[int] = [i for b in batches[: min(W, n)] for i in b]
    while len(seed_pool) < W * batch_size:
        seed_pool = seed_pool + seed_pool
    out = [list(b) for b in batches]
    cursor = 0
    if not full_last:
        need = batch_size - len(out[-1])
        out[-1] = out[-1] + seed_pool[cursor : cursor + need]
        cursor += need
    while len(out) % W:
        out.append(seed_pool[cursor : cursor + batch_size])
        cursor += batch_size
    return out[rank::W]


class ShardedBatchSampler(Sampler[List[int]]):
    """Batch sampler with accelerate-compatible data-parallel sharding and batch skipping."""

    def __init__(
        self,
        batch_sampler: BatchSampler,
        num_replicas: int = 1,
        rank: int = 0,
        even_batches: bool = True,
        skip: int = 0,
    ):
        self.batch_sampler = batch_sampler
        self.batch_size = batch_sampler.batch_size
        self.drop_last = batch_sampler.drop_last
        self.num_replicas = num_replicas
        self.rank = rank
        self.even_batches = even_batches
        self.skip = skip

    @property
    def sampler(self):
        return self.batch_sampler.sampler

    def set_epoch(self, epoch: int) -> None:
        if hasattr(self.sampler, "set_epoch"):
            self.sampler.set_epoch(epoch)

    def local_batches(self) -> List[List[int]]:
        mine = shard_batches(
            [list(b) for b in self.batch_sampler],
            self.batch_size,
            self.num_replicas,
            self.rank,
            self.drop_last,
            self.even_batches,
        )
        return mine[self.skip :]

    def __iter__(self):
        return iter(self.local_batches())

    def _sharded_len(self) -> int:
        n = len(self.batch_sampler)
        W = self.num_replicas
        if W == 1 or n % W == 0:
            return n // W
        if self.drop_last:
            return n // W
        if self.even_batches:
            return n // W + 1
        return n // W + (1 if self.rank < n % W else 0)

    def __len__(self) -> int:
        return max(0, self._sharded_len() - self.skip)


class GradientState:
    """GA / end-of-dataloader state shared by the engine and its loaders."""

    def __init__(self, num_steps: int = 1):
        self.num_steps = num_steps
        self.sync_gradients = True
        self._loaders: List[Any] = []

    @property
    def active_dataloader(self):
        return self._loaders[-1] if self._loaders else None

    @property
    def end_of_dataloader(self) -> bool:
        dl = self.active_dataloader
        return bool(dl is not None and dl.end_of_dataloader)

    @property
    def remainder(self) -> int:
        dl = self.active_dataloader
        return dl.remainder if dl is not None else -1

    @property
    def in_dataloader(self) -> bool:
        return bool(self._loaders)

    def push(self, loader) -> None:
        self._loaders.append(loader)

    def pop(self, loader) -> None:
        if loader in self._loaders:
            self._loaders.remove(loader)


class _LoaderBase:
    """Shared epoch/one-ahead/gradient-state logic of host and device loaders."""

    def __init__(self, dataset, batch_sampler: ShardedBatchSampler, gradient_state: GradientState | None):
        self.dataset = dataset
        self.batch_sampler = batch_sampler
        self.gradient_state = gradient_state
        self.end_of_dataloader = False
        self.remainder = -1
        self.iteration = 0
        self.device: Optional[torch.device] = None

    @property
    def batch_size(self) -> int:
        return self.batch_sampler.batch_size

    @property
    def total_batch_size(self) -> int:
        return self.batch_sampler.batch_size * self.batch_sampler.num_replicas

    def set_epoch(self, epoch: int) -> None:
        self.iteration = int(epoch)
        self.batch_sampler.set_epoch(epoch)

    def __len__(self) -> int:
        return len(self.batch_sampler)

    def _begin(self) -> None:
        self.end_of_dataloader = False
        self.remainder = -1
        if not self.batch_sampler.drop_last:
            try:
                self.remainder = len(self.dataset) % self.total_batch_size
            except TypeError:
                self.remainder = -1
        if self.gradient_state is not None:
            self.gradient_state.push(self)

    def _end(self) -> None:
        if self.gradient_state is not None:
            self.gradient_state.pop(self)

    def _batches(self) -> Iterator[Any]:
        raise NotImplementedError

    def _to_device(self, batch):
        return batch

    def __iter__(self):
        self._begin()
        self.set_epoch(self.iteration)
        it = self._batches()
        try:
            current = self._to_device(next(it))
        except StopIteration:
            self._end()
            return
        while True:
            try:
                nxt = self._to_device(next(it))  # issued before `current` is consumed: overlap
            except StopIteration:
                self.end_of_dataloader = True
                yield current
                break
            yield current
            current = nxt
        self.iteration += 1
        self._end()

    def with_skip(self, num_batches: int) -> "_LoaderBase":
        raise NotImplementedError


class ShardedLoader(_LoaderBase):
    """Host dataset → (pinned) batches → device, sharded across ranks.

    Construction mirrors ``torch.utils.data.DataLoader`` kwargs
    (reference ``Dataset(dataset, **dataloader_kwargs)``).
    """

    def __init__(
        self,
        dataset,
        batch_size: int = 1,
        shuffle: bool = False,
        sampler: Sampler | None = None,
        batch_sampler: BatchSampler | None = None,
        drop_last: bool = False,
        num_replicas: int = 1,
        rank: int = 0,
        even_batches: bool = True,
        seed: int = 0,
        skip: int = 0,
        gradient_state: GradientState | None = None,
        device: torch.device | None = None,
        **loader_kwargs,
    ):
        if batch_sampler is None:
            if sampler is None or isinstance(sampler, (RandomSampler, SequentialSampler)):
                shuffle = shuffle or isinstance(sampler, RandomSampler)
                sampler = EpochSampler(len(dataset), shuffle=shuffle, seed=seed)
            batch_sampler = BatchSampler(sampler, batch_size, drop_last)
        sharded = ShardedBatchSampler(batch_sampler, num_replicas, rank, even_batches, skip)
        super().__init__(dataset, sharded, gradient_state)
        self._ctor = dict(
            batch_sampler=batch_sampler,
            num_replicas=num_replicas,
            rank=rank,
            even_batches=even_batches,
            seed=seed,
            gradient_state=gradient_state,
            device=device,
            **loader_kwargs,
        )
        if device is not None and device.type == "cuda":
            loader_kwargs.setdefault("pin_memory", True)
        self._loader_kwargs = loader_kwargs
        self.device = device
        self.base_dataloader = DataLoader(dataset, batch_sampler=sharded, **loader_kwargs)

    def _batches(self):
        return iter(self.base_dataloader)

    def _to_device(self, batch):
        if self.device is None:
            return batch
        from rocket_amd.utils.torch import torch_move

        return torch_move(batch, self.device)

    def with_skip(self, num_batches: int) -> "ShardedLoader":
        out = ShardedLoader(self.dataset, skip=num_batches, **self._ctor)
        out.set_epoch(self.iteration)
        return out


def mark_ring(sets: List[tuple]) -> None:
    """Flag a ring of persistent batch buffer sets (one tuple of tensors per slot).

    Every buffer gets ``_rocket_persistent`` (a captured step reads it in place) and
    ``_rocket_ring = (sets, slot, index)`` so the step executor can capture the graph
    variants of ALL slots in one warm-up pass instead of one per slot as they come
    round (:meth:`rocket_amd.runtime.graphs.StepGraphs.launch`).
    """
    for k, bufs in enumerate(sets):
        for j, b in enumerate(bufs):
            b._rocket_persistent = True
            b._rocket_ring = (sets, k, j)


class PendingRows:
    """A device-loader batch whose rows are not gathered yet (:class:`DeviceLoader` deferred mode).

    Attached to each of the batch's buffers as ``_rocket_pending``.  The batch's dataset rows are
    staged on the device in the loader's persistent ``rows`` buffer (indices ``rows[0:n]``), and
    after the batch an epoch cursor (``meta = {cursor, table length}``) is advanced and the NEXT
    batch's rows staged (``rk_rows_next``) — all device-side, so a captured step that consumes
    the batch consumes the next one on every replay.  Exactly one of:

    * :meth:`materialize` — a gather launch fills the buffers from ``rows``, then the advance;
    * :meth:`claim` — a consumer whose own kernels read the rows (the fused LeNet step kernel) takes
      over: they write the rows into the buffers (for every later reader), and the step's last
      kernel performs the advance (:meth:`advance_args`, then :meth:`mark_advanced`).

    ``done`` flips when the batch was gathered or claimed (at capture time: by the captured step).
    A claimed batch whose advance never ran is advanced by the loader before the next batch.
    """

    __slots__ = ("loader", "bufs", "gather", "n", "done", "advanced")

    def __init__(self, loader, bufs, gather, n):
        self.loader, self.bufs, self.gather, self.n = loader, bufs, gather, n
        self.done = self.advanced = False

    def advance_args(self):
        """(table, meta, rows, n, batch size) pointers for ``rk_rows_next`` / ``rk_mlp3_set_rows``."""
        ld = self.loader
        return ld._table.data_ptr(), ld._meta.data_ptr(), ld._rows.data_ptr(), self.n, ld._rows.numel()

    def mark_advanced(self) -> None:
        self.advanced = True

    def advance(self) -> None:
        """The advance as a launch of its own (a claimed batch whose step did not do it)."""
        if self.advanced:
            return
        self.advanced = True
        from rocket_amd.ops import _lib

        _lib.check(_lib.kernels().rk_rows_next(*self.advance_args(), _lib.stream_ptr(self.loader.device)),
                   "rk_rows_next")

    def materialize(self) -> None:
        if self.done:
            return
        self.done = True
        self.gather(self.loader._rows[: self.n])
        self.advance()

    def claim(self):
        """((image source, label source), staged rows) for a consumer that gathers the rows itself."""
        self.done = True
        return self.loader.dataset.tensors, self.loader._rows

    def rebind(self, bufs) -> "PendingRows":
        """The same pending batch on another ring slot's buffers (graph variant capture)."""
        gather = next((g for b, g in self.loader._rings.get(self.n, []) if b[0] is bufs[0]), None)
        return PendingRows(self.loader, bufs, gather, self.n)


def pending_rows(batch) -> Optional[PendingRows]:
    """The not-yet-gathered :class:`PendingRows` of a batch (tensor / tuple / list / dict), or None."""
    if isinstance(batch, torch.Tensor):
        p = getattr(batch, "_rocket_pending", None)
        return p if (p is not None and not p.done and any(b is batch for b in p.bufs)) else None
    if isinstance(batch, dict):
        batch = list(batch.values())
    if isinstance(batch, (list, tuple)):
        for b in batch:
            p = pending_rows(b)
            if p is not None:
                return p
    return None


def materialize_batch(batch) -> None:
    """Gather a deferred device-loader batch now (no-op for ordinary batches)."""
    p = pending_rows(batch)
    if p is not None:
        p.materialize()


class DeviceTensorDataset(torch.utils.data.Dataset):
    """A dataset of aligned tensors resident on one device (typically HBM).

    Indexing returns a tuple of per-sample views, so it is also usable by host
    loaders; :class:`DeviceLoader` batches it with on-device gathers instead.

    ``pre_sharded=True``: the tensors are THIS rank's shard only (each rank generated or loaded
    its own part, e.g. synthetic benchmark data): the loader batches all of it locally instead of
    taking every W-th batch of a global set, so no rank holds the other ranks' samples.  Every rank
    must then hold the same number of samples (equal batch counts keep the ranks in step).
    """

    def __init__(self, *tensors: torch.Tensor, pre_sharded: bool = False):
        if not tensors:
            raise ValueError("DeviceTensorDataset needs at least one tensor")
        n = tensors[0].shape[0]
        if any(t.shape[0] != n for t in tensors):
            raise ValueError("all tensors must share their first dimension")
        self.tensors = tensors
        self.pre_sharded = bool(pre_sharded)

    @property
    def device(self) -> torch.device:
        return self.tensors[0].device

    def __len__(self) -> int:
        return self.tensors[0].shape[0]

    def __getitem__(self, i):
        return tuple(t[i] for t in self.tensors)


class DeviceLoader(_LoaderBase):
    """Loader over a :class:`DeviceTensorDataset`: per-epoch index table, on-device gathers.

    On a HIP device every batch is assembled by ONE native gather launch
    (all dataset tensors at once) into a small ring of persistent batch
    buffers (``RING`` deep, per batch size).  The buffers carry
    ``_rocket_persistent`` so a captured training step reads them in place —
    no per-step copy into static graph inputs.  Consequently a yielded batch
    stays valid for ``RING - 1`` further batches; clone it to keep it longer.
    """

    RING = 4
    #: ROCKET_PREFETCH=1: gather each batch on a side stream, overlapped with the previous step.
    #: Ordering: the gather into ring slot k waits for the step that last read slot k (an event
    #: recorded on the compute stream RING-1 batches earlier), and the compute stream waits for the
    #: gather before the step that reads it.  Off by default: on the LeNet step (4.6 us gather,
    #: 55 us step) the cross-queue event wait costs more than the overlap saves (17.3M -> 13.7M
    #: samples/s measured on 1x MI355X).
    PREFETCH = os.environ.get("ROCKET_PREFETCH", "0") == "1"
    #: ROCKET_GATHER_ANY_ORDER=0 disables: batch gathers are launched without the AQL barrier bit, so
    #: a gather overlaps the tail kernel of the step queued before it instead of adding a dependent
    #: dispatch to the chain.  Safe because the loader gathers one batch ahead into a ring slot that
    #: no in-flight step reads (the slot's last reader is RING - 1 steps back, and every packet but
    #: the immediately preceding one has completed when the gather starts), and because the first
    #: gather after an index-table upload keeps the barrier (it reads the uploaded table).
    ANY_ORDER = os.environ.get("ROCKET_GATHER_ANY_ORDER", "1") != "0"
    #: deferred mode (``defer = True``, set by the Looper when the consumer of the batches is a
    #: model that gathers its own rows, see :class:`PendingRows`): batches are yielded as ring
    #: slots still to be filled, and the row indices live in a persistent device table read through
    #: a device-side cursor.  ROCKET_DEFER_GATHER=0 disables it.
    DEFER = os.environ.get("ROCKET_DEFER_GATHER", "1") != "0"

    def __init__(
        self,
        dataset: DeviceTensorDataset,
        batch_size: int = 1,
        shuffle: bool = False,
        drop_last: bool = False,
        num_replicas: int = 1,
        rank: int = 0,
        even_batches: bool = True,
        seed: int = 0,
        skip: int = 0,
        gradient_state: GradientState | None = None,
        **unused,
    ):
        sampler = EpochSampler(len(dataset), shuffle=shuffle, seed=seed)
        bs = BatchSampler(sampler, batch_size, drop_last)
        if getattr(dataset, "pre_sharded", False):  # already this rank's shard: batch all of it
            num_replicas, rank = 1, 0
        super().__init__(dataset, ShardedBatchSampler(bs, num_replicas, rank, even_batches, skip), gradient_state)
        self._ctor = dict(
            batch_size=batch_size,
            shuffle=shuffle,
            drop_last=drop_last,
            num_replicas=num_replicas,
            rank=rank,
            even_batches=even_batches,
            seed=seed,
            gradient_state=gradient_state,
        )
        self.device = dataset.device
        self._rings: dict = {}
        self._ring_pos: dict = {}
        self._fresh_table = True  # the next gather reads a just-uploaded index table
        self.defer = False
        self._table = self._meta = self._rows = None
        self._last_pending: Optional[PendingRows] = None

    def index_table(self) -> List[torch.Tensor]:
        batches = self.batch_sampler.local_batches()
        if not batches:
            return []
        lens = [len(b) for b in batches]
        flat = torch.tensor([i for b in batches for i in b], dtype=torch.int64)
        if self.device.type == "cuda":
            flat = flat.pin_memory().to(self.device, non_blocking=True)
        return list(torch.split(flat, lens))

    device_resident = True  # batches are produced on the dataset's device: no torch_move needed

    def _gather(self, idx: torch.Tensor):
        tensors = self.dataset.tensors
        if self.device.type != "cuda":
            return tuple(t.index_select(0, idx) for t in tensors)
        from rocket_amd.ops.data import RowGather

        n = idx.numel()
        ring = self._rings.get(n)
        if ring is None:
            ring = []
            for _ in range(self.RING):
                bufs = tuple(torch.empty((n,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device) for t in tensors)
                ring.append((bufs, RowGather([t.contiguous() for t in tensors], bufs)))
            mark_ring([bufs for bufs, _ in ring])
            self._rings[n] = ring
        k = self._ring_pos.get(n, 0)
        self._ring_pos[n] = (k + 1) % self.RING
        bufs, gather = ring[k]
        if not self.PREFETCH or torch.cuda.is_current_stream_capturing():
            any_order = (self.ANY_ORDER and not self._fresh_table and self.RING >= 3
                         and not torch.cuda.is_current_stream_capturing())
            self._fresh_table = False
            gather(idx, any_order=any_order)
            return bufs
        compute = torch.cuda.current_stream(self.device)
        side = self._side_stream()
        # compute has queued every step up to the previous batch: mark that point; the gather into
        # slot k may start once the step of batch j - RING (the last reader of slot k) is done
        mark = torch.cuda.Event()
        mark.record(compute)
        self._marks.append(mark)
        if len(self._marks) >= self.RING:
            side.wait_event(self._marks[-self.RING])
        if len(self._marks) > self.RING:
            self._marks.pop(0)
        if self._idx_ready is not None:  # this epoch's index table was uploaded on the compute stream
            side.wait_event(self._idx_ready)
            self._idx_ready = None
        with torch.cuda.stream(side):
            gather(idx)
        done = torch.cuda.Event()
        done.record(side)
        compute.wait_event(done)
        return bufs

    def _deferred(self, n: int):
        """Deferred mode: the next ring slot, tagged with its :class:`PendingRows`.  A previous
        batch nobody gathered (consumed neither by a claiming model nor by a materialising reader)
        is gathered first, so the device cursor stays in step with the batches handed out."""
        last = self._last_pending
        if last is not None:
            if not last.done:
                last.materialize()
            elif not last.advanced:
                last.advance()  # claimed, but the consuming step's advance never ran
        bufs, gather = self._slot(n)
        p = PendingRows(self, bufs, gather, n)
        for b in bufs:
            b._rocket_pending = p
        self._last_pending = p
        return bufs

    def _slot(self, n: int):
        from rocket_amd.ops.data import RowGather

        ring = self._rings.get(n)
        if ring is None:
            tensors = self.dataset.tensors
            ring = []
            for _ in range(self.RING):
                bufs = tuple(torch.empty((n,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device) for t in tensors)
                ring.append((bufs, RowGather([t.contiguous() for t in tensors], bufs)))
            mark_ring([bufs for bufs, _ in ring])
            self._rings[n] = ring
        k = self._ring_pos.get(n, 0)
        self._ring_pos[n] = (k + 1) % self.RING
        return ring[k]

    def _upload_table(self, batches) -> int:
        """Deferred mode: this epoch's row order into the persistent device table, cursor 0 and the
        first batch's rows staged (host-to-device copies, ordered before the epoch's first step)."""
        flat = [i for b in batches for i in b]
        self._ensure_table()
        if len(flat) > self._table.numel():
            raise RuntimeError("deferred device loader: epoch row table larger than its capacity")
        host = torch.tensor(flat + [0, len(flat)], dtype=torch.int64).pin_memory()
        if flat:
            self._table[: len(flat)].copy_(host[: len(flat)], non_blocking=True)
            k = min(len(flat), self._rows.numel())
            self._rows[:k].copy_(host[:k], non_blocking=True)
        self._meta.copy_(host[len(flat):], non_blocking=True)
        self._table_host = host  # pinned source alive until the copies ran
        return len(flat)

    def _ensure_table(self) -> None:
        """Allocate the persistent row table, cursor and staged rows once: captured steps keep their
        addresses, so a loader and its ``with_skip`` copies (a resumed epoch) must share them."""
        if self._table is None:
            cap = len(self.dataset) + 2 * self.total_batch_size  # even_batches may repeat a few rows
            self._table = torch.zeros(cap, dtype=torch.int64, device=self.device)
            self._meta = torch.zeros(2, dtype=torch.int64, device=self.device)  # cursor, table length
            self._rows = torch.zeros(self.batch_size, dtype=torch.int64, device=self.device)

    def __iter__(self):
        if not (self.defer and self.DEFER and self.device.type == "cuda"):
            yield from super().__iter__()
            return
        # deferred: no gather one batch ahead (the consumer gathers each batch in its own step)
        self._begin()
        self.set_epoch(self.iteration)
        batches = self.batch_sampler.local_batches()
        self._upload_table(batches)
        self._last_pending = None
        for i, b in enumerate(batches):
            if i == len(batches) - 1:
                self.end_of_dataloader = True
            yield self._deferred(len(b))
        last = self._last_pending
        if last is not None:
            if not last.done:
                last.materialize()
            elif not last.advanced:
                last.advance()
        self.iteration += 1
        self._end()

    def _side_stream(self):
        if getattr(self, "_side", None) is None:
            self._side = torch.cuda.Stream(self.device)
            self._marks = []
            self._idx_ready = None
        return self._side

    def _batches(self):
        table = self.index_table()
        self._fresh_table = True
        if table and self.PREFETCH and self.device.type == "cuda":
            self._side_stream()
            self._idx_ready = torch.cuda.Event()
            self._idx_ready.record(torch.cuda.current_stream(self.device))
        for idx in table:
            yield self._gather(idx)

    def with_skip(self, num_batches: int) -> "DeviceLoader":
        out = DeviceLoader(self.dataset, skip=num_batches, **self._ctor)
        out.set_epoch(self.iteration)
        out._rings, out._ring_pos = self._rings, self._ring_pos  # same buffers -> same captured graphs
        out.defer = self.defer
        if self.device.type == "cuda":
            self._ensure_table()
        out._table, out._meta, out._rows = self._table, self._meta, self._rows
        return out


def num_batches(n: int, batch_size: int, drop_last: bool, world: int, even: bool = True) -> int:
    """Batches per rank per epoch for a dataset of ``n`` samples."""
    b = n // batch_size if drop_last else math.ceil(n / batch_size)
    if world == 1 or b % world == 0 or drop_last:
        return b // world
    return b // world + 1 if even else b // world
