"""The buffered label datasets of the reference's data module (picard/dataset.py), with the label
store kept in HBM.

`IterableDatasetWithInternalBatch` is the boundary the label path sits behind:
the reference's `PicardDataModule` builds it from a generator's `dataset_with_gradients`
(picard/data.py:291-297, selected in `get_dataset_details`, :1620-1661) and pulls batches from it.
Here the generator is `deeppicarditeration_amd.data.OnlineDataGenerator`, whose
`sample_with_gradients` returns device tensors, so every buffer, every cached copy and every
yielded batch stays on the GPU:

- `DeviceMemorySaver` replaces `InMemorySaver` (picard/data_saver.py:69-83), which copied every
  label to host memory and back;
- `TensorDatasetBuiltInShuffle` batches the cached labels with one device gather per batch instead
  of a DataLoader over a TensorDataset (picard/data_saver.py:58-66);
- `CacheToFileWrapper` writes the reference's H5 files through `h5.H5Saver`.
"""
import math
from typing import Optional, Sequence, Tuple, Union

import torch
from torch.utils.data import IterableDataset

from . import h5


class Saver:
    """picard/data_saver.py:10-21."""

    def save(self, data: Sequence[torch.Tensor], length: int):
        raise NotImplementedError

    def close(self):
        pass


class DeviceMemorySaver(Saver):
    """InMemorySaver (picard/data_saver.py:69-83) holding the rows where they were produced: the
    (n_total, d) stores are allocated on the first save, on that batch's device and dtype."""

    def __init__(self, n_total: int, n_dims: Sequence[int]):
        self.n_total = int(n_total)
        self.n_dims = [int(d) for d in n_dims]
        self.position = 0
        self.data = None

    def save(self, data: Sequence[torch.Tensor], length: int):
        if self.data is None:
            self.data = [torch.empty(self.n_total, d, dtype=x.dtype, device=x.device)
                         for d, x in zip(self.n_dims, data)]
        if self.position + length > self.n_total:
            raise ValueError(f"saver holds {self.n_total} rows; {self.position} + {length} would overflow it")
        for store, x in zip(self.data, data):
            store[self.position:self.position + length] = x
        self.position += length

    def create_torch_dataset(self, batch_size: int, **dataloader_kwargs):
        if self.data is None or self.position < self.n_total:
            raise ValueError("Not all data are filled.")
        return TensorDatasetBuiltInShuffle(*self.data, batch_size=batch_size, **dataloader_kwargs)


class TensorDatasetBuiltInShuffle(IterableDataset):
    """Mini-batches over cached tensors (picard/data_saver.py:58-66: a DataLoader with `batch_size`,
    `shuffle`, `drop_last`).  The permutation is drawn on the tensors' device from torch's global
    generator for that device, once per pass, and each batch is one `index_select` per tensor."""

    def __init__(self, *tensors, batch_size: int, shuffle: bool = False, drop_last: bool = False, **unused):
        n = tensors[0].shape[0]
        if any(t.shape[0] != n for t in tensors):
            raise ValueError("Size mismatch between tensors")
        self.tensors = tensors
        self.batch_size = int(batch_size)
        self.shuffle = bool(shuffle)
        self.drop_last = bool(drop_last)

    def __len__(self):
        n = self.tensors[0].shape[0]
        return n // self.batch_size if self.drop_last else math.ceil(n / self.batch_size)

    def __iter__(self):
        n = self.tensors[0].shape[0]
        dev = self.tensors[0].device
        order = torch.randperm(n, device=dev) if self.shuffle else None
        for b in range(len(self)):
            lo, hi = b * self.batch_size, min(n, (b + 1) * self.batch_size)
            if order is None:
                yield [t[lo:hi] for t in self.tensors]
            else:
                idx = order[lo:hi]
                yield [t.index_select(0, idx) for t in self.tensors]


def buffer_plan(n_batch_buffer: Union[int, float], batch_size: int) -> Tuple[int, int, int, int]:
    """How one buffer is produced (picard/dataset.py:55-77): (batches per buffer, samples per
    buffer, generator calls per buffer, samples per call).  An integral `n_batch_buffer` (within
    1e-5) means one call producing that many batches; a fraction f in (0, 1) means 1/f calls each
    producing batch_size·f samples, which together make one batch."""
    if abs(round(n_batch_buffer) - n_batch_buffer) < 1e-5:
        n_batch_buffer = round(n_batch_buffer)
    if isinstance(n_batch_buffer, int):
        if n_batch_buffer < 1:
            raise AssertionError(f"n_batch_buffer must be >= 1 or a fraction in (0, 1) (got {n_batch_buffer})")
        return n_batch_buffer, n_batch_buffer * batch_size, 1, n_batch_buffer * batch_size
    if not (isinstance(n_batch_buffer, float) and 0 < n_batch_buffer < 1):
        raise AssertionError(f"n_batch_buffer must be an integer or a fraction in (0, 1) (got {n_batch_buffer})")
    calls = round(1 / n_batch_buffer)
    per_call = batch_size // calls
    if per_call * calls != batch_size:
        raise AssertionError(f"batch_size {batch_size} must be a multiple of "
                             f"n_calls_to_generator_each_buffer {calls}")
    return 1, batch_size, calls, per_call


class IterableDatasetWithInternalBatch(IterableDataset):
    """picard/dataset.py:20-137: yields `batch_size`-row batches cut from buffers, each buffer made
    by `batch_data_generator(n) -> (x (n, ·), y (n, ·))` calls.  Use with `DataLoader(batch_size=None)`.
    `n` must be a multiple of the samples per buffer.

    `range_guard` (the OnlineDataGenerator whose label calls fill the buffers): each buffer's calls
    run in one of its RangeGroups, and buffer k is yielded (and saved) only after its group
    verified, which happens once buffer k+1's calls are enqueued — so the check waits on work the
    GPU finished while it already runs the next buffer, instead of synchronising after every call.
    The buffers are drawn in the same order either way (buffer k+1 is drawn one buffer earlier);
    an iteration abandoned early (break, islice) discards the buffer drawn ahead unread and rewinds
    the generator's point counter by its points, so later draws see the counters they would have
    seen without the guard."""

    def __init__(self, n: int, n_batch_buffer: Union[int, float], batch_size: int, batch_data_generator,
                 range_guard=None):
        super().__init__()
        self.range_guard = range_guard
        (self.n_batch_buffer, self.n_samples_each_buffer, self._n_calls_to_generator_each_buffer,
         self._n_samples_each_call) = buffer_plan(n_batch_buffer, batch_size)
        self.batch_size = int(batch_size)
        self.batch_data_generator = batch_data_generator
        self.n_buffer_refresh = self._get_n_refresh(n)
        self.saver: Optional[Saver] = None

    def _get_n_refresh(self, n: int) -> int:
        k = int(n) // self.n_samples_each_buffer
        if k * self.n_samples_each_buffer != int(n):
            raise AssertionError(f"Total number of data {n} must be a multiple of batch_size({self.batch_size})"
                                 f"*n_batch_buffer({self.n_batch_buffer})={self.n_samples_each_buffer}")
        return k

    def set_size(self, n: int):
        self.n_buffer_refresh = self._get_n_refresh(n)

    def attach_saver(self, saver: Saver):
        if self.saver is not None:
            raise AssertionError("Saver can only be attached once")
        self.saver = saver

    def _calls(self):
        xs, ys = [], []
        for _ in range(self._n_calls_to_generator_each_buffer):
            x, y = self.batch_data_generator(self._n_samples_each_call)[:2]
            xs.append(x)
            ys.append(y)
        return xs, ys

    @staticmethod
    def _joined(xs, ys):
        if len(xs) == 1:
            return xs[0], ys[0]
        return torch.cat(xs, 0), torch.cat(ys, 0)

    def refresh_buffer(self):
        """One buffer: the generator calls' rows concatenated in call order (:110-118)."""
        return self._joined(*self._calls())

    def _emit(self, x, y):
        if self.saver is not None:
            self.saver.save((x, y), self.n_samples_each_buffer)
        x = x.view(self.n_batch_buffer, self.batch_size, -1)
        y = y.view(self.n_batch_buffer, self.batch_size, -1)
        for b in range(self.n_batch_buffer):
            yield x[b], y[b]

    def __iter__(self):
        if self.range_guard is None:
            for _ in range(self.n_buffer_refresh):
                yield from self._emit(*self.refresh_buffer())
        else:
            pending = None  # (group, xs, ys, point counter before its draws) of the buffer drawn, not yet verified
            gen = self.range_guard
            try:
                for _ in range(self.n_buffer_refresh):
                    pb0 = getattr(gen, "point_base", None)
                    with gen.deferred_range_check() as grp:
                        xs, ys = self._calls()
                    prev, pending = pending, (grp, xs, ys, pb0)
                    if prev is not None:
                        g, pxs, pys, _ = prev
                        g.verify()  # joined after the check: a repair writes the calls' own outputs
                        yield from self._emit(*self._joined(pxs, pys))
                if pending is not None:
                    (g, pxs, pys, _), pending = pending, None
                    g.verify()
                    yield from self._emit(*self._joined(pxs, pys))
            finally:
                if pending is not None:  # iteration abandoned: the drawn buffer is dropped unread
                    pending[0].discard()
                    if pending[3] is not None:  # and its points' counters handed back
                        gen.point_base = pending[3]
        if self.saver is not None:
            self.saver.close()

    def __len__(self):
        """Number of batches (internal batching: the DataLoader sees batches, :129-137)."""
        return self.n_buffer_refresh * self.n_batch_buffer


def _preload(dataset: IterableDatasetWithInternalBatch):
    """picard/dataset.py:140-150: run the generator over the whole dataset (filling its saver)."""
    for _ in dataset:
        pass


class CacheToMemoryWrapper(IterableDataset):
    """picard/dataset.py:203-255: the first pass streams from the generator while a saver records
    every buffer; later passes (multi-epoch fits) iterate the cached labels in (shuffled) batches.
    The cache is `DeviceMemorySaver`: labels never leave HBM."""

    def __init__(self, dataset: IterableDatasetWithInternalBatch, batch_size: int = None, **dataloader_kwargs):
        self.dataset = dataset
        self.saver: Optional[DeviceMemorySaver] = None
        self.dataset_from_memory: Optional[TensorDatasetBuiltInShuffle] = None
        self.on_gen_stage = True
        self.batch_size = batch_size or dataset.batch_size
        self.batch_size_modified = self.batch_size != dataset.batch_size
        self.dataloader_kwargs = dataloader_kwargs
        self.len = len(dataset)
        self.h5_saver_args = None

    def init(self, n_total: int, n_dims: Sequence[int], preload: bool = False):
        self.dataset.set_size(n_total)
        self.saver = DeviceMemorySaver(n_total, n_dims)
        self.dataset.attach_saver(self.saver)
        if preload or self.batch_size_modified or self.h5_saver_args is not None:
            _preload(self.dataset)
            self.dataset_from_memory = self.saver.create_torch_dataset(self.batch_size, **self.dataloader_kwargs)
            self.len = len(self.dataset_from_memory)
            self.on_gen_stage = False
            if self.h5_saver_args is not None:
                saver = h5.H5Saver(*self.h5_saver_args)
                saver.save(self.saver.data, self.saver.position)
                saver.close()

    def enable_save_to_file(self, h5_saver_args):
        self.h5_saver_args = h5_saver_args

    def __iter__(self):
        if self.saver is None:
            raise AssertionError("Must call init() before using the iterator")
        if self.on_gen_stage:
            self.on_gen_stage = False
            return iter(self.dataset)
        if self.dataset_from_memory is None:
            self.dataset_from_memory = self.saver.create_torch_dataset(self.batch_size, **self.dataloader_kwargs)
            self.len = len(self.dataset_from_memory)
        return iter(self.dataset_from_memory)

    def __len__(self):
        return self.len


class CacheToFileWrapper(IterableDataset):
    """picard/dataset.py:153-200: the first pass writes the H5 label file, later passes read it
    batch-wise (as device tensors on the generator's device when `device` is given)."""

    def __init__(self, dataset: IterableDatasetWithInternalBatch, device=None):
        self.dataset = dataset
        self.device = device
        self.on_gen_stage = True
        self.saver: Optional[h5.H5Saver] = None
        self.dataset_from_file = None

    def init(self, save_file_path, n_total: int, n_dims: Sequence[int], labels: Sequence[str], dtype,
             preload: bool = False):
        self.dataset.set_size(n_total)
        self.saver = h5.H5Saver(save_file_path, n_total, n_dims, labels, dtype)
        self.dataset.attach_saver(self.saver)
        if preload:
            _preload(self.dataset)
            self.dataset_from_file = self.saver.create_torch_dataset(self.dataset.batch_size)
            self.on_gen_stage = False

    def _from_file(self):
        for batch in self.dataset_from_file:
            yield [b.to(self.device) for b in batch] if self.device is not None else batch

    def __iter__(self):
        if self.saver is None:
            raise AssertionError("Must call init() before using the iterator")
        if self.on_gen_stage:
            self.on_gen_stage = False
            return iter(self.dataset)
        if self.dataset_from_file is None:
            self.dataset_from_file = self.saver.create_torch_dataset(self.dataset.batch_size)
            if len(self.dataset_from_file) != len(self.dataset):
                raise AssertionError(f"len(self.dataset_from_file) {len(self.dataset_from_file)} must be equal to "
                                     f"len(self.dataset) {len(self.dataset)}")
        return self._from_file()

    def __len__(self):
        return len(self.dataset)


class DummyDataset(IterableDataset):
    """picard/dataset.py:258-264 (the validation loader's placeholder)."""

    def __iter__(self):
        yield torch.tensor([1.0]), torch.tensor([1.0])

    def __len__(self):
        return 1
