"""
Device-resident minibatches: the MI355X replacement of the host ``DataLoader`` in the reference's
minibatch example (``examples/minibatch.md:78-88``)::

    loader = DataLoader(TensorDataset(X, y), batch_size=10, shuffle=True)
    for X, y in loader:
        conditioned = mininf.condition(model, X=X, y=y)
        ...

becomes ``loader = DeviceDataLoader(X, y, batch_size=10, shuffle=True)`` with the same loop. The
dataset stays in HBM; each batch is a set of row indices computed on the device
(``mi_minibatch_rows``: a keyed Feistel permutation of the rows per epoch, no sort, no host work),
so a captured training step (:class:`mininf_amd.graph.StepGraph`) draws the next batch on every
replay through :meth:`DeviceDataLoader.next`.

The tensors a batch yields are :class:`Minibatch` tensors of the batch's shape. Their values are
gathered only when something reads them (``mi_gather_rows``); the site kernels that can read the
dataset rows through the index instead (the fused linear-predictor sites, ``mi_linear.row_index``)
never gather them, so the model's ``X @ theta`` and its ``Normal(X @ theta, 1)`` site read
``X`` and ``y`` once, straight from the dataset. ``batch(n)`` scaling (``core.py:267-271``) sees
the batch's shape, exactly as with the host loader.

Validation: the value-support checks of conditioned minibatch values run once over the whole
dataset column (memoised per version, :mod:`mininf_amd.particles`); a batch is a subset, so it
is valid whenever its dataset is. (The reference checks each batch when it is used, so an
invalid row raises here at the first batch rather than at the batch that holds it; the message is
the same.) Sites evaluated by the kernels flag values of the rows they read, as for any data.
"""
from __future__ import annotations

import os
import weakref
from typing import Dict, List, Optional, Tuple

import torch

from . import _native as nat

_functorch = torch._C._functorch

# untyped-storage address of a batch buffer -> (batch, column)
_BUFFERS: Dict[int, Tuple["weakref.ReferenceType[_Batch]", int]] = {}


def _storage_ptr(tensor) -> Optional[int]:
    if not isinstance(tensor, torch.Tensor):
        return None
    base = tensor
    while _functorch.is_batchedtensor(base):
        base = _functorch.get_unwrapped(base)
    try:
        return base.untyped_storage().data_ptr()
    except (RuntimeError, NotImplementedError):
        return None


class _Batch:
    """
    One drawn minibatch: the device row indices and the (lazily gathered) column buffers.

    The rows themselves are drawn lazily too: the ``mi_minibatch_rows`` launch is held back until
    something needs them, so that the one site kernel reading the batch can draw them itself
    (``mi_linear.rows``, one launch less per step -- :meth:`take_rows`); any other reader
    (:attr:`rows`, a gather) launches it first. Batches of one loader are launched in the order
    they were drawn.
    """
    def __init__(self, loader: "DeviceDataLoader", rows: torch.Tensor, count: int) -> None:
        self.loader = loader
        self._rows = rows
        self.count = count
        self.pending = True      # rows not drawn yet (no launch enqueued)
        self.buffers: List[torch.Tensor] = []
        self.filled: List[bool] = []

    @property
    def rows(self) -> torch.Tensor:
        """The batch's int32 row indices (drawn now if still pending)."""
        self.draw_rows()
        return self._rows

    def draw_rows(self) -> None:
        """Enqueue the ``mi_minibatch_rows`` launch of a pending batch."""
        if not self.pending:
            return
        self.pending = False
        loader = self.loader
        nat.check(nat.lib().mi_minibatch_rows(
            loader.counter.data_ptr(), loader.n, loader.batch_size, loader.batches,
            int(loader.shuffle), loader.seed, self._rows.data_ptr(), self.count,
            nat.stream_handle(loader.device)), "mi_minibatch_rows")

    def take_rows(self) -> Optional[nat.Rows]:
        """
        For the single kernel that reads this batch: a ``mi_rows`` descriptor drawing the rows
        inside that kernel (and writing them to the row buffer for later readers), or None when
        they are drawn already. The caller launches it next, or calls :meth:`draw_rows` first.
        """
        if not self.pending or self.count != self.loader.batch_size or \
                os.environ.get("MININF_AMD_FUSE_ROWS", "1") == "0":
            return None
        loader = self.loader
        R = nat.Rows()
        R.counter = loader.counter.data_ptr()
        R.n, R.batch, R.batches = loader.n, loader.batch_size, loader.batches
        R.seed, R.shuffle = loader.seed, int(loader.shuffle)
        R.out = self._rows.data_ptr()
        return R

    def rows_taken(self) -> None:
        """The kernel given :meth:`take_rows`'s descriptor was launched: the rows are drawn."""
        self.pending = False

    def fill(self, column: int) -> None:
        """Gather the column's rows into its buffer (once)."""
        if self.filled[column]:
            return
        base = self.loader.columns[column]
        out = self.buffers[column]
        row_bytes = base[0].numel() * base.element_size() if base.dim() > 1 else base.element_size()
        nat.check(nat.lib().mi_gather_rows(
            base.data_ptr(), base.stride(0) * base.element_size(), row_bytes,
            self.rows.data_ptr(), self.count, out.data_ptr(), row_bytes,
            nat.stream_handle(base.device)), "mi_gather_rows")
        self.filled[column] = True


def _forget(ptrs: List[int], ref) -> None:
    # entries of a collected batch (unless a newer batch's buffer took over the address)
    for ptr in ptrs:
        hit = _BUFFERS.get(ptr)
        if hit is not None and hit[0] is ref:
            del _BUFFERS[ptr]


def lookup(tensor) -> Optional[Tuple[_Batch, int]]:
    """(batch, column) when ``tensor`` (or a view / batched wrapper of it) is a minibatch buffer."""
    if not _BUFFERS:
        return None
    ptr = _storage_ptr(tensor)
    hit = _BUFFERS.get(ptr) if ptr is not None else None
    if hit is None:
        return None
    batch = hit[0]()
    return None if batch is None else (batch, hit[1])


def dataset_column(tensor) -> Optional[torch.Tensor]:
    """The full dataset column a minibatch tensor was drawn from (validation), or None."""
    hit = lookup(tensor)
    return None if hit is None else hit[0].loader.columns[hit[1]]


def ensure_filled(tensor) -> None:
    """Gather a minibatch tensor's values if a kernel is about to read them directly."""
    hit = lookup(tensor)
    if hit is not None:
        hit[0].fill(hit[1])


# Operations that read no values: they run on the (possibly not yet gathered) buffer.
_METADATA = {
    torch.Tensor.size, torch.Tensor.dim, torch.Tensor.ndimension, torch.Tensor.numel,
    torch.Tensor.__len__, torch.Tensor.is_floating_point, torch.Tensor.is_complex,
    torch.Tensor.stride, torch.Tensor.element_size, torch.Tensor.data_ptr,
    torch.Tensor.untyped_storage, torch.Tensor.storage_offset, torch.Tensor.is_contiguous,
    torch.Tensor.shape.__get__, torch.Tensor.dtype.__get__, torch.Tensor.device.__get__,
    torch.Tensor.ndim.__get__, torch.Tensor.requires_grad.__get__, torch.Tensor.is_cuda.__get__,
    torch.Tensor.layout.__get__, torch.Tensor.is_sparse.__get__, torch.Tensor.grad_fn.__get__,
    torch.Tensor.is_leaf.__get__, torch.Tensor.names.__get__, torch.Tensor.__hash__,
    torch.Tensor._version.__get__, torch.Tensor.is_mps.__get__,
}
# Views share the buffer: the result stays a Minibatch (values gathered on first read).
_VIEWS = {
    torch.Tensor.expand, torch.Tensor.expand_as, torch.Tensor.broadcast_to, torch.broadcast_to,
    torch.Tensor.view, torch.Tensor.view_as, torch.Tensor.reshape, torch.Tensor.unsqueeze,
    torch.Tensor.squeeze, torch.Tensor.t, torch.Tensor.transpose, torch.Tensor.permute,
    torch.Tensor.T.__get__, torch.Tensor.mT.__get__, torch.Tensor.detach, torch.unsqueeze,
    torch.squeeze, torch.t, torch.transpose, torch.permute, torch.reshape,
}


class Minibatch(torch.Tensor):
    """
    A column of one drawn minibatch (see the module docstring). Behaves as the gathered rows for
    every operation: anything that reads values first gathers them (one ``mi_gather_rows``
    launch per column and batch); shape queries and views do not.
    """
    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        with torch._C.DisableTorchFunctionSubclass():
            if func in _METADATA:
                return func(*args, **kwargs)
            if func in _VIEWS:
                out = func(*args, **kwargs)
                hit = lookup(out) if isinstance(out, torch.Tensor) else None
                if hit is not None:
                    if not isinstance(out, Minibatch):
                        out = out.as_subclass(Minibatch)
                    # the view shares the batch's buffer: it keeps the batch (its rows and its
                    # lookup entry) alive on its own, also after the yielded tensor is dropped
                    out._mininf_batch = hit[0]
                return out
            stack = [args, kwargs]
            while stack:   # the call's tensors (lists, tuples and dicts walked)
                x = stack.pop()
                if isinstance(x, Minibatch):
                    ensure_filled(x)
                elif isinstance(x, (list, tuple)):
                    stack.extend(x)
                elif isinstance(x, dict):
                    stack.extend(x.values())
            return func(*args, **kwargs)


class DeviceDataLoader:
    """
    ``DataLoader(TensorDataset(*tensors), batch_size, shuffle, drop_last)`` over device-resident
    tensors (same leading dimension). Iterating yields one tuple of :class:`Minibatch` tensors per
    batch of the current epoch, in a fresh random row order per epoch when ``shuffle``.
    :meth:`next` draws the next batch, crossing epochs, with no host work: use it inside a
    captured step (every batch then has ``batch_size`` rows, so ``drop_last`` or a dataset whose
    size ``batch_size`` divides is required).
    """
    def __init__(self, *tensors: torch.Tensor, batch_size: int = 1, shuffle: bool = False,
                 drop_last: bool = False, seed: Optional[int] = None) -> None:
        if not tensors:
            raise ValueError("DeviceDataLoader needs at least one tensor")
        n = tensors[0].shape[0]
        if any(t.shape[0] != n for t in tensors):
            raise ValueError("Size mismatch between tensors")   # TensorDataset's message
        if batch_size < 1:
            raise ValueError(f"batch_size should be a positive integer value, but got "
                             f"batch_size={batch_size}")
        for t in tensors:
            nat.require_device(t, "DeviceDataLoader tensors")
            if t.element_size() * max(1, t[0].numel()) % 4:
                raise nat.NativeError("DeviceDataLoader rows must be a multiple of 4 bytes")
        # rows contiguous in memory (gathered as whole rows)
        self.columns = [t if t.dim() > 0 and t[0].is_contiguous() else t.contiguous()
                        for t in tensors]
        self.n = int(n)
        self.batch_size = int(batch_size)
        self.shuffle = bool(shuffle)
        self.drop_last = bool(drop_last)
        self.seed = int(seed if seed is not None else torch.initial_seed()) & ((1 << 64) - 1)
        self.device = tensors[0].device
        self.batches = self.n // self.batch_size if self.drop_last else \
            -(-self.n // self.batch_size)
        if self.batches < 1:
            raise ValueError("the dataset holds fewer rows than one batch and drop_last is set")
        if self.n >= 2 ** 31:
            raise nat.NativeError("DeviceDataLoader supports fewer than 2^31 rows")
        # batch counter (device): epoch = counter[0] // batches, batch = counter[0] % batches;
        # counter[1] is the rows kernel's completion count
        self.counter = torch.zeros(2, dtype=torch.int64, device=self.device)
        self._position = 0   # host mirror for eager iteration (ragged last batch)
        self._last: Optional[_Batch] = None   # the last drawn batch (rows may be pending)

    def __len__(self) -> int:
        return self.batches

    def _draw(self, count: int) -> Tuple[Minibatch, ...]:
        # the previous batch's rows, if nobody drew them yet, come first (the batch counter
        # orders the batches)
        if self._last is not None:
            self._last.draw_rows()
        rows = torch.empty(count, dtype=torch.int32, device=self.device)
        batch = _Batch(self, rows, count)
        # held until the next draw, which launches its rows if nothing else did (a batch drawn
        # and dropped unused still advances the loader, as with an eager rows launch)
        self._last = batch
        ref = weakref.ref(batch)
        ptrs: List[int] = []
        weakref.finalize(batch, _forget, ptrs, ref)
        out = []
        for column, base in enumerate(self.columns):
            buffer = torch.empty((count,) + tuple(base.shape[1:]), dtype=base.dtype,
                                 device=self.device)
            batch.buffers.append(buffer)
            batch.filled.append(False)
            ptr = buffer.untyped_storage().data_ptr()
            _BUFFERS[ptr] = (ref, column)
            ptrs.append(ptr)
            view = buffer.as_subclass(Minibatch)
            view._mininf_batch = batch   # keeps the batch (and its rows) alive with the tensor
            out.append(view)
        return tuple(out)

    def next(self) -> Tuple[Minibatch, ...]:
        """The next batch (any epoch): ``batch_size`` rows, drawn on the device."""
        if (self.batches - 1) * self.batch_size + self.batch_size > self.n:
            raise ValueError("next() draws full batches: set drop_last=True or use a batch_size "
                             "that divides the dataset size")
        self._position = (self._position + 1) % self.batches
        return self._draw(self.batch_size)

    def __iter__(self):
        for b in range(self.batches):
            count = min(self.batch_size, self.n - b * self.batch_size)
            if self._position != b:
                # the device counter and this iteration agree only from the start of an epoch
                raise RuntimeError("a DeviceDataLoader iteration must start at an epoch boundary")
            self._position = (self._position + 1) % self.batches
            yield self._draw(count)
