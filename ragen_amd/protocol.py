"""DataProto — the batch container RAGEN's trainer moves between the rollout, the reward and
the worker groups (verl.DataProto; verl is absent offline, so this is a from-scratch
container with the surface ``RayAgentTrainer.fit`` uses, agent_trainer.py:514-633).

* ``batch``: a ``TensorBatch`` — a dict of tensors sharing the first dimension (TensorDict
  semantics: ``len()`` is the row count, indexing with an int / slice / index tensor / bool
  mask selects rows of every entry);
* ``non_tensor_batch``: a dict of numpy object arrays with the same row count;
* ``meta_info``: a plain dict.

Row operations keep the three in step: ``select_idxs`` / ``__getitem__`` / ``slice``,
``reorder`` (in place, used by ``_balance_batch``), ``repeat``, ``chunk`` / ``split`` and
``concat`` (the DP dispatch of the worker groups), ``union`` (with verl's conflict checks),
``pop``, ``select``, ``rename`` and ``to``.
"""
import copy
from typing import Dict, Iterable, List, Optional, Sequence

import numpy as np
import torch


def _index(idx, n):
    """Normalise a row selector to an int64 index tensor (bool masks -> their positions)."""
    if isinstance(idx, slice):
        return torch.arange(n)[idx]
    if isinstance(idx, torch.Tensor):
        t = idx.cpu()
    else:
        t = torch.as_tensor(np.asarray(idx))
    if t.dtype == torch.bool:
        if t.numel() != n:
            raise IndexError(f"boolean index of length {t.numel()} for {n} rows")
        return t.nonzero().flatten()
    return t.to(torch.int64).flatten()


class TensorBatch:
    """A dict of tensors with a common first dimension (the TensorDict subset verl uses)."""

    def __init__(self, d: Optional[Dict[str, torch.Tensor]] = None, batch_size=None):
        self._d: Dict[str, torch.Tensor] = {}
        self._n = None
        if batch_size is not None:
            self._n = int(batch_size[0] if isinstance(batch_size, (list, tuple, torch.Size)) else batch_size)
        for k, v in (d or {}).items():
            self[k] = v

    # ---- mapping surface
    @property
    def batch_size(self):
        return torch.Size([self._n if self._n is not None else 0])

    def __len__(self):
        return self._n if self._n is not None else 0

    def __contains__(self, k):
        return k in self._d

    def keys(self):
        return list(self._d.keys())

    def values(self):
        return list(self._d.values())

    def items(self):
        return list(self._d.items())

    def get(self, k, default=None):
        return self._d.get(k, default)

    def __iter__(self):
        return iter(self._d)

    def __setitem__(self, k, v):
        if not isinstance(k, str):
            raise TypeError("TensorBatch keys are strings")
        if not isinstance(v, torch.Tensor):
            raise TypeError(f"{k}: TensorBatch holds tensors")
        if self._n is None:
            self._n = v.shape[0]
        elif v.shape[0] != self._n:
            raise ValueError(f"{k}: {v.shape[0]} rows in a batch of {self._n}")
        self._d[k] = v

    def __getitem__(self, k):
        if isinstance(k, str):
            return self._d[k]
        idx = _index(k, len(self))
        return TensorBatch({kk: v[idx.to(v.device)] for kk, v in self._d.items()}, batch_size=[idx.numel()])

    def __delitem__(self, k):
        del self._d[k]

    def pop(self, k, *default):
        return self._d.pop(k, *default)

    def update(self, other):
        for k, v in (other.items() if isinstance(other, TensorBatch) else dict(other).items()):
            self[k] = v

    def select(self, *keys):
        return TensorBatch({k: self._d[k] for k in keys}, batch_size=[len(self)])

    def to(self, device):
        return TensorBatch({k: v.to(device) for k, v in self._d.items()}, batch_size=[len(self)])

    def clone(self):
        return TensorBatch({k: v.clone() for k, v in self._d.items()}, batch_size=[len(self)])

    @staticmethod
    def cat(parts: Sequence["TensorBatch"]) -> "TensorBatch":
        keys = parts[0].keys()
        for p in parts[1:]:
            if set(p.keys()) != set(keys):
                raise ValueError("concat of batches with different keys")
        return TensorBatch({k: torch.cat([p[k] for p in parts], dim=0) for k in keys},
                           batch_size=[sum(len(p) for p in parts)])

    def __repr__(self):
        return f"TensorBatch(batch_size={len(self)}, keys={self.keys()})"


def _union_tensors(a: TensorBatch, b: TensorBatch) -> TensorBatch:
    """verl union_tensor_dict: same batch size; a key present in both must hold equal tensors."""
    if len(a) != len(b) and len(a.keys()) and len(b.keys()):
        raise ValueError(f"two batches with different batch sizes: {len(a)} and {len(b)}")
    for k, v in b.items():
        if k in a and not torch.equal(a[k], v):
            raise ValueError(f"{k} in both batches with different values: union would overwrite it")
        a[k] = v
    return a


def _union_numpy(a: dict, b: dict) -> dict:
    for k, v in b.items():
        if k in a:
            x = a[k]
            same = len(x) == len(v) and all((p == q) if not (isinstance(p, float) and np.isnan(p)) else
                                            (isinstance(q, float) and np.isnan(q)) for p, q in zip(x, v))
            if not same:
                raise ValueError(f"{k} in both non-tensor batches with different values")
        a[k] = v
    return a


def _rows(v, idx: np.ndarray):
    return v[idx] if isinstance(v, np.ndarray) else [v[i] for i in idx]


class DataProto:
    def __init__(self, batch=None, non_tensor_batch=None, meta_info=None):
        if batch is not None and not isinstance(batch, TensorBatch):
            batch = TensorBatch(batch)
        self.batch: Optional[TensorBatch] = batch
        self.non_tensor_batch: Dict[str, np.ndarray] = non_tensor_batch if non_tensor_batch is not None else {}
        self.meta_info: dict = meta_info if meta_info is not None else {}

    # ---- construction
    @classmethod
    def from_dict(cls, tensors: Optional[dict] = None, non_tensors: Optional[dict] = None, meta_info=None):
        nt = {k: (v if isinstance(v, np.ndarray) else np.array(v, dtype=object)) for k, v in (non_tensors or {}).items()}
        return cls(TensorBatch(tensors or {}) if tensors else None, nt, dict(meta_info or {}))

    @classmethod
    def from_single_dict(cls, data: dict, meta_info=None):
        tensors = {k: v for k, v in data.items() if isinstance(v, torch.Tensor)}
        others = {k: v for k, v in data.items() if not isinstance(v, torch.Tensor)}
        return cls.from_dict(tensors, others, meta_info)

    # ---- size and consistency
    def __len__(self):
        if self.batch is not None and len(self.batch.keys()):
            return len(self.batch)
        if self.non_tensor_batch:
            return len(next(iter(self.non_tensor_batch.values())))
        return 0

    def check_consistency(self):
        n = len(self)
        for k, v in self.non_tensor_batch.items():
            if len(v) != n:
                raise ValueError(f"non_tensor_batch[{k!r}] has {len(v)} rows, batch has {n}")

    # ---- row selection
    def select_idxs(self, idxs) -> "DataProto":
        idx = _index(idxs, len(self))
        batch = self.batch[idx] if self.batch is not None else None
        inp = idx.numpy()
        return DataProto(batch, {k: _rows(v, inp) for k, v in self.non_tensor_batch.items()}, dict(self.meta_info))

    def select_rows(self, mask) -> "DataProto":
        """Row selection as _filter_rollout does it (agent_trainer.py:481-488)."""
        return self.select_idxs(mask)

    def slice(self, start=None, end=None, step=None) -> "DataProto":
        return self.select_idxs(slice(start, end, step))

    def __getitem__(self, item):
        if isinstance(item, (int, np.integer)):
            i = int(item)
            return DataProtoItem({k: v[i] for k, v in (self.batch.items() if self.batch is not None else [])},
                                 {k: v[i] for k, v in self.non_tensor_batch.items()}, self.meta_info)
        return self.select_idxs(item)

    def reorder(self, indices):
        """In place (verl DataProto.reorder, used by _balance_batch)."""
        idx = _index(indices, len(self))
        if self.batch is not None:
            self.batch = self.batch[idx]
        inp = idx.numpy()
        self.non_tensor_batch = {k: _rows(v, inp) for k, v in self.non_tensor_batch.items()}

    def repeat(self, repeat_times: int = 2, interleave: bool = True) -> "DataProto":
        n = len(self)
        idx = (torch.arange(n).repeat_interleave(repeat_times) if interleave else torch.arange(n).repeat(repeat_times))
        return self.select_idxs(idx)

    # ---- key operations
    def select(self, batch_keys=None, non_tensor_batch_keys=None, meta_info_keys=None, deepcopy=False):
        batch = None
        if self.batch is not None:
            keys = batch_keys if batch_keys is not None else self.batch.keys()
            batch = self.batch.select(*keys)
        ntk = non_tensor_batch_keys if non_tensor_batch_keys is not None else list(self.non_tensor_batch)
        mik = meta_info_keys if meta_info_keys is not None else list(self.meta_info)
        nt = {k: self.non_tensor_batch[k] for k in ntk}
        mi = {k: self.meta_info[k] for k in mik}
        if deepcopy:
            nt, mi = copy.deepcopy(nt), copy.deepcopy(mi)
            batch = batch.clone() if batch is not None else None
        return DataProto(batch, nt, mi)

    def pop(self, batch_keys=None, non_tensor_batch_keys=None, meta_info_keys=None) -> "DataProto":
        """Remove the named keys and return them as a new DataProto (agent_trainer.py:538)."""
        tensors = {k: self.batch.pop(k) for k in (batch_keys or [])}
        nt = {k: self.non_tensor_batch.pop(k) for k in (non_tensor_batch_keys or [])}
        mi = {k: self.meta_info.pop(k) for k in (meta_info_keys or [])}
        return DataProto(TensorBatch(tensors) if tensors else None, nt, mi)

    def rename(self, old_keys, new_keys):
        old_keys = [old_keys] if isinstance(old_keys, str) else list(old_keys)
        new_keys = [new_keys] if isinstance(new_keys, str) else list(new_keys)
        if len(old_keys) != len(new_keys):
            raise ValueError("rename needs as many new keys as old ones")
        for o, n in zip(old_keys, new_keys):
            self.batch[n] = self.batch.pop(o)
        return self

    def union(self, other: "DataProto") -> "DataProto":
        """Merge another DataProto into this one (in place, returned).  As verl: the batch
        sizes must agree, and a key present in both must carry the same data."""
        if other.batch is not None and len(other.batch.keys()):
            if self.batch is None:
                self.batch = TensorBatch()
            _union_tensors(self.batch, other.batch)
        _union_numpy(self.non_tensor_batch, other.non_tensor_batch)
        for k, v in other.meta_info.items():
            if k in self.meta_info and self.meta_info[k] != v:
                raise ValueError(f"meta_info[{k!r}] differs between the two DataProtos")
            self.meta_info[k] = v
        return self

    def to(self, device) -> "DataProto":
        if self.batch is not None:
            self.batch = self.batch.to(device)
        return self

    # ---- data-parallel dispatch (the worker groups' DP_COMPUTE_PROTO)
    def chunk(self, chunks: int) -> List["DataProto"]:
        n = len(self)
        if n % chunks != 0:
            raise ValueError(f"only support equal chunk: {n} rows into {chunks} chunks")
        return self.split(n // chunks)

    def split(self, split_size: int) -> List["DataProto"]:
        n = len(self)
        return [self.slice(i, min(i + split_size, n)) for i in range(0, n, split_size)]

    @staticmethod
    def concat(data: Sequence["DataProto"]) -> "DataProto":
        batch = None
        if data[0].batch is not None:
            batch = TensorBatch.cat([d.batch for d in data])
        nt = {}
        for k in data[0].non_tensor_batch:
            parts = [d.non_tensor_batch[k] for d in data]
            nt[k] = np.concatenate(parts) if all(isinstance(p, np.ndarray) for p in parts) else \
                [x for p in parts for x in p]
        return DataProto(batch, nt, dict(data[0].meta_info))

    def make_iterator(self, mini_batch_size: int, epochs: int = 1, seed=None) -> Iterable["DataProto"]:
        g = torch.Generator().manual_seed(seed) if seed is not None else None
        for _ in range(epochs):
            idx = torch.randperm(len(self), generator=g) if g is not None else torch.arange(len(self))
            for i in range(0, len(self), mini_batch_size):
                yield self.select_idxs(idx[i:i + mini_batch_size])

    def __repr__(self):
        return (f"DataProto(len={len(self)}, batch={self.batch.keys() if self.batch is not None else None}, "
                f"non_tensor={list(self.non_tensor_batch)}, meta={list(self.meta_info)})")


class DataProtoItem:
    """One row of a DataProto (verl DataProtoItem)."""

    def __init__(self, batch: dict, non_tensor_batch: dict, meta_info: dict):
        self.batch, self.non_tensor_batch, self.meta_info = batch, non_tensor_batch, meta_info
