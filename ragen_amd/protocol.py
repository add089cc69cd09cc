"""Minimal DataProto-compatible container (verl.DataProto is absent offline).

Covers what the hot path touches: ``batch`` (dict of tensors with a common first dim),
``non_tensor_batch`` (dict of numpy object/int arrays), ``meta_info``; boolean-mask /
index selection (agent_trainer.py:481-488), ``union`` and ``len``.
"""
from typing import Dict, Optional

import numpy as np
import torch


class TensorBatch(dict):
    """dict of tensors; indexing with a mask / index tensor selects rows of every entry."""

    def __init__(self, d=None, batch_size=None):
        super().__init__(d or {})
        self.batch_size = batch_size

    def __getitem__(self, k):
        if isinstance(k, str):
            return dict.__getitem__(self, k)
        return TensorBatch({kk: v[k] for kk, v in self.items()})

    def keys(self):
        return list(dict.keys(self))


class DataProto:
    def __init__(self, batch: Optional[Dict[str, torch.Tensor]] = None, non_tensor_batch=None, meta_info=None):
        self.batch = TensorBatch(batch) if batch is not None and not isinstance(batch, TensorBatch) else batch
        self.non_tensor_batch = non_tensor_batch if non_tensor_batch is not None else {}
        self.meta_info = meta_info if meta_info is not None else {}

    def __len__(self):
        if self.batch:
            return next(iter(self.batch.values())).shape[0]
        if self.non_tensor_batch:
            return len(next(iter(self.non_tensor_batch.values())))
        return 0

    def select_rows(self, mask) -> "DataProto":
        """Row selection as _filter_rollout does it (agent_trainer.py:481-488)."""
        if isinstance(mask, torch.Tensor):
            mask_np = mask.cpu().numpy()
        else:
            mask_np = np.asarray(mask)
        batch = None
        if self.batch is not None:
            idx = torch.as_tensor(mask_np)
            batch = TensorBatch({k: v[idx.to(v.device)] for k, v in self.batch.items()})
        ntb = {}
        for k, v in self.non_tensor_batch.items():
            ntb[k] = v[mask_np] if isinstance(v, np.ndarray) else [x for x, m in zip(v, mask_np) if m]
        return DataProto(batch, ntb, dict(self.meta_info))

    def union(self, other: "DataProto") -> "DataProto":
        if other.batch:
            if self.batch is None:
                self.batch = TensorBatch()
            self.batch.update(other.batch)
        self.non_tensor_batch.update(other.non_tensor_batch)
        self.meta_info.update(other.meta_info)
        return self
