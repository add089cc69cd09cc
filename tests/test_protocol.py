"""CPU tests of ragen_amd.protocol.DataProto: the surface RayAgentTrainer.fit uses on the
rollout's batch (agent_trainer.py:514-633) and the worker groups' DP dispatch needs."""
import numpy as np
import pytest
import torch

from ragen_amd.protocol import DataProto, TensorBatch


def _batch(n=8, L=5):
    g = torch.Generator().manual_seed(0)
    return DataProto.from_dict({"input_ids": torch.randint(0, 100, (n, L), generator=g),
                                "attention_mask": torch.ones(n, L, dtype=torch.int64),
                                "rm_scores": torch.rand(n, L - 1, generator=g)},
                               {"env_ids": np.arange(n), "group_ids": np.arange(n) // 4},
                               {"metrics": {"a": 1.0}})


def test_len_and_tensordict_semantics():
    d = _batch()
    assert len(d) == 8 and len(d.batch) == 8 and d.batch.batch_size[0] == 8  # len(batch.batch): uid count
    assert "rm_scores" in d.batch and "nope" not in d.batch
    with pytest.raises(ValueError):
        d.batch["bad"] = torch.zeros(3)
    sub = d.batch[torch.tensor([True, False] * 4)]  # batch.batch[mask] (agent_trainer.py:481)
    assert len(sub) == 4 and torch.equal(sub["input_ids"], d.batch["input_ids"][::2])


def test_select_rows_and_getitem():
    d = _batch()
    m = np.array([1, 1, 0, 0, 1, 1, 0, 0], bool)
    s = d.select_rows(m)
    assert len(s) == 4 and list(s.non_tensor_batch["env_ids"]) == [0, 1, 4, 5]
    assert torch.equal(s.batch["rm_scores"], d.batch["rm_scores"][torch.from_numpy(m)])
    assert len(d[2:6]) == 4 and d[3].non_tensor_batch["env_ids"] == 3
    assert torch.equal(d[[7, 0]].batch["input_ids"], d.batch["input_ids"][[7, 0]])


def test_union_conflicts_and_pop():
    d = _batch()
    other = DataProto.from_dict({"old_log_probs": torch.zeros(8, 4)}, {"uid": np.array(list("abcdefgh"), object)})
    d.union(other)
    assert "old_log_probs" in d.batch and "uid" in d.non_tensor_batch
    d.union(DataProto.from_dict({"old_log_probs": torch.zeros(8, 4)}))  # same values: fine
    with pytest.raises(ValueError):
        d.union(DataProto.from_dict({"old_log_probs": torch.ones(8, 4)}))
    with pytest.raises(ValueError):
        d.union(DataProto.from_dict({"x": torch.ones(3, 4)}))
    with pytest.raises(ValueError):
        d.union(DataProto.from_dict(None, {"uid": np.array(list("abcdefgz"), object)}))
    popped = d.pop(batch_keys=["old_log_probs"])  # agent_trainer.py:538
    assert "old_log_probs" not in d.batch and popped.batch["old_log_probs"].shape == (8, 4)


def test_reorder_balance_batch():
    """_balance_batch: per-row token counts -> a permutation -> reorder in place."""
    d = _batch()
    d.batch["attention_mask"][:, :2] = torch.tensor([[0, 0], [0, 1], [1, 1], [0, 0], [1, 0], [0, 0], [1, 1], [0, 1]])
    before = {int(e): d.batch["input_ids"][i].clone() for i, e in enumerate(d.non_tensor_batch["env_ids"])}
    seqlen = d.batch["attention_mask"].view(len(d), -1).sum(-1).tolist()
    perm = np.argsort(seqlen, kind="stable")[::-1].copy()
    d.reorder(torch.from_numpy(perm))
    assert d.batch["attention_mask"].sum(-1).tolist() == sorted(seqlen, reverse=True)
    for i, e in enumerate(d.non_tensor_batch["env_ids"]):
        assert torch.equal(d.batch["input_ids"][i], before[int(e)])


def test_chunk_concat_repeat_select():
    d = _batch()
    parts = d.chunk(4)  # DP_COMPUTE_PROTO: one chunk per worker
    assert [len(p) for p in parts] == [2, 2, 2, 2]
    back = DataProto.concat(parts)
    for k in d.batch.keys():
        assert torch.equal(back.batch[k], d.batch[k])
    assert list(back.non_tensor_batch["env_ids"]) == list(range(8))
    with pytest.raises(ValueError):
        d.chunk(3)
    r = d.repeat(2, interleave=True)
    assert len(r) == 16 and list(r.non_tensor_batch["env_ids"][:4]) == [0, 0, 1, 1]
    r2 = d.repeat(2, interleave=False)
    assert list(r2.non_tensor_batch["env_ids"][:3]) == [0, 1, 2]
    s = d.select(batch_keys=["rm_scores"], non_tensor_batch_keys=["env_ids"], deepcopy=True)
    assert s.batch.keys() == ["rm_scores"] and list(s.non_tensor_batch) == ["env_ids"]
    d.rename("rm_scores", "token_level_scores")
    assert "token_level_scores" in d.batch and "rm_scores" not in d.batch
    mbs = list(d.make_iterator(3, epochs=1))
    assert [len(m) for m in mbs] == [3, 3, 2]


def test_tensorbatch_cat_and_check_consistency():
    a = TensorBatch({"x": torch.zeros(2, 3)})
    b = TensorBatch({"x": torch.ones(3, 3)})
    assert len(TensorBatch.cat([a, b])) == 5
    d = DataProto(a, {"k": np.arange(3)})
    with pytest.raises(ValueError):
        d.check_consistency()
