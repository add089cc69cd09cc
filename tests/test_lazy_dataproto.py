"""LazyDataProto (the device path's get_lm_inputs / formulate_rollouts result): env ids held as
int64, the reference's object arrays of env / group ids made on first read without building
the messages, everything else built on first access — CPU only."""
import numpy as np
import torch

from ragen_amd.llm_agent.agent_proxy import env_ids_of
from ragen_amd.llm_agent.ctx_manager import LazyDataProto
from ragen_amd.protocol import DataProto


def _lazy(ids, built):
    def build():
        built.append(1)
        return DataProto(None, {"messages_list": np.array([[{"role": "user", "content": str(i)}] for i in ids] +
                                                          [None], dtype=object)[:-1]})
    return LazyDataProto(ids, build)


def test_ids_without_building():
    built = []
    ids = np.arange(10, 18, dtype=np.int64)
    d = _lazy(ids, built)
    assert len(d) == 8 and env_ids_of(d) is d.env_ids_i64
    assert "env_ids" in d.non_tensor_batch and "group_ids" not in d.non_tensor_batch
    e = d.non_tensor_batch["env_ids"]
    assert e.dtype == object and list(e) == list(range(10, 18)) and type(e[0]) is int
    assert d.non_tensor_batch.get("messages_list") is None  # not built by get / in
    assert not built
    d.set_device_batch({"input_ids": torch.zeros(8, 3, dtype=torch.int64)}, ids, 4)
    g = d.non_tensor_batch["group_ids"]
    assert list(g) == [2, 2, 3, 3, 3, 3, 4, 4] and type(g[0]) is int
    assert not built
    assert d.batch["input_ids"].shape == (8, 3) and not built  # the device batch needs no build
    # keys / items / len build the rest, ids included
    assert set(d.non_tensor_batch.keys()) == {"env_ids", "group_ids", "messages_list"} and built == [1]
    assert len(d.non_tensor_batch) == 3


def test_set_device_batch_other_ids():
    d = _lazy(np.arange(4), [])
    _ = d.non_tensor_batch["env_ids"]
    d.set_device_batch({"input_ids": torch.zeros(2, 1)}, np.array([5, 9]), 4)
    assert list(d.non_tensor_batch["env_ids"]) == [5, 9] and list(d.non_tensor_batch["group_ids"]) == [1, 2]
    assert len(d) == 2


def test_env_ids_of_plain_dataproto():
    d = DataProto(None, {"env_ids": np.array([3, 1, 2], dtype=object)})
    ids = env_ids_of(d)
    assert ids.dtype == np.int64 and list(ids) == [3, 1, 2]


def test_freed_without_the_cyclic_gc():
    """A LazyDataProto and its non_tensor_batch hold no reference cycle: the batch is freed as
    soon as the caller drops it (its tensors' block is then free for the next rollout's batch)."""
    import gc
    import weakref
    gc.disable()
    try:
        d = LazyDataProto(np.arange(4), lambda: None)
        d.set_device_batch({"input_ids": torch.zeros(4, 3, dtype=torch.int64)}, np.arange(4), 2)
        assert list(d.non_tensor_batch["group_ids"]) == [0, 0, 1, 1] and "env_ids" in d.non_tensor_batch
        w = weakref.ref(d)
        del d
        assert w() is None
    finally:
        gc.enable()


def test_block_use_count_with_a_held_storage():
    """DevicePrompts.batch_block's reuse check: a block and its held storage object count 2;
    any live view of it (the batch's unbound rows, a slice of them) raises the count."""
    from ragen_amd.llm_agent.prompts import _uses
    t = torch.empty(12, dtype=torch.int64)
    st = t.untyped_storage()
    assert _uses(st) == 2
    a, b, c = t[:9].view(3, 3).unbind(0)
    r = a[1:]
    del a, b, c
    assert _uses(st) > 2  # the slice still holds the block
    del r
    assert _uses(st) == 2
