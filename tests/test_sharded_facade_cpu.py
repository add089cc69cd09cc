"""world_size-2 gloo test of the sharded facade's host logic on the CPU (the HIP kernels need a
GPU; tests/test_gpu_sharded.py runs the whole facade sharded on the GPU):

* ``shard_plan``: group-aligned shards of a mixed-tag config (tag boundaries inside a shard);
* the train seed (es_manager.py:88-89) drawn on rank 0 and broadcast, whatever each rank's
  own Python RNG holds; a sharded manager without a process group refuses to draw one;
* ``gather_formulated``: each rank's left-padded [B_r, S_r] batch padded to the global S and
  all-gathered == the one left-padded batch of all rows (ctx_manager.py:278-306);
* ``ContextManager.device_metrics``: every rank reports the metrics of the whole batch
  (ctx_manager.py:308-329), from the gathered per-env metric rows.
"""
import os
import random
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ragen_amd import distributed as rd
from ragen_amd.config import env_task
from ragen_amd.llm_agent.es_manager import EnvStateManager, shard_plan
from ragen_amd.protocol import DataProto

PAD = 151643
N_ROWS, WORLD = 48, 2


def _rows(seed=3):
    """Ragged token rows (the formulated batch before padding) and per-row scores."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(5, 40, size=N_ROWS)
    lens[7] = 61  # the longest row sits on rank 0 only: rank 1 must pad to it
    return [rng.integers(0, 1000, size=int(n)) for n in lens], rng.standard_normal(N_ROWS).astype(np.float32)


def _formulated(rows, scores, env_lo):
    """What formulate_rollouts returns for these rows: left padded to their own max width."""
    S = max(len(r) for r in rows)
    B = len(rows)
    ids = torch.full((B, S), PAD, dtype=torch.int64)
    am = torch.zeros(B, S, dtype=torch.int64)
    for i, r in enumerate(rows):
        ids[i, S - len(r):] = torch.from_numpy(r)
        am[i, S - len(r):] = 1
    pos = am.cumsum(-1)
    loss = torch.zeros(B, S - 1, dtype=torch.bool)
    loss[:, -3:] = True
    rm = torch.zeros(B, S - 1, dtype=torch.float32)
    rm[:, -1] = torch.from_numpy(scores)
    env_ids = np.arange(env_lo, env_lo + B)
    return DataProto({"input_ids": ids, "attention_mask": am, "position_ids": pos, "responses": ids[:, 1:],
                      "loss_mask": loss, "rm_scores": rm, "original_rm_scores": rm},
                     {"env_ids": np.array(env_ids.tolist(), dtype=object),
                      "group_ids": np.array((env_ids // 4).tolist(), dtype=object)}, {"metrics": {}})


class _MetricEs:
    """The slice of EnvStateManager that device_metrics reads: per-tag metric rows."""

    def __init__(self, parts):
        self._parts = parts

    def metric_arrays(self):
        return self._parts


def _metric_parts(lo, hi):
    """Per-tag (tag, m f64[n,4], custom bool[n], info) rows of the envs [lo, hi): two tags, 16 + 16."""
    rng = np.random.default_rng(11)
    m = np.stack([rng.integers(0, 2, 32), rng.integers(0, 11, 32), rng.random(32), rng.random(32)], 1)
    m[rng.random(32) < 0.3, 2:] = 0.0
    custom = rng.random(32) < 0.8
    out = []
    for tag, a, b in (("SimpleSokoban", 0, 16), ("FrozenLake", 16, 32)):
        s, e = max(a, lo), min(b, hi)
        if e > s:
            out.append((tag, m[s:e], custom[s:e], None))
    return out


def _metrics_cfg():
    cfg = env_task("SimpleSokoban", 8, 4)
    cfg.es_manager.train.env_configs.tags = ["SimpleSokoban", "FrozenLake"]
    cfg.es_manager.train.env_configs.n_groups = [4, 4]
    return cfg


def _ctx(cfg, rank, world, group):
    from ragen_amd.llm_agent.ctx_manager import ContextManager
    return ContextManager(cfg, tokenizer=None, device="cpu", rank=rank, world_size=world, process_group=group)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # train seed: only rank 0's draw counts
        random.seed(5 if rank == 0 else 99)
        es = EnvStateManager.__new__(EnvStateManager)
        es.process_group, es.rank, es.world_size = dist.group.WORLD, rank, world
        seed = es._train_seed(None)
        # the formulated batch of this rank's rows, gathered
        rows, scores = _rows()
        g0, ng = rd.shard_groups(N_ROWS // 4, world, rank)
        lo, hi = g0 * 4, (g0 + ng) * 4
        out = rd.gather_formulated(_formulated(rows[lo:hi], scores[lo:hi], lo), PAD, dist.group.WORLD)
        # numpy copies: a tensor sent through the queue lives in this process's shared memory,
        # which goes away when the worker exits, before the parent may have read it
        batch = {k: out.batch[k].numpy().copy() for k in out.batch.keys()}
        nt = {k: list(out.non_tensor_batch[k]) for k in ("env_ids", "group_ids")}
        aliased = out.batch["original_rm_scores"].data_ptr() == out.batch["rm_scores"].data_ptr()
        # the metrics every rank reports
        cfg = _metrics_cfg()
        ctx = _ctx(cfg, rank, world, dist.group.WORLD)
        met = ctx.device_metrics(_MetricEs(_metric_parts(ctx.env_lo, ctx.env_lo + ctx.n_envs)))
        q.put((rank, seed, batch, nt, aliased, met))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_plan_mixed_tags():
    # 3 tags of 3 / 2 / 3 groups over 3 ranks: rank r owns groups [8r/3, 8(r+1)/3)
    plans = [shard_plan([3, 2, 3], 4, r, 3) for r in range(3)]
    assert plans[0] == (0, 2, [(0, 0, 8)])
    assert plans[1] == (2, 3, [(0, 8, 12), (1, 12, 20)])
    assert plans[2] == (5, 3, [(2, 20, 32)])
    # every env exactly once, in order
    envs = [e for _, _, parts in plans for _, lo, hi in parts for e in range(lo, hi)]
    assert envs == list(range(32))
    assert shard_plan([3, 2, 3], 4, 0, 1) == (0, 8, [(0, 0, 12), (1, 12, 20), (2, 20, 32)])


def test_sharded_manager_needs_a_seed_without_group():
    es = EnvStateManager.__new__(EnvStateManager)
    es.process_group, es.rank, es.world_size = None, 1, 2
    with pytest.raises(ValueError, match="same train seed"):
        es._train_seed(None)
    assert es._train_seed(17) == 17


def test_two_rank_gloo_sharded_facade_host_logic():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    random.seed(5)
    want_seed = random.randint(0, 1000000)
    rows, scores = _rows()
    whole = _formulated(rows, scores, 0)
    cfg = _metrics_cfg()
    want_met = _ctx(cfg, 0, 1, None).device_metrics(_MetricEs(_metric_parts(0, 32)))
    assert any("non-zero" in k for k in want_met) and "FrozenLake/action_is_valid" in want_met
    for rank, seed, batch, nt, aliased, met in res:
        assert seed == want_seed, rank
        assert set(batch) == set(whole.batch.keys())
        for k in whole.batch.keys():
            assert torch.equal(torch.from_numpy(batch[k]), whole.batch[k]), (rank, k)
        assert aliased
        assert nt["env_ids"] == list(range(N_ROWS)) and nt["group_ids"] == [e // 4 for e in range(N_ROWS)]
        assert met == want_met, rank


def test_gather_formulated_lazy_ids():
    """gather_formulated over the device path's LazyDataProto: env / group ids come from its
    int64 ids (the object arrays made on read), without building the messages."""
    from ragen_amd.llm_agent.ctx_manager import LazyDataProto
    port = _free_port()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        rows, scores = _rows()
        plain = _formulated(rows, scores, 0)
        built = []
        lazy = LazyDataProto(np.arange(N_ROWS), lambda: built.append(1))
        lazy.set_device_batch({k: plain.batch[k] for k in plain.batch.keys()}, np.arange(N_ROWS), 4)
        out = rd.gather_formulated(lazy, PAD, dist.group.WORLD)
        assert list(out.non_tensor_batch["env_ids"]) == list(range(N_ROWS))
        assert list(out.non_tensor_batch["group_ids"]) == [e // 4 for e in range(N_ROWS)]
        assert torch.equal(out.batch["input_ids"], plain.batch["input_ids"])
        assert not built  # messages_list was not built
    finally:
        dist.destroy_process_group()
