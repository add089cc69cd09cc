"""BASELINE.json configs[3] — Sokoban 6x6, 65 536 envs sharded 8 x 8192 — on
the HIP path, and the sharded facade end to end.

* The 8 group-aligned shards (group offsets 512 r, env offsets 8192 r) run one after another
  on this GPU through EnvStateManager(rank=r, world_size=8): the concatenated record (episode
  arena, rooms, players, counters) equals one 65 536-env run and the oracle, bit for bit;
  the rollout metrics and trajectory scores too.
* The exchange steps over the 8 shards' partials — what the all-gathers of
  ragen_amd.distributed hand every rank, concatenated in rank order — equal the whole-batch
  results: the rollout filter (agent_trainer.py:461-500) from the shards' scores, and
  masked whitening from the shards' per-row fp64 partials (bit-equal; oracle within 1e-5).
* 8 ranks as 8 processes on this GPU over a gloo group (tests/sharded_worker.py):
  LLMAgentProxy(process_group=..., gather=True) on the device path; every rank uses rank 0's
  train seed (broadcast), sees exactly its envs' prompts, and ends with the gathered
  left-padded batch (ctx_manager.py:278-306) and metrics of the one-process run.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

import oracle
from ragen_amd import ops, synthetic
from ragen_amd.config import env_task
from ragen_amd.env import SokobanBatch
from ragen_amd.llm_agent import EnvStateManager

pytestmark = pytest.mark.gpu

B_ALL, W, T, K, GS = 65536, 8, 5, 5, 16
SEED = synthetic.ENV_SEED
EP_FIELDS = ("num_actions", "flags", "n_turns", "penalty", "turn_reward", "turn_info", "turn_exec")
ENV_FIELDS = ("room_state", "player", "num_env_steps", "boxes_on_target")


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _cfg():
    return env_task("SimpleSokoban", B_ALL // GS, GS, max_turn=T, max_actions_per_turn=K)


def _roll(es, ids, n, lo, hi, device):
    es.reset(seed=SEED)
    for t in range(T):
        es.step_tensor(_t(ids[t, lo:hi], device), _t(n[t, lo:hi], device))
    b = es.tags[0].batch
    rec = {k: getattr(b.ep, k).cpu().numpy() for k in EP_FIELDS}
    rec.update({k: getattr(b, k).cpu().numpy() for k in ENV_FIELDS})
    rec["metrics"] = ops.rollout_metrics(b.ep).cpu().numpy()
    s, p = ops.trajectory_scores(b.ep)
    rec["score"], rec["pen"] = s.cpu().numpy(), p.cpu().numpy()
    return rec


def _cat(parts, k):
    ax = 1 if parts[0][k].ndim == 2 and k.startswith("turn_") else 0  # turn-major [T, B] fields
    return np.concatenate([p[k] for p in parts], axis=ax)


def _token_rows(n_turns, score, g0, ng):
    """GAE rows of groups [g0, g0+ng), each group seeded by its GLOBAL id (sharding-independent)."""
    parts = [synthetic.token_rows(n_turns[g * GS:(g + 1) * GS], score[g * GS:(g + 1) * GS], seed=100 + g0 + g,
                                  max_len=1280) for g in range(ng)]
    return [np.concatenate([p[i] for p in parts]) for i in range(3)]


@pytest.fixture(scope="module")
def sk8(device):
    cfg = _cfg()
    ids, n = synthetic.rollout_actions(B_ALL, T, K, 1, 4)
    whole_es = EnvStateManager(cfg, device=device)
    whole = _roll(whole_es, ids, n, 0, B_ALL, device)
    shards = []
    for r in range(W):
        es = EnvStateManager(cfg, device=device, rank=r, world_size=W)
        assert (es.first_group, es.n_local_groups, es.env_lo, es.n_envs) == (512 * r, 512, 8192 * r, 8192)
        shards.append(_roll(es, ids, n, es.env_lo, es.env_lo + es.n_envs, device))
        np.testing.assert_array_equal(es._seeds, synthetic.env_seeds(8192, first_group=512 * r))
        del es
    return whole, shards, ids, n


def test_sk8_shards_equal_whole_batch_and_oracle(sk8):
    whole, shards, ids, n = sk8
    for k in EP_FIELDS + ENV_FIELDS + ("metrics", "score", "pen"):
        np.testing.assert_array_equal(_cat(shards, k), whole[k], err_msg=k)
    # the oracle on the whole batch, from independently generated rooms of the same seeds
    fixed, state, player = SokobanBatch.generate(synthetic.env_seeds(B_ALL), 6, 6, 1, 300)
    state, player = state.copy(), player.copy()
    oep = oracle.Episode(B_ALL, T)
    nes, bot = np.zeros(B_ALL, np.int32), np.zeros(B_ALL, np.int32)
    for t in range(T):
        err = oracle.sokoban_turn(6, 6, 1, 100, fixed, state, player, nes, bot, oep, t, ids[t], n[t])
        assert not err.any()
    for k in EP_FIELDS:
        np.testing.assert_array_equal(whole[k], getattr(oep, k), err_msg=k)
    np.testing.assert_array_equal(whole["room_state"], state)
    np.testing.assert_array_equal(whole["player"], player)
    np.testing.assert_array_equal(whole["num_env_steps"], nes)
    np.testing.assert_array_equal(whole["boxes_on_target"], bot)
    np.testing.assert_array_equal(whole["metrics"], oracle.rollout_metrics(oep))
    os_, op_ = oracle.trajectory_scores(oep)
    np.testing.assert_array_equal(whole["score"], os_)
    np.testing.assert_array_equal(whole["pen"], op_)
    assert oep.turn_exec.sum() > 500_000  # the workload really stepped (≈68 k env steps per 8192 envs)


def test_sk8_global_filter_over_shards(sk8, device):
    """The filter over the 8 shards' gathered scores == the whole batch's == the oracle; each
    rank keeps its slice of the global keep mask."""
    whole, shards, _, _ = sk8
    G = B_ALL // GS
    gathered = torch.cat([_t(p["score"] + p["pen"], device) for p in shards])  # all_gather_rows, rank order
    for ftype in ("std", "std_rev"):
        keep, met, _ = ops.filter_groups(gathered, G, GS, 0.25, ftype)
        wkeep, wmet, _ = ops.filter_groups(_t(whole["score"] + whole["pen"], device), G, GS, 0.25, ftype)
        okeep, omet, _ = oracle.filter_groups(whole["score"] + whole["pen"], G, GS, 0.25, ftype)
        assert torch.equal(keep, wkeep) and torch.equal(met, wmet)
        np.testing.assert_array_equal(keep.cpu().numpy(), okeep)
        np.testing.assert_array_equal(met.cpu().numpy(), omet)
        assert int(keep.sum()) == G // 4
        # rank r's slice (rd.global_filter keeps keep[g0:g0 + n_local])
        for r in range(W):
            assert torch.equal(keep[512 * r:512 * (r + 1)], wkeep[512 * r:512 * (r + 1)])


def test_sk8_global_whitening_over_shards(sk8, device):
    """GAE per shard with per-row fp64 partials; masked whitening of every shard with the 8
    shards' partials in rank order (rd.global_whiten_stats) == whitening the whole batch."""
    whole, shards, _, _ = sk8
    score = whole["score"] + whole["pen"]
    r, v, m = _token_rows(whole["n_turns"], score, 0, B_ALL // GS)
    tr, tv, tm = _t(r, device), _t(v, device), _t(m, device)
    wstats = torch.zeros(B_ALL, 3, dtype=torch.float64, device=device)
    wadv, wret = ops.gae(tr, tv, tm, 1.0, 1.0, row_stats=wstats)
    ops.masked_whiten_(wadv, tm, wstats)
    advs, rets, stats = [], [], []
    for k in range(W):
        sl = slice(8192 * k, 8192 * (k + 1))
        st = torch.zeros(8192, 3, dtype=torch.float64, device=device)
        a, rt = ops.gae(tr[sl].contiguous(), tv[sl].contiguous(), tm[sl].contiguous(), 1.0, 1.0, row_stats=st)
        advs.append(a)
        rets.append(rt)
        stats.append(st)
    gstats = torch.cat(stats)
    assert torch.equal(gstats, wstats)
    for a in advs:
        ops.masked_whiten_stats_(a, gstats)
    torch.cuda.synchronize()
    assert torch.equal(torch.cat(rets), wret)
    assert torch.equal(torch.cat(advs), wadv)
    oadv, oret = oracle.gae(r, v, m, 1.0, 1.0)
    np.testing.assert_array_equal(wret.cpu().numpy(), oret)
    np.testing.assert_allclose(wadv.cpu().numpy(), oracle.masked_whiten(oadv, m), rtol=0, atol=1e-5)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(400)
def test_sharded_facade_8_ranks_gloo(device, tmp_path):
    """8 ranks (processes) on this GPU over gloo, each rolling out its shard through
    LLMAgentProxy on the device path and gathering the formulated batch, against one process
    rolling out the whole batch."""
    import sharded_worker as sw
    W8 = 8
    port = _free_port()
    here = os.path.dirname(os.path.abspath(__file__))
    procs = []
    for r in range(W8):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(W8), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), OMP_NUM_THREADS="2")
        log = open(tmp_path / f"rank{r}.log", "w")
        procs.append((subprocess.Popen([sys.executable, "-u", os.path.join(here, "sharded_worker.py"), str(tmp_path)],
                                       env=env, stdout=log, stderr=subprocess.STDOUT), log))
    try:
        for p, _ in procs:
            p.wait(timeout=360)
    finally:
        for p, log in procs:
            if p.poll() is None:
                p.kill()
            log.close()
    for r, (p, _) in enumerate(procs):
        assert p.returncode == 0, (tmp_path / f"rank{r}.log").read_text()[-4000:]
    res = [json.loads((tmp_path / f"rank{r}.json").read_text()) for r in range(W8)]
    # the one-process run of the whole batch
    proxy, out, actor = sw.run(device)
    es = proxy.train_es_manager
    seed = int(es._seeds[0])
    want = sw.batch_digests(out)
    want_metrics = {k: float(v) for k, v in out.meta_info["metrics"].items()}
    n_loc = es.n_envs // W8
    for r, d in enumerate(res):
        assert (d["env_lo"], d["n_envs"]) == (r * n_loc, n_loc)
        assert d["train_seed"] == seed, "the train seed was not broadcast from rank 0"
        assert d["device_prompts"] and d["host_rows"] == 0
        assert len(d["turns"]) == len(actor.seen)
        for t, (mine, full) in enumerate(zip(d["turns"], actor.seen)):
            ids = [e for e in full["env_ids"] if r * n_loc <= e < (r + 1) * n_loc]
            assert mine["env_ids"] == ids, (r, t)
            assert mine["prompts"] == {str(e): full["prompts"][e] for e in ids}, (r, t)
        assert d["batch"] == want, r          # the gathered batch == the whole batch, on every rank
        assert d["metrics"] == want_metrics, r
