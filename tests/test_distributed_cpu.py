"""world_size-2 gloo test of the multi-GPU sharding path on the CPU.

Each rank runs its group-aligned shard of the SK rollout (compute by the CPU oracle — the
HIP kernels need a GPU; the kernels' parity with the oracle is covered by the gpu tests),
then the real exchange steps of ragen_amd.distributed: global group scores for the rollout
filter, whitening statistics, and trajectory reassembly.  Every result must equal the
single-process computation on the full batch.
"""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from ragen_amd import distributed as rd
from ragen_amd import ops, synthetic

G_TOTAL, GS, T, K = 32, 16, 5, 5


def _rollout(first_group, n_groups):
    B = n_groups * GS
    seeds = synthetic.env_seeds(B, first_group=first_group)
    uniq, inv = np.unique(seeds, return_inverse=True)
    f, s, p, st = ops.generate_sokoban_rooms(uniq, 6, 6, 1, 300)
    assert not st.any()
    fixed, state, player = f[inv], s[inv].copy(), p[inv].copy()
    ids_all, n_all = synthetic.rollout_actions(G_TOTAL * GS, T, K, 1, 4)
    lo = first_group * GS
    ids, n = ids_all[:, lo:lo + B], n_all[:, lo:lo + B]
    ep = oracle.Episode(B, T)
    nes, bot = np.zeros(B, np.int32), np.zeros(B, np.int32)
    for t in range(T):
        oracle.sokoban_turn(6, 6, 1, 100, fixed, state, player, nes, bot, ep, t, ids[t], n[t])
    score, pen = oracle.trajectory_scores(ep)
    stats = []
    for g in range(n_groups):  # token rows seeded by the GLOBAL group id: independent of sharding
        sl = slice(g * GS, (g + 1) * GS)
        r, v, m = synthetic.token_rows(ep.n_turns[sl], (score + pen)[sl], seed=100 + first_group + g, max_len=1200)
        adv, ret = oracle.gae(r, v, m, 1.0, 1.0)
        a64 = adv.astype(np.float64)
        stats.append(np.stack([(a64 * m).sum(1), ((a64 ** 2) * m).sum(1), m.sum(1).astype(np.float64)], 1))
    stats = np.concatenate(stats)
    return {"score": score + pen, "turn_reward": ep.turn_reward.T.copy(), "stats": stats, "state": state}


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, ng = rd.shard_groups(G_TOTAL, world, rank)
    out = _rollout(first, ng)
    scores = rd.gather_group_scores(torch.from_numpy(out["score"]), GS).numpy()
    stats = rd.global_whiten_stats(torch.from_numpy(out["stats"])).numpy()
    # host-known shard sizes: no size exchange (equal shards: one all_gather_into_tensor)
    sized = rd.global_whiten_stats(torch.from_numpy(out["stats"]), sizes=rd.shard_rows(G_TOTAL, GS, world)).numpy()
    rag = torch.arange(rank + 3, dtype=torch.float64) + 100 * rank  # ragged: 3 and 4 rows
    rag_sized, off = rd.all_gather_rows(rag, with_offset=True, sizes=[3 + r for r in range(world)])
    try:
        rd.all_gather_rows(rag, sizes=[4, 3])  # wrong on both ranks (a rank whose count matches would
        bad = False                            # enter the collective and wait for the other)
    except ValueError:
        bad = True  # raised on the host before any collective
    traj = rd.gather_rollout({"turn_reward": torch.from_numpy(out["turn_reward"]),
                              "state": torch.from_numpy(out["state"])})
    keep, met, _ = oracle.filter_groups(scores, G_TOTAL, GS, 0.25, "std")
    # the whole episode record in one collective (same shard shape on every rank)
    ep = ops.EpisodeState.empty(ng * GS, T, "cpu")
    ep.turn_reward.copy_(torch.from_numpy(out["turn_reward"].T.copy()))
    ep.flags.fill_(rank + 1)
    views = rd.episode_views(rd.gather_episode(ep), ng * GS, T)
    ep_tr = torch.cat([v.turn_reward for v in views], dim=1).numpy()
    ep_fl = [int(v.flags[0]) for v in views]
    extra = {"sized": sized, "rag": rag_sized.numpy(), "rag_unsized": rd.all_gather_rows(rag).numpy(), "off": off,
             "bad": bad}
    q.put((rank, scores, stats, traj["turn_reward"].numpy(), traj["state"].numpy(), keep, met, ep_tr, ep_fl, extra))
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_groups_partition():
    for W in (1, 2, 4, 8):
        parts = [rd.shard_groups(4096, W, r) for r in range(W)]
        assert sum(n for _, n in parts) == 4096
        assert all(parts[i][0] + parts[i][1] == parts[i + 1][0] for i in range(W - 1))
        assert all(n == 4096 // W for _, n in parts)


def test_two_rank_gloo_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = _rollout(0, G_TOTAL)
    fkeep, fmet, _ = oracle.filter_groups(full["score"], G_TOTAL, GS, 0.25, "std")
    for rank, scores, stats, tr, state, keep, met, ep_tr, ep_fl, extra in res:
        np.testing.assert_array_equal(extra["sized"], full["stats"])
        np.testing.assert_array_equal(extra["rag"], [0, 1, 2, 100, 101, 102, 103])
        np.testing.assert_array_equal(extra["rag_unsized"], extra["rag"])
        assert extra["off"] == (0, 3)[rank]
        assert extra["bad"]
        np.testing.assert_array_equal(ep_tr, full["turn_reward"].T)   # gather_episode == full record
        assert ep_fl == [1, 2]
        np.testing.assert_array_equal(scores, full["score"])        # bit-identical global scores
        np.testing.assert_array_equal(tr, full["turn_reward"])
        np.testing.assert_array_equal(state, full["state"])
        np.testing.assert_array_equal(keep, fkeep)                   # identical filter on every rank
        np.testing.assert_array_equal(met, fmet)
        # whitening statistics: per-row partials in global order -> identical global reduction
        assert stats.shape == full["stats"].shape
        np.testing.assert_array_equal(stats, full["stats"])
