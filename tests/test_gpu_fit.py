"""RayAgentTrainer.fit's use of the rollout, replayed on the engine (agent_trainer.py:514-633):
LLMAgentProxy.rollout -> _filter_rollout -> uid -> response_mask -> _balance_batch (reorder)
-> global_token_num -> DummyRewardManager -> worker groups (compute_log_prob /
compute_values through a DP_COMPUTE_PROTO-style chunk + concat) -> union -> token-level
rewards -> compute_advantage -> critic / actor updates, with stub worker groups.  The
formulated batch must be single-device (CPU, as the reference's), every DataProto step must
keep rows aligned, and the advantages must equal the oracle on the final batch."""
import uuid

import numpy as np
import pytest
import torch

import oracle
from fake_tok import FakeQwenTok
from ragen_amd.config import env_task
from ragen_amd.llm_agent import LLMAgentProxy, ScriptedActor
from ragen_amd.protocol import DataProto
from ragen_amd.trainer import DummyRewardManager, compute_advantage, compute_reward, filter_rollout

pytestmark = pytest.mark.gpu


class StubWorkerGroup:
    """A worker group with `world` data-parallel workers: DP_COMPUTE_PROTO splits the batch into
    equal chunks, each worker computes on its chunk, the results are concatenated."""

    def __init__(self, world=4):
        self.world = world
        self.seen = []

    def _dp(self, data: DataProto, fn):
        return DataProto.concat([fn(p) for p in data.chunk(self.world)])

    def compute_log_prob(self, data):
        return self._dp(data, lambda p: DataProto.from_dict(
            {"old_log_probs": -(p.batch["responses"].float() % 7) / 10}))

    def compute_values(self, data):
        def values(p):
            g = torch.Generator().manual_seed(int(p.batch["input_ids"].sum()) % (2 ** 31))
            return DataProto.from_dict({"values": torch.randn(p.batch["responses"].shape, generator=g)
                                        * p.batch["response_mask"].float()})
        return self._dp(data, values)

    def _update(self, data, kind):
        for p in data.chunk(self.world):
            assert {"advantages", "returns", "response_mask", "old_log_probs"} <= set(p.batch.keys())
            self.seen.append((kind, len(p)))
        return DataProto(meta_info={"metrics": {f"{kind}/loss": 0.0}})

    def update_critic(self, data):
        return self._update(data, "critic")

    def update_actor(self, data):
        return self._update(data, "actor")


def _rollout(device, groups=8, gs=16):
    cfg = env_task("SimpleSokoban", groups, gs, max_turn=5, max_actions_per_turn=5)
    cfg.agent_proxy.reward_normalization.method = "mean_std"
    rng = np.random.default_rng(1)
    names = ["Up", "Down", "Left", "Right", "Jump"]

    def policy(env_id, turn):
        acts = " || ".join(names[int(x)] for x in rng.integers(0, 5, size=int(rng.integers(1, 4))))
        return f"think</think><answer>{acts}</answer>"
    tok = FakeQwenTok()
    proxy = LLMAgentProxy(cfg, ScriptedActor(policy), tok, device=device)
    return proxy.rollout(DataProto(meta_info={}), val=False), tok


@pytest.mark.parametrize("estimator,bi_level", [("gae", False), ("gae", True), ("grpo", False)])
def test_fit_sequence_on_rollout(device, estimator, bi_level):
    groups, gs = 8, 16
    batch, tok = _rollout(device, groups, gs)
    # the formulated batch is single-device, on the CPU like the reference's
    assert {v.device.type for v in batch.batch.values()} == {"cpu"}, {k: v.device for k, v in batch.batch.items()}
    assert batch.batch["original_rm_scores"] is batch.batch["rm_scores"]
    # _filter_rollout (agent_trainer.py:461-500)
    batch, metrics = filter_rollout(batch, groups, gs, 0.5, "std")
    assert len(batch) == groups // 2 * gs
    metrics.update({"train/" + k: v for k, v in batch.meta_info["metrics"].items()})
    # _process_batch_for_logging
    inputs = [tok.decode(ids, skip_special_tokens=True) for ids in batch.batch["input_ids"]]
    scores = batch.batch["rm_scores"].sum(-1).cpu().tolist()
    assert len(inputs) == len(scores) == len(batch)
    env_of_row = {i: int(e) for i, e in enumerate(batch.non_tensor_batch["env_ids"])}
    score_of_env = {env_of_row[i]: s for i, s in enumerate(scores)}
    # uid, response_mask
    batch.non_tensor_batch["uid"] = np.array([str(uuid.uuid4()) for _ in range(len(batch.batch))], dtype=object)
    batch.batch["response_mask"] = batch.batch["loss_mask"]
    # _balance_batch: token counts -> a balanced order -> reorder in place
    seqlen = batch.batch["attention_mask"].view(len(batch), -1).sum(-1)
    perm = torch.argsort(seqlen, descending=True, stable=True)
    perm = torch.cat([perm[i::4] for i in range(4)])  # round-robin over 4 DP ranks
    batch.reorder(perm)
    for i, e in enumerate(batch.non_tensor_batch["env_ids"]):  # rows stay aligned
        assert abs(float(batch.batch["rm_scores"][i].sum()) - score_of_env[int(e)]) < 1e-6
    batch.meta_info["global_token_num"] = torch.sum(batch.batch["attention_mask"], dim=-1).tolist()
    # reward, old log-probs, values
    reward_tensor, extra = compute_reward(batch, DummyRewardManager(tok, 0))
    assert reward_tensor is batch.batch["rm_scores"]
    wg, critic = StubWorkerGroup(), StubWorkerGroup()
    batch = batch.union(wg.compute_log_prob(batch))
    values = critic.compute_values(batch)
    batch = batch.union(values)
    with pytest.raises(ValueError):
        batch.union(DataProto.from_dict({"values": values.batch["values"] + 1}))
    batch.batch["token_level_scores"] = reward_tensor
    batch.batch["token_level_rewards"] = batch.batch["token_level_scores"]
    r = batch.batch["token_level_rewards"].numpy()
    v = batch.batch["values"].numpy()
    m = batch.batch["response_mask"].numpy().astype(np.uint8)
    kw = dict(gamma=1.0, lam=1.0, num_repeat=1, norm_adv_by_std_in_grpo=True, multi_turn=True, high_level_gamma=0.95,
              bi_level_gae=bi_level)
    if bi_level and oracle.bilevel_gae(r, v, m, 1.0, 1.0, 0.95)[2].any():
        with pytest.raises(IndexError):  # a row whose score is exactly 0 (core_algos.py:79)
            compute_advantage(batch, estimator, **kw)
        nz = r[:, -1] != 0
        batch = batch.select_idxs(torch.from_numpy(nz))
        r, v, m = r[nz], v[nz], m[nz]
    batch = compute_advantage(batch, estimator, **kw)
    adv, ret = batch.batch["advantages"], batch.batch["returns"]
    assert adv.device.type == "cpu" and adv.shape == batch.batch["responses"].shape
    if estimator == "gae" and not bi_level:
        oadv, oret = oracle.gae(r, v, m, 1.0, 1.0)
        np.testing.assert_array_equal(ret.numpy(), oret)
        np.testing.assert_allclose(adv.numpy(), oracle.masked_whiten(oadv, m), rtol=0, atol=1e-5)
    elif estimator == "gae":
        oadv, oret, oerr = oracle.bilevel_gae(r, v, m, 1.0, 1.0, 0.95)
        assert not oerr.any()
        np.testing.assert_array_equal(ret.numpy(), oret)
        np.testing.assert_allclose(adv.numpy(), oracle.masked_whiten(oadv, m), rtol=0, atol=1e-5)
    else:
        seg = np.arange(len(batch) + 1, dtype=np.int32)  # unique uids: groups of one
        oadv, _ = oracle.grpo(r, m, seg)
        np.testing.assert_allclose(adv.numpy(), oadv, rtol=1e-6, atol=1e-6)
    if len(batch) % 4 == 0:
        critic.update_critic(batch)
        batch.meta_info["multi_turn"] = True
        wg.update_actor(batch)
        assert [n for _, n in critic.seen] == [len(batch) // 4] * 4


def test_estimator_errors_with_gpu_inputs(device):
    """verl's / RAGEN's error cases raise for GPU callers too (check=True, the default): a mask
    sum of 0 or 1 (verl masked_var -> ValueError) and a bi-level row whose last loss-mask
    position carries no reward (core_algos.py:79 -> IndexError); check=False leaves them
    unread (no host synchronisation)."""
    from ragen_amd.trainer import core_algos
    B, L = 4, 16
    r = torch.zeros(B, L, device=device)
    v = torch.randn(B, L, device=device)
    for n_on in (0, 1):
        m = torch.zeros(B, L, dtype=torch.uint8, device=device)
        m.view(-1)[:n_on] = 1
        with pytest.raises(ValueError):
            core_algos.compute_gae_advantage_return(r, v, m, 1.0, 1.0)
        with pytest.raises(ValueError):
            core_algos.masked_whiten(v, m)
        core_algos.compute_gae_advantage_return(r, v, m, 1.0, 1.0, check=False)
    m = torch.ones(B, L, dtype=torch.uint8, device=device)
    rb = torch.zeros(B, L, device=device)
    rb[:, 5] = 1.0  # the reward is not on the last valid column of any row
    with pytest.raises(IndexError):
        core_algos.compute_bi_level_gae_advantage_return(rb, v, m, 1.0, 1.0, 0.95)
    rb[:, -1] = 2.0
    adv, ret = core_algos.compute_bi_level_gae_advantage_return(rb, v, m, 1.0, 1.0, 0.95)
    assert adv.is_cuda and torch.isfinite(adv).all()
