"""The validation rollout, agent_trainer._validate's `rollout(val=True)` (agent_trainer.py:241):
LLMAgentProxy.rollout on the val managers -- EnvStateManager(mode="val"), the fixed seed 123
(es_manager.py:88-91), group_size 1 (base.yaml:119-123) -- against the reference's own run of
the same loop (tests/golden/val_rollout.json, make_golden_val.py: 256 SimpleSokoban + 32
FrozenLake groups, synthetic generations, the FakeQwenTok character tokenizer).

Both paths: the device path (generations as token ids on the GPU, decoded, parsed, stepped,
rendered and prompted on the device) and the dict path (host decode + list-of-dict turns).
Every turn's generation batch the actor reads, the formulated batch, its metrics, the env /
group ids and the rollout cache must equal the reference's."""
import hashlib

import numpy as np
import pytest
import torch

from fake_tok import FakeQwenTok
from ragen_amd import ops
from ragen_amd.config import default_config
from ragen_amd.llm_agent import LLMAgentProxy, TokenActor
from ragen_amd.protocol import DataProto
from test_gpu_facade import _hashseed0_reseed
from test_val_fixture_cpu import load_val

pytestmark = pytest.mark.gpu


def _digest(t):
    return hashlib.sha256(t.detach().cpu().contiguous().numpy().tobytes()).hexdigest()


def _jsonable(x):
    if isinstance(x, dict):
        return {str(k): _jsonable(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_jsonable(v) for v in x]
    if isinstance(x, np.floating):
        return float(x)
    if isinstance(x, np.integer):
        return int(x)
    if isinstance(x, np.bool_):
        return bool(x)
    return x


def _turn_tokens(d, tok, n_envs, device):
    """Per turn the generations as token ids, one row per env (envs without one: padding)."""
    out = []
    for turn in d["turns"]:
        rows = {e: tok._ids(x) for e, x in zip(turn["env_ids"], turn["responses"])}
        R = max(len(r) for r in rows.values())
        a = np.full((n_envs, R), tok.pad_token_id, np.int64)
        for e, r in rows.items():
            a[e, :len(r)] = r
        out.append(torch.from_numpy(a).to(device))
    return out


@pytest.mark.parametrize("device_path", [True, False], ids=["device", "dict"])
def test_val_rollout_matches_reference(device, device_path, monkeypatch):
    from ragen_amd.env import SokobanBatch
    monkeypatch.setattr(SokobanBatch, "reseed_fn", staticmethod(_hashseed0_reseed))
    d = load_val()
    cfg = default_config(**d["overrides"])
    tok = FakeQwenTok()
    actor = TokenActor(_turn_tokens(d, tok, 288, device), read_prompts=True)
    proxy = LLMAgentProxy(cfg, actor, tok, device=device)
    if device_path:
        proxy.val_ctx_manager.set_device_vocab(ops.VocabTable.from_bytes(*tok.byte_table(), device))
    out = proxy.rollout(DataProto(meta_info={}), val=True)
    es = proxy.val_es_manager
    assert es.mode == "val" and proxy.train_es_manager.rollout_id == 0  # the train managers untouched
    # every turn's generation batch, as the actor read it
    assert len(actor.prompts) == len(d["turns"])
    for t, (p, ref) in enumerate(zip(actor.prompts, d["turns"])):
        assert list(p[0].shape) == ref["shape"], t
        for k, x in zip(("input_ids", "attention_mask", "position_ids"), p):
            assert _digest(x) == ref["sha256"][k], (t, k)
    # the formulated batch (ctx_manager.py:354-356)
    f = d["formulated"]
    b = out.batch
    assert list(b["input_ids"].shape) == f["shape"]
    for k in ("input_ids", "attention_mask", "position_ids", "responses", "loss_mask", "rm_scores",
              "original_rm_scores"):
        assert _digest(b[k]) == f["sha256"][k], k
    assert [int(e) for e in out.non_tensor_batch["env_ids"]] == f["env_ids"]
    assert [int(g) for g in out.non_tensor_batch["group_ids"]] == f["group_ids"]
    assert _jsonable(out.meta_info["metrics"]) == f["metrics"]
    # the rollout cache after formulate (its histories trimmed in place, as the reference's)
    assert _jsonable(es.rollout_cache) == d["rollout_cache"]
    if device_path:
        pr = proxy.val_ctx_manager.prompts()
        assert pr is not None and pr.host_rows_used == 0
        assert b["input_ids"].is_cuda


def test_val_reset_is_seed_123_every_time(device, monkeypatch):
    """Two val rollouts start from the same rooms (seed 123 regardless of `random`), unlike
    train resets (a drawn seed)."""
    from ragen_amd.env import SokobanBatch
    from ragen_amd.llm_agent import EnvStateManager
    monkeypatch.setattr(SokobanBatch, "reseed_fn", staticmethod(_hashseed0_reseed))
    d = load_val()
    cfg = default_config(**d["overrides"])
    es = EnvStateManager(cfg, mode="val", device=device)
    first = [o["history"][0]["state"] for o in es.reset()]
    import random
    random.seed(99)
    second = [o["history"][0]["state"] for o in es.reset()]
    assert first == second == d["init_obs"]
