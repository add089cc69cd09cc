"""LLMAgentProxy — drop-in for ragen/llm_agent/agent_proxy.py:115-159 (the turn loop).

The actor is any object with ``generate_sequences(DataProto) -> DataProto`` (a veRL
RayWorkerGroup, a vLLM wrapper, or a scripted policy in tests/benchmarks).  LLM
generation itself (vLLM, API clients) is outside this engine's scope.
"""
import time
from typing import Dict, List

import numpy as np
import torch

from ..protocol import DataProto
from .ctx_manager import ContextManager
from .es_manager import EnvStateManager


def env_ids_of(dp: DataProto) -> np.ndarray:
    """The env ids of a batch as int64: a device-path LazyDataProto's own array (no trip through
    the reference's object array), else non_tensor_batch["env_ids"] converted."""
    ids = getattr(dp, "env_ids_i64", None)
    return ids if ids is not None else np.asarray(dp.non_tensor_batch["env_ids"], dtype=np.int64)


class ScriptedActor:
    """Stand-in LLM: returns one response text per env from a user callable
    ``policy(env_id, turn) -> str`` (no tokenizer round trip: non_tensor 'response_texts')."""

    def __init__(self, policy):
        self.policy = policy
        self.turn = 0

    def generate_sequences(self, lm_inputs: DataProto) -> DataProto:
        env_ids = lm_inputs.non_tensor_batch["env_ids"]
        out = DataProto(None, {"env_ids": env_ids,
                               "response_texts": [self.policy(int(e), self.turn) for e in env_ids]},
                        dict(lm_inputs.meta_info))
        self.turn += 1
        return out


class TokenActor:
    """Stand-in LLM whose generations are token ids on the GPU (what a device-resident policy or
    a vLLM worker on the same GPU hands back): ``turn_tokens[t]`` i64[n_envs, R] holds every
    env's response ids for turn t (rows by global env id - ``env_lo``); each call returns the
    rows of the envs asked for.  With ``read_prompts`` it reads the prompt batch the way a real
    actor does (agent_proxy.py:128-141: input_ids, attention_mask, position_ids), and keeps
    each turn's shapes in ``prompt_shapes``."""

    def __init__(self, turn_tokens, read_prompts: bool = False, env_lo: int = 0):
        self.turn_tokens = turn_tokens
        self.turn = 0
        self.read_prompts = read_prompts
        self.env_lo = env_lo
        self.prompt_shapes = []
        self.prompts = []

    def generate_sequences(self, lm_inputs: DataProto) -> DataProto:
        env_ids = env_ids_of(lm_inputs)
        if self.read_prompts:
            b = lm_inputs.batch
            self.prompt_shapes.append(tuple(b["input_ids"].shape))
            self.prompts.append((b["input_ids"], b["attention_mask"], b["position_ids"]))
        tok = self.turn_tokens[self.turn]
        rows = getattr(lm_inputs, "env_rows_device", None)
        if rows is not None and getattr(lm_inputs, "env_rows_lo", None) == self.env_lo:
            # the batch's env rows, ascending, on the device already: every env, or a gather
            resp = tok if rows.numel() == tok.shape[0] else tok.index_select(0, rows)
            self.turn += 1
            return DataProto({"responses": resp}, {"env_ids": env_ids}, {})
        if env_ids is not getattr(self, "_ids_seen", None) or tok.shape[0] != self._ids_n:
            local = env_ids - self.env_lo  # (the manager hands the same array each turn)
            self._ids_seen, self._ids_n = env_ids, tok.shape[0]
            self._ids_all = len(local) == tok.shape[0] and np.array_equal(local, np.arange(len(local)))
        if self._ids_all:
            resp = tok  # every env, in order
        else:
            from .. import ops
            resp = tok[ops.h2d(env_ids - self.env_lo, tok.device)]
        self.turn += 1
        return DataProto({"responses": resp}, {"env_ids": env_ids}, {})


class LLMAgentProxy:
    """agent_proxy.py:115-159.  Sharded (rank / world_size, or a process_group): each rank rolls
    out its group-aligned shard of the envs (EnvStateManager); with ``gather=True`` (and a
    process group) ``rollout`` reassembles the whole left-padded batch on every rank
    (ragen_amd.distributed.gather_formulated), as the single-controller reference builds it."""

    def __init__(self, config, actor_rollout_wg, tokenizer, device=None, rank=None, world_size=None,
                 process_group=None, gather: bool = False):
        self.config = config
        kw = dict(device=device, rank=rank, world_size=world_size, process_group=process_group)
        self.train_ctx_manager = ContextManager(config, tokenizer, mode="train", **kw)
        self.train_es_manager = EnvStateManager(config, mode="train", **kw)
        self.val_ctx_manager = ContextManager(config, tokenizer, mode="val", **kw)
        self.val_es_manager = EnvStateManager(config, mode="val", **kw)
        self.train_ctx_manager.attach_env_manager(self.train_es_manager)
        self.val_ctx_manager.attach_env_manager(self.val_es_manager)
        self.actor_wg = actor_rollout_wg
        self.tokenizer = tokenizer
        self.process_group = process_group
        self.gather = gather

    def generate_sequences(self, lm_inputs: DataProto) -> DataProto:
        out = self.actor_wg.generate_sequences(lm_inputs)
        if "env_ids" not in out.non_tensor_batch:
            out.non_tensor_batch["env_ids"] = lm_inputs.non_tensor_batch["env_ids"]
        return out

    def rollout(self, dataproto: DataProto, val: bool = False) -> DataProto:
        """agent_proxy.py:143-159."""
        es = self.val_es_manager if val else self.train_es_manager
        ctx = self.val_ctx_manager if val else self.train_ctx_manager
        if hasattr(self.actor_wg, "turn"):
            self.actor_wg.turn = 0
        from ..ops import D2H_COUNT  # device -> host readbacks of the device path, per phase
        c0 = D2H_COUNT[0]
        t0 = time.perf_counter()
        env_outputs: List[Dict] = es.reset()
        t1 = time.perf_counter()
        c1 = D2H_COUNT[0]
        for _ in range(self.config.agent_proxy.max_turn):
            lm_inputs = ctx.get_lm_inputs(env_outputs, prepare_for_update=False)
            lm_inputs.meta_info = dataproto.meta_info
            lm_outputs = self.generate_sequences(lm_inputs)
            env_inputs = ctx.get_env_inputs(lm_outputs)
            env_outputs = es.step(env_inputs)
            if len(env_outputs) == 0:
                break
        t2 = time.perf_counter()
        c2 = D2H_COUNT[0]
        rollout_states = es.get_rollout_states()
        t3 = time.perf_counter()
        out = ctx.formulate_rollouts(rollout_states)
        if self.gather and self.process_group is not None:
            from .. import distributed as rd
            pad = self.tokenizer.pad_token_id if getattr(self.tokenizer, "pad_token_id", None) is not None else 0
            out = rd.gather_formulated(out, pad, self.process_group, sizes=ctx.shard_sizes())
        # phase wall times of the last call (the turn loop is what env-steps/s is measured on)
        self.last_timing = {"reset_s": t1 - t0, "turns_s": t2 - t1, "rollout_states_s": t3 - t2,
                            "formulate_s": time.perf_counter() - t3,
                            "readbacks": {"reset": c1 - c0, "turns": c2 - c1, "after": D2H_COUNT[0] - c2}}
        # the next reset's room generation, behind the caller's use of this batch (the update)
        es.prefetch_next()
        return out
