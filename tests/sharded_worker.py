"""One rank of the sharded facade run (tests/test_gpu_sharded.py): started as a child process
(RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in the environment), joins a gloo process
group, rolls out its group-aligned shard through LLMAgentProxy on the device path (response
token ids on the GPU, device prompts) with gather=True, and writes what it saw to
``<out>/rank<r>.json``: the train seed its EnvStateManager used, each turn's generation batch
(env ids and a digest of every env's unpadded prompt ids), and digests of the gathered
formulated batch and its metrics."""
import hashlib
import json
import os
import random
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from fake_tok import FakeQwenTok  # noqa: E402
from ragen_amd import ops  # noqa: E402
from ragen_amd.config import env_task  # noqa: E402
from ragen_amd.llm_agent import LLMAgentProxy, TokenActor  # noqa: E402
from ragen_amd.protocol import DataProto  # noqa: E402

N_GROUPS, GS, T, K = 128, 16, 5, 5
NAMES = {1: "Up", 2: "Down", 3: "Left", 4: "Right", 0: "Jump"}  # 0: a name outside the lookup


def config():
    return env_task("SimpleSokoban", N_GROUPS, GS, max_turn=T, max_actions_per_turn=K)


def response_tokens(device):
    """Every env's response ids per turn (global env order), FakeQwenTok's one id per character:
    the synthetic actions written as '<thoughts></think> <answer>A || B</answer>'."""
    from ragen_amd import synthetic
    B = N_GROUPS * GS
    ids, n = synthetic.rollout_actions(B, T, K, 1, 4, seed=77)
    out = []
    for t in range(T):
        rows = []
        for i in range(B):
            acts = " || ".join(NAMES[int(a)] for a in ids[t, i, :int(n[t, i])])
            rows.append(f"env {i} turn {t}</think> <answer>{acts}</answer>".encode())
        R = max(len(r) for r in rows)
        a = np.full((B, R), FakeQwenTok.PAD, np.int64)
        for i, r in enumerate(rows):
            a[i, :len(r)] = np.frombuffer(r, np.uint8)
        out.append(torch.from_numpy(a).to(device))
    return out


def digest(*arrays) -> str:
    h = hashlib.sha256()
    for a in arrays:
        a = np.ascontiguousarray(a)
        h.update(str((a.dtype.str, a.shape)).encode())
        h.update(a.tobytes())
    return h.hexdigest()


def prompt_digests(input_ids, attention_mask, env_ids):
    """env id -> digest of its unpadded prompt ids (the batch is left-padded to its own width)."""
    ids, am = input_ids.cpu().numpy(), attention_mask.cpu().numpy().astype(bool)
    return {int(e): digest(ids[i][am[i]]) for i, e in enumerate(env_ids)}


def batch_digests(out):
    b = out.batch
    d = {k: digest(b[k].cpu().numpy()) for k in sorted(b.keys())}
    d["env_ids"] = digest(np.asarray(out.non_tensor_batch["env_ids"], np.int64))
    d["group_ids"] = digest(np.asarray(out.non_tensor_batch["group_ids"], np.int64))
    d["shape"] = list(b["input_ids"].shape)
    return d


class RecordingActor(TokenActor):
    """TokenActor that keeps each turn's (env ids, per-env prompt digests)."""

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.seen = []

    def generate_sequences(self, lm_inputs):
        b = lm_inputs.batch
        env_ids = np.asarray(lm_inputs.non_tensor_batch["env_ids"], np.int64)
        self.seen.append({"env_ids": env_ids.tolist(),
                          "prompts": prompt_digests(b["input_ids"], b["attention_mask"], env_ids)})
        return super().generate_sequences(lm_inputs)


def run(device, rank=None, world=None, group=None, train_seed_rng=7):
    """One rollout through the facade; -> (proxy, formulated batch, actor)."""
    tok = FakeQwenTok()
    cfg = config()
    tokens = response_tokens(device)
    kw = {}
    lo = 0
    if group is not None:
        from ragen_amd import distributed as rd
        g0, _ = rd.shard_groups(N_GROUPS, world, rank)
        lo = g0 * GS
        kw = dict(process_group=group, gather=True)
    actor = RecordingActor([x[lo:] for x in tokens], env_lo=lo)
    proxy = LLMAgentProxy(cfg, actor, tok, device=device, **kw)
    proxy.train_ctx_manager.set_device_vocab(ops.VocabTable.from_bytes(*tok.byte_table(), device))
    random.seed(train_seed_rng)  # rank 0's draw is the one every rank must use (broadcast)
    out = proxy.rollout(DataProto(meta_info={}), val=False)
    return proxy, out, actor


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    out_dir = sys.argv[1]
    device = torch.device("cuda", 0)
    torch.cuda.set_device(device)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # ranks other than 0 seed Python's RNG differently: only the broadcast makes them agree
        proxy, out, actor = run(device, rank, world, dist.group.WORLD, train_seed_rng=7 if rank == 0 else 1000 + rank)
        es = proxy.train_es_manager
        pr = proxy.train_ctx_manager.prompts()
        res = {"rank": rank, "env_lo": es.env_lo, "n_envs": es.n_envs,
               "train_seed": int(es._seeds[0] - es.env_lo // GS),
               "device_prompts": pr is not None, "host_rows": pr.host_rows_used if pr is not None else None,
               "turns": actor.seen, "batch": batch_digests(out),
               "metrics": {k: float(v) for k, v in out.meta_info["metrics"].items()}}
        with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
            json.dump(res, f)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
