"""cProfile of the API leg's two paths (bench.api_leg): the EnvStateManager.step dict facade,
and LLMAgentProxy.rollout on the device path with device prompts — top functions by own time."""
import cProfile
import os
import pstats
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from ragen_amd import ops, synthetic  # noqa: E402
from ragen_amd.config import env_task  # noqa: E402
from ragen_amd.llm_agent import EnvStateManager, LLMAgentProxy, TokenActor  # noqa: E402
from ragen_amd.protocol import DataProto  # noqa: E402

dev = torch.device("cuda", 0)
B, T, K = bench.B_PER_GPU, bench.T_TURNS, bench.K_ACTIONS
cfg = env_task("SimpleSokoban", B // bench.GROUP, bench.GROUP, max_turn=T, max_actions_per_turn=K)
ids, n = synthetic.rollout_actions(B, T, K, 1, 4)
names = {1: "Up", 2: "Down", 3: "Left", 4: "Right", 0: "Jump"}
turn_inputs = [[[names[int(a)] for a in ids[t, i, :int(n[t, i])]] for i in range(B)] for t in range(T)]


def dict_rollout(es):
    es.reset(seed=synthetic.ENV_SEED)
    active = list(range(B))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(T):
        outs = es.step([{"env_id": i, "llm_response": "", "llm_raw_response": "", "actions": turn_inputs[t][i]}
                        for i in active])
        active = [o["env_id"] for o in outs]
    return time.perf_counter() - t0


es = EnvStateManager(cfg, mode="train", device=dev)
for _ in range(2):
    print("dict path s:", dict_rollout(es))
pr = cProfile.Profile()
pr.enable()
dict_rollout(es)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(30)

tok = synthetic.qwen_like_tokenizer()
lk = {1: "Up", 2: "Down", 3: "Left", 4: "Right"}
tokens = []
for t in range(T):
    enc = tok(synthetic.responses_for_actions(ids[t], n[t], lk, seed=100 + t), padding=False).input_ids
    a = np.full((B, max(len(x) for x in enc)), tok.pad_token_id, np.int64)
    for i, x in enumerate(enc):
        a[i, :len(x)] = x
    tokens.append(torch.from_numpy(a).to(dev))
actor = TokenActor(tokens, read_prompts=True)
proxy = LLMAgentProxy(cfg, actor, tok, device=dev)
proxy.train_ctx_manager.set_device_vocab(ops.VocabTable.from_tokenizer(tok, dev))


def dev_rollout():
    random.seed(0)
    actor.turn = 0
    torch.cuda.synchronize()
    proxy.rollout(DataProto(meta_info={}), val=False)
    torch.cuda.synchronize()
    return dict(proxy.last_timing)


for _ in range(2):
    print("device path:", dev_rollout())
pr = cProfile.Profile()
pr.enable()
print("device path (profiled):", dev_rollout())
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(40)
pstats.Stats(pr).sort_stats("cumulative").print_stats(70)
