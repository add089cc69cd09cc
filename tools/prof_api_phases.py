"""Where the device-path turn loop's time goes (diagnostic): bench.api_leg's rollout with each
phase wrapped in a synchronize + wall clock (so the GPU work of a phase is charged to it), and
the rollout timed plain for comparison.  Phases: DevicePrompts.start / advance (prompt text +
BPE), gen_batch, the actor, get_env_inputs, EnvStateManager.step, get_rollout_states,
formulate_rollouts."""
import os
import random
import sys
import time
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from ragen_amd import ops, synthetic  # noqa: E402
from ragen_amd.config import env_task  # noqa: E402
from ragen_amd.llm_agent import LLMAgentProxy, TokenActor  # noqa: E402
from ragen_amd.llm_agent import ctx_manager as cm, es_manager as em, prompts as pm  # noqa: E402
from ragen_amd.protocol import DataProto  # noqa: E402

dev = torch.device("cuda", 0)
B, T, K = bench.B_PER_GPU, bench.T_TURNS, bench.K_ACTIONS
cfg = env_task("SimpleSokoban", B // bench.GROUP, bench.GROUP, max_turn=T, max_actions_per_turn=K)
ids, n = synthetic.rollout_actions(B, T, K, 1, 4)
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


def run():
    random.seed(0)
    actor.turn = 0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    proxy.rollout(DataProto(meta_info={}), val=False)
    torch.cuda.synchronize()
    return time.perf_counter() - t0, dict(proxy.last_timing)


for _ in range(3):
    wall, tm = run()
print("plain:", {k: (round(v * 1e3, 2) if isinstance(v, float) else v) for k, v in tm.items()}, "ms")

acc = defaultdict(float)
cnt = defaultdict(int)


def wrap(obj, name, label):
    f = getattr(obj, name)

    def g(*a, **kw):
        torch.cuda.synchronize()
        t = time.perf_counter()
        r = f(*a, **kw)
        torch.cuda.synchronize()
        acc[label] += time.perf_counter() - t
        cnt[label] += 1
        return r
    setattr(obj, name, g)


wrap(pm.DevicePrompts, "start", "prompts.start")
wrap(pm.DevicePrompts, "advance", "prompts.advance")
wrap(pm.DevicePrompts, "gen_batch", "prompts.gen_batch")
wrap(pm.DevicePrompts, "_run_text", "  prompt_text")
wrap(pm.DevicePrompts, "_encode", "  bpe encode + host rows")
wrap(TokenActor, "generate_sequences", "actor")
wrap(cm.ContextManager, "get_env_inputs", "get_env_inputs")
wrap(em.EnvStateManager, "_step_device", "es.step (device)")
wrap(em.EnvStateManager, "_decode_parse", "  detok_parse")
wrap(em.EnvStateManager, "_parsed_turn", "  turn")
wrap(em.EnvStateManager, "get_rollout_states", "get_rollout_states")
wrap(cm.ContextManager, "formulate_rollouts", "formulate_rollouts")
wall, tm = run()
acc.clear()
cnt.clear()
wall, tm = run()
print("phased:", {k: (round(v * 1e3, 2) if isinstance(v, float) else v) for k, v in tm.items()}, "ms")
for k in acc:
    print(f"  {k:28s} {acc[k] * 1e3:8.2f} ms  ({cnt[k]} calls)")
