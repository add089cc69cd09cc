"""cProfile of the device-path turn loop (diagnostic): bench.api_leg's rollout (LLMAgentProxy on
the device path, an actor reading input_ids every turn; the setup of tools/prof_api_phases.py
without its synchronising wrappers), warmed up, then one rollout under cProfile; prints the top
functions by cumulative and by own time."""
import cProfile
import os
import pstats
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from ragen_amd import ops, synthetic  # noqa: E402
from ragen_amd.config import env_task  # noqa: E402
from ragen_amd.llm_agent import LLMAgentProxy, TokenActor  # noqa: E402
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


random.seed(0)  # one train-seed sequence: each reset takes the rooms the one before prefetched


def run():
    actor.turn = 0
    actor.prompts, actor.prompt_shapes = [], []  # (as bench.api_leg: the last rollout's batches let go)
    torch.cuda.synchronize()
    proxy.rollout(DataProto(meta_info={}), val=False)
    torch.cuda.synchronize()
    return dict(proxy.last_timing)


for _ in range(3):
    tm = run()
if __name__ == "__main__":  # (imported by prof_api_host.py for the setup and warm-up)
    print("plain:", {k: (round(v * 1e3, 2) if isinstance(v, float) else v) for k, v in tm.items()}, "ms")
    pr = cProfile.Profile()
    pr.enable()
    tm = run()
    pr.disable()
    print("profiled:", {k: (round(v * 1e3, 2) if isinstance(v, float) else v) for k, v in tm.items()}, "ms")
    st = pstats.Stats(pr)
    st.sort_stats("cumulative").print_stats(50)
    st.sort_stats("tottime").print_stats(35)
    st.sort_stats("cumulative").print_callees(r"es_manager.py:\d+\(reset\)")
    st.sort_stats("cumulative").print_callees(r"sokoban.py:\d+\(reset\)")
