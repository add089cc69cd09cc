"""Host cost of the calls one device-path turn makes (diagnostic): after a warm rollout of
bench.api_leg's setup, each call timed on the host alone (synchronised before, the enqueue
time measured, then synchronised) — what the turn loop pays per call when the GPU is idle."""
import os
import sys
import time

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
ctx = proxy.train_ctx_manager
ctx.set_device_vocab(ops.VocabTable.from_tokenizer(tok, dev))
for _ in range(2):
    actor.turn, actor.prompts = 0, []
    proxy.rollout(DataProto(meta_info={}), val=False)
torch.cuda.synchronize()
pr = ctx.prompts()
es = proxy.train_es_manager
env_ids = es.env_lo + np.arange(es.n_envs, dtype=np.int64)


def host(label, fn, reps=50):
    fn()
    torch.cuda.synchronize()
    tot = 0.0
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        tot += time.perf_counter() - t0
        torch.cuda.synchronize()
    print(f"{label:44s} {tot / reps * 1e6:8.1f} us")


x8 = torch.zeros(B, dtype=torch.uint8, device=dev)
xi = torch.zeros(B, dtype=torch.int32, device=dev)
rows = torch.arange(B, dtype=torch.int64, device=dev)
S = int(pr.len.max()) + pr.tail.numel()
host("torch.zeros(B, u8)", lambda: torch.zeros(B, dtype=torch.uint8, device=dev))
host("x & 4 == 0 (2 ops)", lambda: (x8 & 4) == 0)
host("int(x.max()) (op + sync)", lambda: int(xi.max()))
host("torch.from_numpy(ids).to(dev)", lambda: torch.from_numpy(env_ids).to(dev))
host("torch.cat([x8, x8]).cpu().numpy()", lambda: torch.cat([x8, x8]).cpu().numpy())
host("ops.pad_rows (ctypes)", lambda: ops.pad_rows(pr.arena, pr.len, rows, pr.tail, S, 0))
host("torch.ops.ragen_amd.pad_rows", lambda: torch.ops.ragen_amd.pad_rows(pr.arena, pr.len, rows, pr.tail, S, 0))
host("DevicePrompts.gen_batch", lambda: pr.gen_batch(env_ids))
tg = es.tags[0]
host("sokoban render_rows (op)", lambda: tg.batch.render_rows())
host("LazyDataProto + set_device_batch", lambda: __import__("ragen_amd.llm_agent.ctx_manager", fromlist=["x"])
     .LazyDataProto(env_ids, None).set_device_batch({"input_ids": x8}, env_ids, 16))
