"""Where the time of the device prompt kernels goes (diagnostic, not product): builds
prompt.hip or bpe.hip with RMI_STAMPS (tools/build_variant.sh prst prompt.hip -DRMI_STAMPS /
bpst bpe.hip -DRMI_STAMPS), runs bench.api_leg's rollout (8192 envs) on that library and prints,
per launch of the rollout, the mean cycles of each phase and the peak number of resident waves.
    python tools/prof_prompt_stamps.py prompt|bpe"""
import ctypes
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WHICH = sys.argv[1] if len(sys.argv) > 1 else "prompt"
SO = os.environ.get("RAGEN_AMD_STAMP_SO") or os.path.join(
    os.environ.get("RAGEN_AMD_VARIANT_DIR", os.path.join(ROOT, "tools", "_build")),
    "libragen_amd_%s.so" % ("prst" if WHICH == "prompt" else "bpst"))
os.environ["RAGEN_AMD_LIB"] = SO
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from ragen_amd import ops, synthetic  # noqa: E402
from ragen_amd.config import env_task  # noqa: E402
from ragen_amd.llm_agent import LLMAgentProxy, TokenActor  # noqa: E402
from ragen_amd.llm_agent import prompts as pm  # noqa: E402
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

lib = ctypes.CDLL(SO)
setter = lib.rmi_prompt_set_stamps if WHICH == "prompt" else lib.rmi_bpe_set_stamps
stamps = torch.zeros(B * 16, dtype=torch.int64, device=dev)
dummy = torch.zeros(B * 16, dtype=torch.int64, device=dev)
# the stamped kernels write through g_stamps unconditionally: point it at a buffer before any
# launch (the prompt builder's constructor already encodes)
assert setter(ctypes.c_void_p(dummy.data_ptr())) == 0
calls = [0]
name = "_run_text" if WHICH == "prompt" else "_encode"
orig = getattr(pm.DevicePrompts, name)
bufs, lens = [], []


def hooked(self, *a, **kw):
    calls[0] += 1
    torch.cuda.synchronize()
    buf = torch.zeros(B * 16, dtype=torch.int64, device=dev)
    bufs.append(buf)
    if WHICH == "bpe":
        lens.append(int(a[1].max()))
    setter(ctypes.c_void_p(buf.data_ptr()))
    return orig(self, *a, **kw)


setattr(pm.DevicePrompts, name, hooked)
# the chained turns (round 5: rmi_turn_chain runs the prompt text and the BPE of every turn)
from ragen_amd.llm_agent import turn_chain as tcm  # noqa: E402
orig_run = tcm.TurnChain.run


def hooked_run(self, inp, t):
    calls[0] += 1
    torch.cuda.synchronize()
    buf = torch.zeros(B * 16, dtype=torch.int64, device=dev)
    setter(ctypes.c_void_p(buf.data_ptr()))
    r = orig_run(self, inp, t)
    if r is not None:
        bufs.append(buf)
        if WHICH == "bpe":
            lens.append(r[2].prompt[3])  # the BPE launch's row bound
    return r


tcm.TurnChain.run = hooked_run
random.seed(0)
actor.turn = 0
proxy.rollout(DataProto(meta_info={}), val=False)
torch.cuda.synchronize()
names = {"prompt": ["stage", "pieces up to the reward", "the reward piece", "the rest + stores"],
         "bpe": ["stage", "classes + added + match lengths + chain", "word cache + symbols", "merges"]}[WHICH]
if WHICH == "bpe" and ("fine" in os.path.basename(SO) or "bpstf" in os.path.basename(SO)):  # -DRMI_BPE_FINE
    names = ["1 classes", "2 added tokens", "3 match lengths", "4 chain"]
for c, buf in enumerate(bufs):
    s = buf.view(B, 16).cpu().numpy().astype(np.float64)
    ok = (s[:, 0] > 0) & np.all(np.diff(s[:, 0:10:2], axis=1) > 0, axis=1)
    a = s[ok]
    if not len(a):
        continue
    ph = [a[:, 2 * (i + 1)] - a[:, 2 * i] for i in range(4)]
    # waves resident at once: a sweep over the (start, end) realtime events
    ev = sorted([(t, 1) for t in a[:, 1]] + [(t, -1) for t in a[:, 9]])
    cur = peak = 0
    for _, d in ev:
        cur += d
        peak = max(peak, cur)
    ml = f" max_len {lens[c]}" if lens else ""
    print(f"{WHICH} call {c}:{ml} {int(ok.sum())} of {B} waves: mean cycles "
          + "  ".join(f"{nm} {p.mean():.0f}" for nm, p in zip(names, ph))
          + f"  | span {(a[:, 8] - a[:, 0]).mean():.0f} cycles, {(a[:, 9] - a[:, 1]).mean() / 100:.2f} us realtime; "
          f"first-to-last wave start {(a[:, 1].max() - a[:, 1].min()) / 100:.1f} us, "
          f"window {(a[:, 9].max() - a[:, 1].min()) / 100:.1f} us, peak resident waves {peak}")
