"""Diagnostic: wall-clock stamps of the device turn loop with the turn chain (round 5) -- the
host's time between the chain's readback and the next launches, per call of the facade's
functions; the last of 4 warm rollouts of bench.api_leg's setup.  Prints the stamp trace and a
per-label sum of the time spent inside each stamped call (nested calls counted in both)."""
import collections
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import prof_api_cprofile as base  # noqa: E402  (the proxy, warmed up)
from ragen_amd import _lib, ops  # noqa: E402
from ragen_amd.llm_agent import agent_proxy as ap, ctx_manager as cm, es_manager as em, prompts as pm  # noqa: E402
from ragen_amd.llm_agent import turn_chain as tc  # noqa: E402
import ragen_amd.torch_ops as to  # noqa: E402
from ragen_amd import tokenizer as tk  # noqa: E402

ST = []


def stamp(label, fn):
    def run(*a, **k):
        ST.append((label + ">", time.perf_counter()))
        r = fn(*a, **k)
        ST.append((label + "<", time.perf_counter()))
        return r
    return run


for nm in ("d2h", "h2d", "count_nonzero_into"):
    setattr(ops, nm, stamp(nm, getattr(ops, nm)))
for cls, names in ((em.EnvStateManager, ("step", "_step_device", "_turn_chain", "get_rollout_states")),
                   (em.LazyEnvOutputs, ("__init__",)),
                   (cm.ContextManager, ("get_lm_inputs", "get_env_inputs", "_device_env_inputs", "_sync_prompts",
                                        "prompts", "formulate_rollouts")),
                   (cm.LazyDataProto, ("__init__", "set_device_batch")),
                   (pm.DevicePrompts, ("gen_batch", "_pad_rows", "_resolve", "turn_pieces", "_program", "_text_bound",
                                       "_obs_bound")),
                   (cm.ContextManager, ("turn_packs",)),
                   (tc.TurnChain, ("run", "_slot", "_parse")),
                   (tk.DeviceTokenizer, ("bpe_struct",)),
                   (ap.LLMAgentProxy, ("generate_sequences",))):
    for nm in names:
        setattr(cls, nm, stamp(nm, getattr(cls, nm)))
pm._storage_uses = stamp("_storage_uses", pm._storage_uses)
import torch  # noqa: E402
_empty = torch.empty
torch.empty = stamp("torch.empty", _empty)
em.STEP_STAMPS = ST  # _step_device's own checkpoints (t1..t5) into the same trace
es_cls = em.EnvStateManager
es_cls._ascending = stamp("_ascending", es_cls._ascending)
L = _lib.lib()
L.rmi_turn_chain = stamp("rmi_turn_chain", L.rmi_turn_chain)
to.direct.pad_rows = stamp("pad_rows", to.direct.pad_rows)
base.actor.generate_sequences = stamp("actor", base.actor.generate_sequences)
for _ in range(3):
    base.run()
ST.clear()
tm = base.run()
print("rollout", {k: (round(v * 1e3, 3) if isinstance(v, float) else v) for k, v in tm.items()})
t_prev = ST[0][1]
for lab, t in ST:
    print(f"{(t - t_prev) * 1e6:9.1f} us  {lab}")
    t_prev = t
inside = collections.defaultdict(float)
count = collections.Counter()
open_ = {}
for lab, t in ST:
    name, kind = lab[:-1], lab[-1]
    if kind not in "<>":  # (a checkpoint, no span)
        continue
    if kind == ">":
        open_.setdefault(name, []).append(t)
    else:
        inside[name] += t - open_[name].pop()
        count[name] += 1
print("\nper label: total us, calls")
for name, v in sorted(inside.items(), key=lambda x: -x[1]):
    print(f"  {name:28s} {v * 1e6:9.1f} {count[name]:4d}")
# the rows the chain's kernels saw against the bounds they were sized by
ch = base.proxy.train_es_manager.__dict__.get("_chain")
if ch is not None:
    print("\nslot: decode stride / longest decoded row | prompt row bound (pstride, bpe stride) / longest prompt text")
    for t, s in sorted(ch.slots.items()):
        if s.prompt is None:
            continue
        print(f"  turn {t}: {s.text.shape[1]} / {int(s.tlen.max())} | {s.prompt[2]}, {s.prompt[3]} / "
              f"{int(s.ptext_len.max())}  (mean {float(s.ptext_len.float().mean()):.1f})")
