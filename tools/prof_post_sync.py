"""Diagnostic: host time from the turn's readback to the next launch (the GPU idles meanwhile) --
wall-clock stamps at the readback's return, the end of EnvStateManager.step, the start of
get_lm_inputs, the generation batch's pad_rows call and the actor, for the last of 4 rollouts
of bench.api_leg's setup; microseconds after the readback, per turn."""
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import prof_api_cprofile as base  # noqa: E402  (the proxy, warmed up)
from ragen_amd import ops  # noqa: E402
from ragen_amd.llm_agent import ctx_manager as cm, es_manager as em, prompts as pm  # noqa: E402

ST = []


def stamp(label, fn):
    def run(*a, **k):
        ST.append((label + ">", time.perf_counter()))
        r = fn(*a, **k)
        ST.append((label + "<", time.perf_counter()))
        return r
    return run


ops.d2h = stamp("d2h", ops.d2h)
for cls, names in ((em.EnvStateManager, ("step", "_device_pass")), (cm.ContextManager, ("get_lm_inputs", "get_env_inputs")),
                   (pm.DevicePrompts, ("gen_batch", "advance_eager"))):
    for nm in names:
        setattr(cls, nm, stamp(nm, getattr(cls, nm)))
import ragen_amd.torch_ops as to  # noqa: E402
for nm in ("pad_rows", "detok_parse", "prompt_text", "bpe_encode", "gen_rows"):
    fn = getattr(to.direct, nm)
    setattr(to.direct, nm, stamp(nm, fn))
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
