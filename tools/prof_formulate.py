"""Host anatomy of formulate_rollouts on the device path (diagnostic): bench.api_leg's rollout
(tools/prof_api_cprofile.py's setup and warm-up), then 16 rollouts, FormulateChain.overlap on
and off alternating, with perf_counter wrappers around the pieces of FormulateChain.run; prints
per piece the median microseconds per rollout, and the phase's wall time per form."""
import os
import sys
import time
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numpy as np  # noqa: E402

import prof_api_cprofile as base  # noqa: E402  (builds the proxy, 3 warm-up rollouts)
from ragen_amd import _lib  # noqa: E402
from ragen_amd.llm_agent import ctx_manager, turn_chain  # noqa: E402

T = defaultdict(list)
cur = defaultdict(float)


def wrap(obj, name, label):
    f = getattr(obj, name)

    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            cur[label] += time.perf_counter() - t0
    setattr(obj, name, w)


L = _lib.lib()
for fn in ("rmi_formulate_stats", "rmi_readback", "rmi_formulate_chain"):
    wrap(L, fn, fn)
ctx = base.proxy.train_ctx_manager
wrap(ctx, "device_metrics", "device_metrics")
wrap(ctx, "_sync_prompts", "_sync_prompts")
wrap(ctx_manager.LazyDataProto, "set_device_batch", "set_device_batch")
wrap(ctx_manager.LazyDataProto, "__init__", "LazyDataProto.__init__")
wrap(turn_chain, "ref_f32_mean", "ref_f32_mean")
pr = ctx.prompts()
wrap(pr, "update_rows", "update_rows")
wrap(pr, "_resolve", "_resolve")
wrap(turn_chain.FormulateChain, "run", "FormulateChain.run")
wrap(ctx, "formulate_rollouts", "formulate_rollouts")

for i in range(16):  # alternating: the host's reductions beside the assembly / after it
    turn_chain.FormulateChain.overlap = i % 2 == 0
    cur.clear()
    tm = base.run()
    for k, v in cur.items():
        T[k].append(v)
    tag = "overlap" if i % 2 == 0 else "serial"
    T[f"(proxy formulate_s, {tag})"].append(tm["formulate_s"])
    T["(proxy turns_s)"].append(tm["turns_s"])
turn_chain.FormulateChain.overlap = True
print("median us per rollout over 16 rollouts (8 per formulate form)")
for k, v in sorted(T.items(), key=lambda kv: -np.median(kv[1])):
    print(f"{np.median(v) * 1e6:10.1f}  {k}")
