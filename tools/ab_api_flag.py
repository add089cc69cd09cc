"""A/B (diagnostic) of a class-attribute switch on the API rollout, in one process: bench.api_leg's
rollout (tools/prof_api_cprofile.py's setup and warm-up), then 2 x N rollouts alternating the
attribute between True and False; prints the median turn-loop, formulate and rollout times.
    python tools/ab_api_flag.py ragen_amd.llm_agent.prompts:DevicePrompts.first_bound [N]"""
import importlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numpy as np  # noqa: E402

import prof_api_cprofile as base  # noqa: E402  (builds the proxy, 3 warm-up rollouts)

mod, attr = sys.argv[1].split(":")
cls_name, field = attr.split(".")
cls = getattr(importlib.import_module(mod), cls_name)
N = int(sys.argv[2]) if len(sys.argv) > 2 else 10
res = {True: [], False: []}
for i in range(2 * N):
    v = i % 2 == 0
    setattr(cls, field, v)
    tm = base.run()
    res[v].append((tm["turns_s"], tm["formulate_s"], tm["turns_s"] + tm["rollout_states_s"] + tm["formulate_s"]))
setattr(cls, field, True)
for v in (True, False):
    a = np.array(res[v]) * 1e6
    print(f"{attr}={v}: turns {np.median(a[:, 0]):.1f} us, formulate {np.median(a[:, 1]):.1f} us, "
          f"rollout {np.median(a[:, 2]):.1f} us (median of {len(a)})")
