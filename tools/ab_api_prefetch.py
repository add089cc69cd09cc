"""A/B (diagnostic): the API leg (bench.api_leg's device path) with the next reset's rooms
prefetched behind the rollout (EnvStateManager.prefetch_resets) and without, alternating, 4 runs
each (4 runs, both orders); prints env-steps/s, env-steps/s with the reset, the turn loop, the reset and whether the
reset took prefetched rooms."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from ragen_amd.llm_agent.es_manager import EnvStateManager  # noqa: E402

dev = torch.device("cuda", 0)
res = {"prefetch": [], "none": []}
for rep in range(4):
    for mode in (("prefetch", "none") if rep % 2 == 0 else ("none", "prefetch")):  # both orders
        EnvStateManager.prefetch_resets = mode == "prefetch"
        d = bench.api_leg(dev)["device_path"]
        res[mode].append((round(d["env_steps_per_s"] / 1e6, 2), round(d["env_steps_per_s_with_reset"] / 1e6, 2),
                          round(d["turn_loop_s"] * 1e3, 3), round(d["reset_s"] * 1e3, 3),
                          d["reset_rooms_prefetched"]))
print(json.dumps(res))
