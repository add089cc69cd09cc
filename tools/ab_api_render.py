"""A/B (diagnostic): the API leg (bench.api_leg's device path) with the turn's render fused into
the turn launch (SokobanBatch.fused_render) and with the separate render launch, alternating,
3 runs each; prints env-steps/s and the turn loop per run."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from ragen_amd.env import SokobanBatch  # noqa: E402

dev = torch.device("cuda", 0)
res = {"fused": [], "separate": []}
for _ in range(3):
    for mode in ("fused", "separate"):
        SokobanBatch.fused_render = mode == "fused"
        d = bench.api_leg(dev)["device_path"]
        res[mode].append((round(d["env_steps_per_s"] / 1e6, 2), round(d["turn_loop_s"] * 1e3, 3)))
print(json.dumps(res))
