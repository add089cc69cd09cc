"""Run bench.api_leg alone (the LLMAgentProxy.rollout device path and the dict facade) and
print its JSON; with --profile, cProfile the device-path rollout's turn loop."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    if "--profile" in sys.argv:
        import cProfile
        import pstats
        cProfile.run("bench.api_leg(dev)", "/tmp/api.prof")
        pstats.Stats("/tmp/api.prof").sort_stats("cumulative").print_stats(40)
    print(json.dumps(bench.api_leg(dev)))
