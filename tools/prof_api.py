"""Host profile of the EnvStateManager facade on the SK workload (cProfile, top functions)."""
import cProfile
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    bench.api_leg(dev)  # warm
    pr = cProfile.Profile()
    pr.enable()
    print(bench.api_leg(dev))
    pr.disable()
    pstats.Stats(pr).sort_stats("cumulative").print_stats(25)
