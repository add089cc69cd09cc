"""Run bench.toytext_legs alone (FrozenLake 4096 x 8 and Countdown 16384 x 4 rollouts, graph
replayed) and print its JSON."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    print(json.dumps(bench.toytext_legs(torch.device("cuda", 0))))
