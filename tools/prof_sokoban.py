"""Profiling driver: the bench workload's rollout, eager, `--reps` times (for rocprofv3 --pmc).

    rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES ... -d out -o pmc --output-format csv -- python3 tools/prof_sokoban.py
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from bench import Rollout  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--envs", type=int, default=8192)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    R = Rollout(dev, 0, B=a.envs)
    for _ in range(a.reps):
        R.step_unfused()  # T plain turn launches: the per-launch counters of the turn kernel alone
    torch.cuda.synchronize()
    print("steps per rollout", int(R.env.ep.turn_exec.sum().item()))


if __name__ == "__main__":
    main()
