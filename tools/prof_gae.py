"""Profiling driver: the bench's advantage leg (GAE legacy + row stats, then whitening) on
SK-shaped token rows, `--reps` times (for rocprofv3 --pmc / --kernel-trace)."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ragen_amd import ops, synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rows", type=int, default=8192)
    ap.add_argument("--cols", type=int, default=0, help="left-pad the rows to this many tokens (0: the batch max)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    n_turns = rng.integers(1, 6, size=a.rows)
    r, v, m = synthetic.token_rows(n_turns, rng.standard_normal(a.rows).astype(np.float32), seed=11, max_len=a.cols or None)
    r, v, m = (torch.from_numpy(x).to(dev) for x in (r, v, m))
    stats = torch.empty(a.rows, 3, dtype=torch.float64, device=dev)
    for _ in range(a.reps):
        adv, ret = ops.gae(r, v, m, 1.0, 1.0, row_stats=stats)
        ops.masked_whiten_(adv, m, stats)
    torch.cuda.synchronize()
    print("rows", r.shape)


if __name__ == "__main__":
    main()
