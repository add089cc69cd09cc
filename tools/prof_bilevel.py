"""Bi-level GAE timing (diagnostic, not product): SK-shaped turn-score rows (the bench's
advantage leg shape: 8192 rows, 1-5 turns, reward on each turn's last response token), the
segment-parallel kernel and the tiled kernel (RAGEN_AMD_BILEVEL_TILED=1) alternated, HIP events
on the launch stream.   python tools/prof_bilevel.py [--rows 8192] [--reps 50]"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ragen_amd import ops, synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=8192)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--max-len", type=int, default=None, help="left-pad the rows to this many tokens (4096: out of cache)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    n_turns = rng.integers(1, 6, size=a.rows)
    tr = np.full((a.rows, 5), 0.5, np.float32)
    r, v, m = synthetic.token_rows(n_turns, np.zeros(a.rows, np.float32), seed=12, turn_scores=tr, max_len=a.max_len)
    tokens = r.size
    r, v, m = (torch.from_numpy(x).to(dev) for x in (r, v, m))
    res = {}
    for rnd in range(3):
        for mode in ("0", "1"):
            os.environ["RAGEN_AMD_BILEVEL_TILED"] = mode
            for _ in range(3):
                ops.bilevel_gae(r, v, m, 1.0, 0.95, 0.95, check_errors=False)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(2_000_000)
            e0.record()
            for _ in range(a.reps):
                ops.bilevel_gae(r, v, m, 1.0, 0.95, 0.95, check_errors=False)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.reps
            res.setdefault(mode, []).append(us)
    for mode, name in (("0", "segment"), ("1", "tiled")):
        us = min(res[mode])
        print(f"{name:8s} {us:8.2f} us  {17 * tokens / us / 1e3:7.1f} GB/s  (rows {tuple(r.shape)}, runs {res[mode]})")


if __name__ == "__main__":
    main()
