"""rmi_assemble_batch / rmi_masks_and_scores timing (diagnostic, not product): the bench's
advantage-leg shapes (8192 rows of up to 1106 ids, ragged rows of L/2..L+1 tokens), HIP events
on the launch stream.   python tools/prof_assemble.py [--rows 8192] [--L 1105] [--reps 50]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ragen_amd import ops  # noqa: E402


def timed(fn, reps):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(2_000_000)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=8192)
    ap.add_argument("--L", type=int, default=1105)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    B, L, T = a.rows, a.L, 5
    g = torch.Generator(device=dev).manual_seed(3)
    ids = torch.randint(100, 1000, (B, L + 1), generator=g, device=dev, dtype=torch.int64)
    ids[torch.rand(B, L + 1, generator=g, device=dev) < 0.02] = 151644
    ids[torch.rand(B, L + 1, generator=g, device=dev) < 0.01] = 151645
    sc = torch.rand(T, B, generator=g, device=dev, dtype=torch.float64)
    n_sc = torch.randint(1, T + 1, (B,), generator=g, device=dev, dtype=torch.int32)
    lens = torch.randint(L // 2, L + 2, (B,), generator=g, device=dev)
    keep = torch.arange(L + 1, device=dev)[None, :] < lens[:, None]
    toks = ids[keep].contiguous()
    off = torch.zeros(B + 1, dtype=torch.int64, device=dev)
    off[1:] = torch.cumsum(lens, 0)
    S = int(lens.max())
    res = {}
    for _ in range(3):
        res.setdefault("masks", []).append(timed(
            lambda: ops.masks_and_scores(ids, 151644, 151645, sc, n_sc, T, False, True, True), a.reps))
        res.setdefault("assemble", []).append(timed(
            lambda: ops.assemble_batch(toks, off, S, 151643, 151644, 151645, sc, n_sc, T, False, True, True), a.reps))
    mb = B * (L + 1) * 14
    ab = toks.numel() * 8 + B * S * 24 + B * (S - 1) * 6
    for k, nb in (("masks", mb), ("assemble", ab)):
        us = min(res[k])
        print(f"{k:9s} {us:8.2f} us  {nb / us / 1e3:7.1f} GB/s  ({nb / 1e6:.1f} MB, runs {[round(x, 2) for x in res[k]]})")


if __name__ == "__main__":
    main()
