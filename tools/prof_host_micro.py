"""Diagnostic: host cost of single calls of the turn loop (the GPU idle before each): a large
torch.empty of a generation batch's shape, ops.pad_rows, ops.h2d, the actor's row gather."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from ragen_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)


def t(fn, n=50):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        torch.cuda.synchronize()
        a = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - a)
    torch.cuda.synchronize()
    return f"{np.median(ts) * 1e6:7.1f} us (min {min(ts) * 1e6:.1f})"


n, S, cap = 7719, 638, 8192
arena = torch.zeros(8192, cap, dtype=torch.int64, device=dev)
alen = torch.full((8192,), 600, dtype=torch.int32, device=dev)
rows = torch.arange(n, dtype=torch.int64, device=dev)
tail = torch.arange(3, dtype=torch.int64, device=dev)
print("empty(3,n,S) i64      ", t(lambda: torch.empty(3, n, S, dtype=torch.int64, device=dev)))
print("empty(n,S) i64 x3     ", t(lambda: [torch.empty(n, S, dtype=torch.int64, device=dev) for _ in range(3)]))
print("empty(8192) u8        ", t(lambda: torch.empty(8192, dtype=torch.uint8, device=dev)))
print("ops.pad_rows          ", t(lambda: ops.pad_rows(arena, alen, rows, tail, S, 0)))
keep = []
print("pad_rows, kept (actor)", t(lambda: keep.append(ops.pad_rows(arena, alen, rows, tail, S, 0)), n=5))
keep.clear()
loc = np.arange(n, dtype=np.int64)
print("ops.h2d 60 KB         ", t(lambda: ops.h2d(loc, dev)))
tok = torch.zeros(8192, 80, dtype=torch.int64, device=dev)
print("actor gather          ", t(lambda: tok[ops.h2d(loc, dev)]))
print("torch.cuda.synchronize", t(lambda: None))
x = torch.zeros(16, dtype=torch.int32, device=dev)
print("ops.d2h               ", t(lambda: ops.d2h(x, ops)))
