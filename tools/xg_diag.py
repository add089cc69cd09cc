"""Diagnose the in-process one-shot exchange at W ranks: per rank and row, how many bytes of
the gathered slot differ from the senders' arenas, whether the differing bytes are zeros, and
whether a second read agrees.  python tools/xg_diag.py W mode epochs"""
import sys

import torch

sys.path.insert(0, ".")
from ragen_amd import _lib  # noqa: E402
from ragen_amd.exchange import ArenaExchange, close_all  # noqa: E402

W, mode, E = int(sys.argv[1]), sys.argv[2], int(sys.argv[3])
nbytes = 499712
dev = torch.device("cuda", 0)
exs = ArenaExchange.in_process(W, nbytes, dev, mode=mode)
g = torch.Generator(device="cpu").manual_seed(W)
srcs = [torch.randint(1, 256, (nbytes,), dtype=torch.uint8, generator=g).to(dev) for _ in range(W)]
for e in range(1, E + 1):
    for r in range(W):
        srcs[r].add_(1)
        srcs[r].clamp_(min=1)
    for r in range(W):
        exs[r].run(srcs[r], _lib.XG_PUBLISH)
    for r in range(W):
        exs[r].run(None, _lib.XG_WAIT)
    torch.cuda.synchronize()
    want = torch.stack(srcs)
    for r in range(W):
        got = exs[r].slot()
        bad = got != want
        if bad.any():
            rows = bad.sum(1).tolist()
            z = int((got[bad] == 0).sum())
            idx = bad.nonzero()[:4].tolist()
            again = exs[r].slot().clone()
            print(f"e={e} rank={r} bad_per_row={rows} zeros={z}/{int(bad.sum())} first={idx} "
                  f"reread_bad={int((again != want).sum())} err={exs[r].error()}", flush=True)
print("state", [x.state.tolist() for x in exs][:2], "err", [x.error() for x in exs], flush=True)
close_all(exs)
