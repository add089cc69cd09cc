"""Reproduce tests/test_gpu_exchange.py's W sequence (1, 2, 4 closed, then 8) and report where
the sources of the W=8 run get altered: pointers of every region and source, and after each
launch whether any source still equals its host copy."""
import sys

import torch

sys.path.insert(0, ".")
from ragen_amd import _lib  # noqa: E402
from ragen_amd.exchange import ArenaExchange, close_all  # noqa: E402

dev = torch.device("cuda", 0)
ARENA = 499712


def run(W, nbytes, epochs, verbose):
    exs = ArenaExchange.in_process(W, nbytes, dev)
    g = torch.Generator(device="cpu").manual_seed(W)
    host = [torch.randint(0, 256, (nbytes,), dtype=torch.uint8, generator=g) for _ in range(W)]
    srcs = [h.to(dev) for h in host]
    if verbose:
        print("regions", [hex(r) for r in exs[0].regions], flush=True)
        print("srcs", [hex(s.data_ptr()) for s in srcs], flush=True)
        print("state", [hex(x.state.data_ptr()) for x in exs], "err", [hex(x.err.data_ptr()) for x in exs], flush=True)

    def check(tag):
        torch.cuda.synchronize()
        bad = [r for r in range(W) if not torch.equal(srcs[r].cpu(), host[r])]
        if bad:
            r = bad[0]
            d = (srcs[r].cpu() != host[r]).nonzero().flatten()
            print(f"  {tag}: sources altered {bad}; rank {r}: {d.numel()} bytes at {d[:4].tolist()}..{d[-4:].tolist()}",
                  flush=True)
        return not bad

    for e in range(1, epochs + 1):
        for r in range(W):
            exs[r].run(srcs[r], _lib.XG_PUBLISH)
            if verbose and not check(f"e{e} after publish {r}"):
                break
        for r in range(W):
            exs[r].run(None, _lib.XG_WAIT)
            if verbose and not check(f"e{e} after wait {r}"):
                break
        want = torch.stack(srcs)
        for r in range(W):
            if not torch.equal(exs[r].slot(), want):
                print(f"W={W} e={e} rank {r}: slot != sources", flush=True)
                break
    torch.cuda.synchronize()
    close_all(exs)


for W, nb in ((1, ARENA), (2, ARENA), (4, 4096 + 48)):
    run(W, nb, 3, False)
    print("done", W, flush=True)
run(8, ARENA, 2, True)
print("end", flush=True)
