"""tests/test_gpu_exchange.py's split test body, in one process, for the W sequence 1, 2, 4, 8,
under variants: receive memory mode, whether closed exchanges free their regions, and a
synchronize after every epoch.  Prints the first failure of each variant.
  python tools/xg_diag3.py MODE FREE SYNC"""
import sys

import torch

sys.path.insert(0, ".")
from ragen_amd import _lib  # noqa: E402
from ragen_amd.exchange import ArenaExchange  # noqa: E402

mode, free, sync = sys.argv[1], sys.argv[2] == "1", sys.argv[3] == "1"
dev = torch.device("cuda", 0)
ARENA = 499712
keep = []


def _arena(rank, epoch, base):
    return base[rank] ^ torch.tensor((rank * 131 + epoch * 29) & 255, dtype=torch.uint8, device=base[rank].device)


def body(W, nbytes, epochs=20):
    exs = ArenaExchange.in_process(W, nbytes, dev, mode=mode)
    g = torch.Generator(device="cpu").manual_seed(W)
    base = [torch.randint(0, 256, (nbytes,), dtype=torch.uint8, generator=g).to(dev) for _ in range(W)]
    base_h = [b.cpu() for b in base]
    srcs = [torch.empty(nbytes, dtype=torch.uint8, device=dev) for _ in range(W)]
    msg = "ok"
    for e in range(1, epochs + 1):
        for r in range(W):
            srcs[r].copy_(_arena(r, e, base))
        for r in range(W):
            exs[r].run(srcs[r], _lib.XG_PUBLISH)
        for r in range(W):
            exs[r].run(None, _lib.XG_WAIT)
        if sync:
            torch.cuda.synchronize()
        want = torch.stack(srcs)
        bad_base = [q for q in range(W) if not torch.equal(base[q].cpu(), base_h[q])]
        bad_slot = [r for r in range(W) if not torch.equal(exs[r].slot(), want)]
        exp = [(base_h[q] ^ ((q * 131 + e * 29) & 255)) for q in range(W)]
        bad_src = [q for q in range(W) if not torch.equal(srcs[q].cpu(), exp[q])]
        bad_row = [q for q in range(W) if not torch.equal(exs[0].slot()[q].cpu(), exp[q])]
        if bad_base or bad_slot or bad_src:
            from ragen_amd.exchange import region_bytes
            nreg = region_bytes(W, nbytes)
            ptrs = [x.data_ptr() for x in srcs + base + [t for x in exs for t in (x.state, x.err)]]
            overlap = [hex(p) for p in ptrs for r in exs[0].regions if r <= p < r + nreg]
            msg = (f"e={e} base altered {bad_base} slots!=srcs {bad_slot} srcs!=expected {bad_src} "
                   f"slot0 rows!=expected {bad_row} overlap {overlap}")
            break
    torch.cuda.synchronize()
    errs = [x.error() for x in exs]
    if free:
        for x in exs:
            x.close()
    else:
        keep.append(exs)
    print(f"  W={W}: {msg} err {errs}", flush=True)


print(f"== mode={mode} free={free} sync={sync}", flush=True)
for W, nb in ((1, ARENA), (2, ARENA), (4, 4096 + 48), (8, ARENA)):
    body(W, nb)
