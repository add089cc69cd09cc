"""rmi_pad_rows (the generation batch of the device prompt path: ctx_manager.py:265-278's
left-padded input_ids / attention_mask / position_ids) against a torch restatement, on the
kernel's two forms: 16-B column pairs when the three outputs agree mod 16 B (rows that start at 8
mod 16 B store their first column alone, an odd remainder its last), and one column per lane when
they do not.  Covered: S odd and even, S = 1 and 2, overlong rows (the last S tokens, err =
RMI_ERR_UNSUP), empty arena rows, a row subset in any order."""
import numpy as np
import pytest
import torch

from ragen_amd import _lib
from ragen_amd._lib import lib

pytestmark = pytest.mark.gpu

PAD = 151643


def _want(arena, alen, rows, tail, S):
    n = rows.numel()
    ids = torch.full((n, S), PAD, dtype=torch.int64)
    am = torch.zeros(n, S, dtype=torch.int64)
    pos = torch.zeros(n, S, dtype=torch.int64)
    err = torch.zeros(n, dtype=torch.uint8)
    a, al, t = arena.cpu(), alen.cpu(), tail.cpu()
    for i, r in enumerate(rows.cpu().tolist()):
        tok = torch.cat([a[r, :int(al[r])], t])
        if tok.numel() > S:
            tok = tok[-S:]
            err[i] = _lib.ERR_UNSUP
        k = tok.numel()
        ids[i, S - k:] = tok
        am[i, S - k:] = 1
        pos[i, S - k:] = torch.arange(1, k + 1)
    return ids, am, pos, err


def _out(n, S, offs, dev):
    """Three [n, S] outputs at element offsets offs inside their own buffers (offset 1: 8 mod 16 B)."""
    outs = []
    for o in offs:
        buf = torch.full((n * S + 2,), -7, dtype=torch.int64, device=dev)
        outs.append(buf[o:o + n * S].view(n, S))
    return outs


@pytest.mark.parametrize("S", [1, 2, 5, 160, 1001])
@pytest.mark.parametrize("offs", [(0, 0, 0), (1, 1, 1), (0, 1, 0)])
def test_pad_rows_equals_torch(device, S, offs):
    g = torch.Generator().manual_seed(S * 7 + sum(offs))
    n_arena, cap = 300, 1200
    arena = torch.randint(0, 150000, (n_arena, cap), generator=g, dtype=torch.int64).to(device)
    alen = torch.randint(0, min(cap, S + 40) + 1, (n_arena,), generator=g).to(torch.int32)
    alen[:5] = 0
    alen = alen.to(device)
    rows = torch.randperm(n_arena, generator=g)[:257].to(device)  # odd row count: odd n * S offsets
    tail = torch.tensor([151644, 77091, 198], dtype=torch.int64, device=device)
    ids, am, pos = _out(rows.numel(), S, offs, device)
    err = torch.full((rows.numel(),), 0xEE, dtype=torch.uint8, device=device)
    rc = lib().rmi_pad_rows(arena.data_ptr(), cap, alen.data_ptr(), rows.data_ptr(), rows.numel(), tail.data_ptr(),
                            tail.numel(), S, PAD, ids.data_ptr(), am.data_ptr(), pos.data_ptr(), err.data_ptr(),
                            torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    w = _want(arena, alen, rows, tail, S)
    for got, want, name in zip((ids, am, pos, err), w, ("input_ids", "attention_mask", "position_ids", "err")):
        assert torch.equal(got.cpu(), want), name
    assert np.any(w[3].numpy() != 0) or S > 1000  # overlong rows are exercised
