"""The one-shot arena exchange (ragen_amd/exchange.py, rmi_xgather) on the GPU.

* W ranks' exchanges inside one process (regions shared directly, no IPC), every rank's PUBLISH
  then every rank's WAIT on one stream, 100 epochs: every rank's slot of every epoch == the W
  arenas of that epoch (the two-slot reuse and the consumed back-pressure included).
* The fused form (PUBLISH + WAIT in one launch) at W = 1, and the 1-rank exchange's error
  path: a missing peer (a region nobody writes) ends in RMI_XG_ERR_* within the timeout, the
  grid drained.
* W ranks as W processes on this GPU (tests/xgather_worker.py): regions mapped through HIP IPC,
  handles exchanged over gloo, 100 fused exchanges each, every slot checked byte for byte and
  by the owners' all-gathered digests (bench.arena_digests)."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

from ragen_amd import _lib
from ragen_amd.exchange import ArenaExchange, close_all, plan

pytestmark = pytest.mark.gpu
ARENA = 499712  # the SK arena: 8192 envs x 5 turns (EpisodeState.layout)


def _arena(rank, epoch, base):
    return base[rank] ^ torch.tensor((rank * 131 + epoch * 29) & 255, dtype=torch.uint8, device=base[rank].device)


@pytest.mark.parametrize("W,nbytes", [(1, ARENA), (2, ARENA), (4, 4096 + 48), (8, ARENA)])
def test_in_process_split_exchange(device, W, nbytes):
    exs = ArenaExchange.in_process(W, nbytes, device, timeout_us=2_000_000)
    try:
        g = torch.Generator(device="cpu").manual_seed(W)
        base = [torch.randint(0, 256, (nbytes,), dtype=torch.uint8, generator=g).to(device) for _ in range(W)]
        srcs = [torch.empty(nbytes, dtype=torch.uint8, device=device) for _ in range(W)]
        for e in range(1, 101):
            for r in range(W):
                srcs[r].copy_(_arena(r, e, base))
            for r in range(W):
                exs[r].run(srcs[r], _lib.XG_PUBLISH)
            for r in range(W):
                exs[r].run(None, _lib.XG_WAIT)
            want = torch.stack(srcs)
            for r in range(W):
                assert exs[r].epoch == e
                got = exs[r].slot()
                if not torch.equal(got, want):
                    d = (got != want).nonzero()
                    exp = torch.stack([_arena(q, e, base) for q in range(W)])
                    raise AssertionError(
                        f"W={W} e={e} rank {r}: {d.shape[0]} bytes differ, first {d[:3].tolist()} last {d[-3:].tolist()}; "
                        f"slot==regenerated {torch.equal(got, exp)} sources==regenerated {torch.equal(want, exp)}; "
                        f"srcs {[hex(x.data_ptr()) for x in srcs]} regions {[hex(q) for q in exs[0].regions]} "
                        f"state {[hex(x.state.data_ptr()) for x in exs]} err {[hex(x.err.data_ptr()) for x in exs]} "
                        f"base {[hex(x.data_ptr()) for x in base]}")
            if e >= 2:  # the previous epoch's slot is intact until epoch e + 1 rewrites it
                prev = torch.stack([_arena(q, e - 1, base) for q in range(W)])
                assert torch.equal(exs[0].slot(e - 1), prev)
        assert all(x.error() == 0 for x in exs)
        assert [int(v) for v in exs[0].state.cpu()] == [100, 100 * W * plan(W, nbytes)["blocks_per_peer"]]
    finally:
        torch.cuda.synchronize(device)
        close_all(exs)


def test_fused_single_rank_and_plan(device):
    """W = 1: the fused launch (the --double-buffer shape) leaves the arena in slot e & 1."""
    (ex,) = ArenaExchange.in_process(1, ARENA, device)
    try:
        p = plan(1, ARENA)
        assert p["blocks_per_peer"] == 61 and p["grid"] == 62 and p["row_bytes"] == 499712
        src = torch.randint(0, 256, (ARENA,), dtype=torch.uint8, device=device)
        for e in range(1, 6):
            src.add_(1)
            ex.run(src)
            assert torch.equal(ex.slot()[0], src)
        assert ex.error() == 0
    finally:
        close_all([ex])


def test_missing_peer_times_out_and_drains(device):
    """Rank 0 of 2 exchanges alone: its WAIT sees no arrivals from rank 1 and sets
    RMI_XG_ERR_ARRIVALS after the 20-ms timeout; then its third PUBLISH finds rank 1's consumed
    stuck at 0 and sets RMI_XG_ERR_PEER_BUSY.  Every launch returns (the stream drains)."""
    exs = ArenaExchange.in_process(2, 4096, device, timeout_us=20_000)
    try:
        src = torch.ones(4096, dtype=torch.uint8, device=device)
        exs[0].run(src)
        torch.cuda.synchronize(device)
        assert exs[0].error() & _lib.XG_ERR_ARRIVALS
        exs[0].run(src)
        exs[0].run(src)
        torch.cuda.synchronize(device)
        assert exs[0].error() & _lib.XG_ERR_PEER_BUSY
    finally:
        close_all(exs)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.timeout(300)
@pytest.mark.parametrize("W", [2, 4])
def test_multi_process_ipc_exchange(device, tmp_path, W):
    port = _free_port()
    here = os.path.dirname(os.path.abspath(__file__))
    procs = []
    for r in range(W):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(W), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), OMP_NUM_THREADS="2")
        log = open(tmp_path / f"rank{r}.log", "w")
        procs.append((subprocess.Popen([sys.executable, "-u", os.path.join(here, "xgather_worker.py"), str(tmp_path),
                                        str(ARENA), "100"], env=env, stdout=log, stderr=subprocess.STDOUT), log))
    try:
        for p, _ in procs:
            p.wait(timeout=240)
    finally:
        for p, log in procs:
            if p.poll() is None:
                p.kill()
            log.close()
    for r, (p, _) in enumerate(procs):
        assert p.returncode == 0, (tmp_path / f"rank{r}.log").read_text()[-4000:]
    for r in range(W):
        d = json.loads((tmp_path / f"rank{r}.json").read_text())
        assert d["epochs"] == 100 and d["bad"] == [] and d["err"] == 0 and d["digest_checks"] == 10, d
