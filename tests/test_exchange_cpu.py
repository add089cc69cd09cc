"""The one-shot exchange's host side on the CPU (no GPU): the layout plan every rank computes on
its own, and the handle exchange over a gloo world-2 process group (random 64-B stand-ins for
HIP IPC handles: the same all-gather carries the real ones on the GPU box)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ragen_amd import exchange


def test_plan_layout():
    p = exchange.plan(8, 499712)
    assert p["row_bytes"] == 499712 and p["blocks_per_peer"] == 61 and p["grid"] == 8 * 61 + 1
    assert p["region_bytes"] == 4096 + 2 * 8 * 499712
    assert p["slot_offsets"] == [4096 + 8 * 499712, 4096]  # epoch 1 -> slot 1, epoch 2 -> slot 0
    assert exchange.slot_offset(8, 499712, 3) == exchange.slot_offset(8, 499712, 1)
    q = exchange.plan(3, 4096 + 48)
    assert q["row_bytes"] == 8192 and q["region_bytes"] == 4096 + 2 * 3 * 8192 and q["blocks_per_peer"] == 1
    assert exchange.plan(16, 1 << 30)["blocks_per_peer"] == 256
    for bad in ((0, 16), (17, 16), (2, 0)):
        with pytest.raises(ValueError):
            exchange.region_bytes(*bad)
    with pytest.raises(ValueError):
        exchange.slot_offset(2, 16, 0)
    assert exchange.exchange_handles(bytes(range(64))) == [bytes(range(64))]  # no process group
    with pytest.raises(ValueError):
        exchange.exchange_handles(b"short")


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(100 + rank)
        mine = bytes(torch.randint(0, 256, (64,), dtype=torch.uint8, generator=g).tolist())
        got = exchange.exchange_handles(mine)
        # every rank's plan is computed locally and must agree without communication
        plans = [None] * world
        dist.all_gather_object(plans, exchange.plan(world, 499712))
        q.put((rank, mine, got, all(p == plans[0] for p in plans)))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_handle_exchange_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, port = 2, _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    handles = [m for _, m, _, _ in res]
    for rank, mine, got, same_plan in res:
        assert got == handles and got[rank] == mine and same_plan
