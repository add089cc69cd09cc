"""bench.py's multi-GPU launch logic and its N>1 exchange check, on the CPU.

* launch_plan: `--gpus N` either runs as one rank of a launcher's world, spawns N ranks, or
  exits non-zero -- never a 1-GPU run labelled N;
* `python bench.py --gpus 2` on a box without 2 devices exits 2 with the reason, before any
  GPU work;
* check_gathered over a gloo world of 2: every rank's row of the gathered set is checked
  against the digest its owner all-gathered; a corrupted or duplicated row fails on every rank.
"""
import os
import socket
import subprocess
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from ragen_amd import distributed as rd  # noqa: E402


def test_launch_plan_single():
    assert bench.launch_plan(1, {}, 0) == ("run", 1)
    assert bench.launch_plan(1, {}, 8) == ("run", 1)


def test_launch_plan_spawns_without_launcher():
    assert bench.launch_plan(8, {}, 8) == ("spawn", 8)
    assert bench.launch_plan(2, {}, 8) == ("spawn", 2)


def test_launch_plan_refuses_too_few_devices():
    act, msg = bench.launch_plan(2, {}, 1)
    assert act == "error" and "1 GPU" in msg
    assert bench.launch_plan(0, {}, 1)[0] == "error"


def test_launch_plan_under_torchrun():
    env = {"WORLD_SIZE": "4", "RANK": "3", "LOCAL_RANK": "3"}
    assert bench.launch_plan(4, env, 8) == ("run", 4)
    act, msg = bench.launch_plan(8, env, 8)      # launcher world disagrees with --gpus
    assert act == "error" and "WORLD_SIZE=4" in msg
    act, msg = bench.launch_plan(4, env, 2)      # local rank without a device
    assert act == "error" and "LOCAL_RANK 3" in msg


def test_bench_gpus2_exits_cleanly_without_devices():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    env["HIP_VISIBLE_DEVICES"] = ""  # no device visible even if one existed
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--no-extras"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode == 2, p.stderr
    assert "--gpus 2" in p.stderr and p.stdout == ""


def test_arena_digests_position_sensitive():
    g = torch.Generator().manual_seed(0)
    a = torch.randint(0, 256, (3, 1001), dtype=torch.uint8, generator=g)
    d = bench.arena_digests(a)
    assert d.shape == (3,) and d.dtype == torch.int64
    b = a.clone()
    b[1, 500], b[1, 501] = a[1, 501], a[1, 500]   # swap two bytes: a plain sum would not notice
    if a[1, 500] != a[1, 501]:
        assert bench.arena_digests(b)[1] != d[1]
    assert torch.equal(bench.arena_digests(b)[[0, 2]], d[[0, 2]])


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = torch.Generator().manual_seed(10 + rank)
    own = torch.randint(0, 256, (4096 + 3,), dtype=torch.uint8, generator=g)
    out = torch.empty(world * own.numel(), dtype=torch.uint8)
    rd.gather_bytes(own, out)
    good = bench.check_gathered(own, out, world, rank)
    bad_other = out.clone()
    bad_other.view(world, -1)[1 - rank, 7] ^= 0x5A       # another rank's row corrupted
    corrupt = bench.check_gathered(own, bad_other, world, rank)
    dup = out.clone()
    dup.view(world, -1)[1 - rank] = own                   # another rank's row replaced by this rank's
    duplicated = bench.check_gathered(own, dup, world, rank)
    same = bench.check_gathered(torch.zeros(16, dtype=torch.uint8),
                                torch.zeros(world * 16, dtype=torch.uint8), world, rank)
    q.put((rank, good, corrupt, duplicated, same))
    dist.destroy_process_group()


def test_check_gathered_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, good, corrupt, duplicated, same in res:
        assert good
        assert not corrupt
        assert not duplicated
        assert not same   # identical sets on every rank: not distinct


def test_exchange_default_is_a_serial_gather_per_rollout():
    """The N>1 headline runs StarPO's order by default (agent_trainer.py:514-655): each rollout's
    record all-gathered right after it, on the critical path; amortised / overlapped placements
    only on request."""
    args = bench.make_parser().parse_args([])
    assert args.exchange == "serial" and args.rollouts_per_gather == 1
    assert bench.exchange_plan(args.exchange, args.rollouts_per_gather, 4) == ("serial", 1)
    assert bench.exchange_plan("serial", 4, 4) == ("serial", 4)
    assert bench.exchange_plan("overlap", 1, 4) == ("overlap", 4)   # overlap gathers a whole replay
    assert "every rollout" in bench.exchange_label("serial", 1, 4, "serial", True)
    assert "extra" in bench.exchange_label("overlap", 4, 4, "overlap", True)
    assert "extra" in bench.exchange_label("serial", 4, 4, "serial", True)
    for bad in ((0, 4), (3, 4)):
        try:
            bench.exchange_plan("serial", *bad)
        except ValueError:
            continue
        raise AssertionError(f"exchange_plan accepted --rollouts-per-gather {bad[0]} for G={bad[1]}")


def _serial_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    G, n = 4, 37
    arenas = torch.zeros(G * n, dtype=torch.uint8)
    order = []

    def step(j):  # rollout j writes its arena (rank- and rollout-specific bytes)
        order.append(("roll", j))
        arenas[j * n:(j + 1) * n] = torch.arange(n, dtype=torch.uint8) * (rank + 1) + 17 * j

    def gather(buf, out):
        order.append(("gather", len([o for o in order if o[0] == "gather"])))
        rd.gather_bytes(buf, out)

    res = {}
    for p in (1, G):
        order.clear()
        arenas.zero_()
        outs = [torch.empty(world * p * n, dtype=torch.uint8) for _ in range(G // p)]
        bench.serial_exchange(step, lambda q_, k: arenas[k * q_ * n:(k + 1) * q_ * n], outs, G, p, gather=gather)
        ok = all(bench.check_gathered(arenas[k * p * n:(k + 1) * p * n], outs[k], world, rank) for k in range(G // p))
        res[p] = (list(order), ok)
    q.put((rank, res))
    dist.destroy_process_group()


def test_serial_exchange_gathers_each_rollout_before_the_next_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=_serial_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, r in res:
        order1, ok1 = r[1]
        assert ok1 and order1 == [x for j in range(4) for x in (("roll", j), ("gather", j))]
        order4, ok4 = r[4]
        assert ok4 and order4 == [("roll", j) for j in range(4)] + [("gather", 0)]
