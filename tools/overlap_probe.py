"""Probe: how to overlap the per-rollout episode-arena exchange with the next rollouts.

Times bench.py's Rollout, G rollouts per graph replay (their G arenas contiguous, gathered by
ONE collective), with the exchange placed in different ways:
  roll        rollouts only (no exchange)
  serial      one single-stream graph: G rollouts, then the gather
  fork        one graph, the gather of the previous set on a forked stream (multi-stream capture)
  ev_only     rollouts graph + the cross-stream event pair, no gather (cost of the ordering)
  ev_graph    rollouts graph on the main stream, gather graph on a comm stream, events between
  ev_eager    as ev_graph with the gather launched eagerly on the comm stream
The gather is a spin kernel of --gather-us per set (an RCCL all-gather is latency-bound the
same way; spins occupy one CU), or with --rccl the real all-gather in a 1-rank RCCL group.

  python tools/overlap_probe.py [--group 8] [--gather-us 120] [--rccl]
"""
import argparse
import os
import sys
import time

import torch
import torch.distributed as tdist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from ragen_amd import distributed as rd  # noqa: E402
from ragen_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--group", type=int, default=8)
    ap.add_argument("--gather-us", type=float, default=120.0)
    ap.add_argument("--rccl", action="store_true")
    ap.add_argument("--steps", type=int, default=400)
    args = ap.parse_args()
    G = args.group
    device = torch.device("cuda", 0)
    torch.cuda.set_device(device)
    if args.rccl:
        for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29519"), ("RANK", "0"), ("WORLD_SIZE", "1")):
            os.environ.setdefault(k, v)
        tdist.init_process_group("nccl", device_id=device)
    R = bench.Rollout(device, 0)
    pool, eps = ops.EpisodeState.pool(2 * G, R.env.B, R.env.T, device)
    sets = pool.view(2, -1)
    outs = [torch.empty_like(sets[h]) for h in (0, 1)]
    cycles = int(args.gather_us * 2400)  # spin kernel: ~2.4 GHz shader clock

    def gather(h):
        if args.rccl:
            rd.gather_bytes(sets[h], outs[h])
        else:
            torch.cuda._sleep(cycles)

    main_s = torch.cuda.current_stream(device)
    comm, cap_s = torch.cuda.Stream(device), torch.cuda.Stream(device)

    def rollouts(h):
        for j in range(G):
            R.env.ep = eps[h * G + j]
            R.step()

    for h in (0, 1):  # eager warm-up (communicator setup outside capture)
        rollouts(h)
        with torch.cuda.stream(comm):
            gather(h)
    torch.cuda.synchronize()

    def capture(fn, stream=None):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            fn()
        return g

    roll_g = [capture(lambda h=h: rollouts(h)) for h in (0, 1)]
    serial_g = [capture(lambda h=h: (rollouts(h), gather(h))) for h in (0, 1)]

    def fork_body(h):
        cur = torch.cuda.current_stream(device)
        comm.wait_stream(cur)
        with torch.cuda.stream(comm):
            gather(1 - h)
        rollouts(h)
        cur.wait_stream(comm)

    fork_g = [capture(lambda h=h: fork_body(h)) for h in (0, 1)]
    gather_g = [capture(lambda h=h: gather(h), stream=cap_s) for h in (0, 1)]
    rolled = [torch.cuda.Event(), torch.cuda.Event()]
    gathered = [torch.cuda.Event(), torch.cuda.Event()]

    def alt(gs):
        n = [0]

        def run():
            gs[n[0] & 1].replay()
            n[0] += 1
        return run

    def events(mode):
        n = [0]

        def run():
            h = n[0] & 1
            if n[0] >= 2:
                main_s.wait_event(gathered[h])
            roll_g[h].replay()
            rolled[h].record(main_s)
            torch.cuda.set_stream(comm)
            comm.wait_event(rolled[h])
            if mode == "graph":
                gather_g[h].replay()
            elif mode == "eager":
                gather(h)
            gathered[h].record(comm)
            torch.cuda.set_stream(main_s)
            n[0] += 1
        return run

    variants = {"roll": alt(roll_g), "serial": alt(serial_g), "fork": alt(fork_g),
                "ev_only": events("none"), "ev_graph": events("graph"), "ev_eager": events("eager")}
    reps = max(2, args.steps // G)
    for name, run in variants.items():
        for _ in range(6):
            run()
        torch.cuda.synchronize()
        # host enqueue cost alone: queued behind a long spin kernel, so the GPU never waits on it
        torch.cuda._sleep(200_000_000)
        h0 = time.perf_counter()
        for _ in range(20):
            run()
        host_us = (time.perf_counter() - h0) / (20 * G) * 1e6
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            run()
        torch.cuda.synchronize()
        wall_us = (time.perf_counter() - t0) / (reps * G) * 1e6
        print(f"{name:10s} G={G} host-enqueue {host_us:7.1f} us/rollout   wall {wall_us:7.1f} us/rollout", flush=True)
    if args.rccl:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
