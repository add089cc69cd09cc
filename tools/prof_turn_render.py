"""Diagnostic: the fused turn + render against the turn alone and the separate render (bench
workload: 8192 Sokoban 6x6 envs, the first-turn form, which restores the rooms each launch so
every launch steps the same envs).  HIP events around 200 back-to-back launches each, graph
replayed and eager."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from ragen_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
R = bench.Rollout(dev, 0)
R.step()
e = R.env
ts = ops.turn_struct(0, R.ids[0], R.n[0], None, bench.MAX_ACTIONS, -0.1)
obs = ops.render_buffers(R.B, 6, 6, dev)
ro = ops.render_struct(e.config.grid_lookup, 6, 6, *obs)
variants = {
    "first": lambda: ops.sokoban_step_turn_first(R.st, e.ep, ts, e.init_state, e.init_player),
    "first+render(fused)": lambda: ops.sokoban_step_turn_render(R.st, e.ep, ts, ro, init_state=e.init_state,
                                                                init_player=e.init_player),
    "render": lambda: ops.sokoban_render(R.st, R.B, e.config.grid_lookup, dev, out=obs),
    "first;render": lambda: (ops.sokoban_step_turn_first(R.st, e.ep, ts, e.init_state, e.init_player),
                             ops.sokoban_render(R.st, R.B, e.config.grid_lookup, dev, out=obs)),
}
N = 200
for name, fn in variants.items():
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        for _ in range(20):
            fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(1_000_000)
    a.record()
    for _ in range(N // 20):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    gus = a.elapsed_time(b) * 1e3 / N
    torch.cuda._sleep(1_000_000)
    a.record()
    for _ in range(N):
        fn()
    b.record()
    torch.cuda.synchronize()
    print(f"{name:24s} graph {gus:7.2f} us/launch-set   eager {a.elapsed_time(b) * 1e3 / N:7.2f} us")
