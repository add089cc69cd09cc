"""FrozenLake turn launches of the bench's toytext leg (4096 envs x 8 turns, K=5), eager,
back-to-back per turn: per-launch time from HIP events, for rocprofv3 --pmc passes
(diagnostic, not product).   python tools/prof_frozenlake.py [B]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ragen_amd import ops, synthetic  # noqa: E402
from ragen_amd.env import FrozenLakeBatch  # noqa: E402
from ragen_amd.env.configs import FrozenLakeEnvConfig  # noqa: E402

dev = torch.device("cuda", 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
T, K = 8, 5
fl = FrozenLakeBatch(FrozenLakeEnvConfig(), B, T, K, dev)
fl.reset(synthetic.env_seeds(B))
ids, n = synthetic.rollout_actions(B, T, K, 1, 4, seed=synthetic.ACTION_SEED + 1)
ids, n = torch.from_numpy(ids).to(dev), torch.from_numpy(n).to(dev)
turns = [ops.turn_struct(t, ids[t], n[t], None, 10, -0.1) for t in range(T)]
st = fl.struct()


def rollout():
    ops.frozenlake_step_turn_first(st, fl.ep, turns[0], fl.init_desc, fl.init_s, fl.init_rng)
    for t in range(1, T):
        ops.frozenlake_step_turn(st, fl.ep, turns[t])


for _ in range(3):
    rollout()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda._sleep(1_000_000)
e0.record()
for _ in range(20):
    rollout()
e1.record()
torch.cuda.synchronize()
print(f"B={B}: {e0.elapsed_time(e1) * 1000 / 20 / T:.2f} us per turn launch (eager, back-to-back)")
