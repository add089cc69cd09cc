"""The Sokoban turn kernel at 1 048 576 envs (the bench batch tiled 128x), for PMC passes:
rocprofv3 --pmc FETCH_SIZE (then WRITE_SIZE) --kernel-trace -- python3 tools/prof_scale_pmc.py"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench

dev = torch.device("cuda", 0)
R = bench.Rollout(dev, 0)
R.step()
torch.cuda.synchronize()
for _ in range(2):
    dur, B = bench.scale_leg(R, dev, tile=128)
n_turns = R.env.ep.n_turns.cpu().numpy()
act = sum(int((n_turns > t).sum()) for t in range(bench.T_TURNS)) * 128
print({"envs": B, "us_per_launch": dur / bench.T_TURNS * 1e6, "active_env_turns": act,
       "algorithmic_bytes_per_launch": act * 141 / bench.T_TURNS})
