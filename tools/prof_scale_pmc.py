"""The Sokoban turn kernel on the bench batch tiled `tile` times (argv[1], default 512 =
4 194 304 envs, past the Infinity Cache), for PMC passes:
rocprofv3 --pmc FETCH_SIZE (then WRITE_SIZE) --kernel-trace -- python3 tools/prof_scale_pmc.py [tile]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench

dev = torch.device("cuda", 0)
R = bench.Rollout(dev, 0)
R.step()
torch.cuda.synchronize()
tile = int(sys.argv[1]) if len(sys.argv) > 1 else 512
for _ in range(2):
    dur, B = bench.scale_leg(R, dev, tile=tile)
n_turns = R.env.ep.n_turns.cpu().numpy()
act = sum(int((n_turns > t).sum()) for t in range(bench.T_TURNS)) * tile
print({"envs": B, "us_per_launch": dur / bench.T_TURNS * 1e6, "active_env_turns": act,
       "algorithmic_bytes_per_launch": act * 141 / bench.T_TURNS})
