"""cProfile of bench.api_leg (the EnvStateManager.step facade on the SK workload)."""
import cProfile, os, pstats, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench

dev = torch.device("cuda", 0)
print(bench.api_leg(dev))
pr = cProfile.Profile()
pr.enable()
r = bench.api_leg(dev)
pr.disable()
print(r)
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
