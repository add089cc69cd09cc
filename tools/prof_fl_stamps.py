"""Where the time of one FrozenLake turn launch goes (diagnostic, not product).  Builds
toytext.hip with RMI_STAMPS into tools/_build/libragen_amd_flst.so (tools/build_variant.sh) and
prints, over the waves of one plain turn launch of the bench's toytext leg (4096 envs, K=5),
the mean cycles of each phase: loads landed | map bitboards | the turn (draws + steps) |
outputs, and the wave span in s_memrealtime (100 MHz) ticks.
    python tools/prof_fl_stamps.py [build]"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "tools", "_build", "libragen_amd_flst.so")
if len(sys.argv) > 1 and sys.argv[1] == "build":
    subprocess.run([os.path.join(ROOT, "tools", "build_variant.sh"), "flst", "toytext.hip", "-DRMI_STAMPS"],
                   check=True)
    sys.exit(0)
os.environ["RAGEN_AMD_LIB"] = SO
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from ragen_amd import ops, synthetic, _lib  # noqa: E402
from ragen_amd.env import FrozenLakeBatch  # noqa: E402
from ragen_amd.env.configs import FrozenLakeEnvConfig  # noqa: E402

dev = torch.device("cuda", 0)
B, T, K = 4096, 8, 5
fl = FrozenLakeBatch(FrozenLakeEnvConfig(), B, T, K, dev)
fl.reset(synthetic.env_seeds(B))
ids, n = synthetic.rollout_actions(B, T, K, 1, 4, seed=synthetic.ACTION_SEED + 1)
ids, n = torch.from_numpy(ids).to(dev), torch.from_numpy(n).to(dev)
turns = [ops.turn_struct(t, ids[t], n[t], None, 10, -0.1) for t in range(T)]
st = fl.struct()
waves = (4 * B + 63) // 64  # four lanes per env
stamps = torch.zeros(waves, 16, dtype=torch.int64, device=dev)
lib = ctypes.CDLL(SO)
assert lib.rmi_toytext_set_stamps(ctypes.c_void_p(stamps.data_ptr())) == 0
for rep in range(3):
    ops.frozenlake_step_turn_first(st, fl.ep, turns[0], fl.init_desc, fl.init_s, fl.init_rng)
    for t in range(1, 4):
        ops.frozenlake_step_turn(st, fl.ep, turns[t])
    torch.cuda.synchronize()
a = stamps.cpu().numpy().astype(np.float64)
ok = np.all(np.diff(a[:, 0:10:2], axis=1) >= 0, axis=1)  # waves that took the 4x4 path (stamps 2, 3 set)
a = a[ok]
ph = [a[:, 2 * (i + 1)] - a[:, 2 * i] for i in range(4)]
names = ["loads landed", "bitboards", "turn", "outputs"]
print(f"B={B}, plain turn 3, {int(ok.sum())} of {waves} waves: mean cycles " +
      "  ".join(f"{nm} {p.mean():.0f}" for nm, p in zip(names, ph)) +
      f"  | span {(a[:, 8] - a[:, 0]).mean():.0f} cycles, {(a[:, 9] - a[:, 1]).mean() / 100:.2f} us realtime; "
      f"first-to-last wave start {(a[:, 1].max() - a[:, 1].min()) / 100:.2f} us, "
      f"kernel window {(a[:, 9].max() - a[:, 1].min()) / 100:.2f} us; of the turn: the {K} draws "
      f"{(a[:, 11] - a[:, 4]).mean():.0f} cycles (incl. the exec list)")
