"""Where the time of one Sokoban turn launch goes, at the bench's SK workload (diagnostic, not
product).  Builds sokoban.hip with RMI_STAMPS into tools/_build/libragen_amd_skst.so
(tools/build_variant.sh), runs the bench rollout's first three launches eagerly and prints,
over the waves of the third (a plain turn), the mean cycles of each phase (loads landed |
decode + regular test | the turn | outputs issued), the mean wave span and, in s_memrealtime
(100 MHz) time, how far apart the waves started and the window from the first start to the last
end.   python tools/prof_sokoban_stamps.py [build]"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.environ.get("PROBE_SO") or os.path.join(ROOT, "tools", "_build", "libragen_amd_skst.so")
if len(sys.argv) > 1 and sys.argv[1] == "build":
    subprocess.run([os.path.join(ROOT, "tools", "build_variant.sh"), "skst", "sokoban.hip", "-DRMI_STAMPS"],
                   check=True)
    sys.exit(0)
os.environ["RAGEN_AMD_LIB"] = SO
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from ragen_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
R = bench.Rollout(dev, 0)
B = R.env.ep.flags.shape[0]
waves = (B + 63) // 64
stamps = torch.zeros(waves, 16, dtype=torch.int64, device=dev)
assert ctypes.CDLL(SO).rmi_sokoban_set_stamps(ctypes.c_void_p(stamps.data_ptr())) == 0
e = R.env
# "noboards": every turn decodes its rows (the form before the board cache)
st0, stn = (R.st, R.st) if "noboards" in sys.argv else (R.st_first, R.st_next)
for rep in range(5):
    ops.sokoban_step_turn_first(st0, e.ep, R.turns[0], e.init_state, e.init_player)
    for t in range(1, 3):
        ops.sokoban_step_turn(stn, e.ep, R.turns[t])
    torch.cuda.synchronize()
a = stamps.cpu().numpy().astype(np.float64)
ph = [a[:, 2 * (i + 1)] - a[:, 2 * i] for i in range(4)]
names = ["loads landed", "decode + test", "turn", "outputs"]
print(f"B={B}, turn 2 (plain), {waves} waves: mean cycles " +
      "  ".join(f"{nm} {p.mean():.0f}" for nm, p in zip(names, ph)) +
      f"  | span {(a[:, 8] - a[:, 0]).mean():.0f} cycles, {(a[:, 9] - a[:, 1]).mean() / 100:.2f} us realtime; "
      f"first-to-last wave start {(a[:, 1].max() - a[:, 1].min()) / 100:.2f} us "
      f"(median start offset {np.median(a[:, 1] - a[:, 1].min()) / 100:.2f} us), "
      f"kernel window {(a[:, 9].max() - a[:, 1].min()) / 100:.2f} us")
