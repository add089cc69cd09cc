"""Where one Countdown turn launch spends its time (diagnostic, not product).  Builds
countdown.hip with RMI_CD_STAMPS into tools/_build/libragen_amd_cdstamps.so (the other objects
from ragen_amd/_build) and prints, over the waves whose first row evaluated an answer, the mean
cycles from kernel entry to: loads landed, answer staged, reward computed, turn done, stores
issued.  Workload: 16384 envs, one turn, the bench's answer mix (half the envs answer)."""
import ctypes, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tools", "_build")
SO = os.path.join(OUT, "libragen_amd_cdstamps.so")
SRC = os.path.join(ROOT, "ragen_amd", "csrc", "countdown.hip")


def build():
    os.makedirs(OUT, exist_ok=True)
    obj = os.path.join(OUT, "countdown_stamps.o")
    subprocess.run(["/opt/rocm/bin/hipcc", "-c", "-x", "hip", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                    "-ffp-contract=off", "-fvisibility=hidden", "-DRMI_CD_STAMPS", "-I", os.path.join(ROOT, "include"),
                    "-I", os.path.join(ROOT, "ragen_amd", "csrc"), SRC, "-o", obj], check=True)
    objs = os.path.join(ROOT, "ragen_amd", "_build")
    others = [os.path.join(objs, f) for f in os.listdir(objs) if f.endswith(".o") and not f.startswith("countdown.")]
    subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "--offload-arch=gfx950", "-o", SO, obj] + others +
                   ["-lpthread"], check=True)
    os.remove(obj)


if len(sys.argv) > 1 and sys.argv[1] == "build":
    build()
    sys.exit(0)
os.environ["RAGEN_AMD_LIB"] = SO
import numpy as np  # noqa: E402
import torch  # noqa: E402
from ragen_amd import ops, synthetic, _lib  # noqa: E402
from ragen_amd.env import CountdownBatch  # noqa: E402
from ragen_amd.env.configs import CountdownEnvConfig  # noqa: E402
from ragen_amd.env.countdown import synthetic_instances  # noqa: E402

dev = torch.device("cuda", 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
p_empty = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
inst = synthetic_instances(1024, 7)
cd = CountdownBatch(CountdownEnvConfig(data=inst), B, 1, 1, dev)
cd.reset(synthetic.env_seeds(B))
ans = synthetic.countdown_answers([inst[int(i)] for i in cd.index], 1, p_empty=p_empty)[0]
lists = [[a] if a is not None else [] for a in ans]
buf, lens = cd.encode_answers(lists)
bt, lt = torch.from_numpy(buf).to(dev), torch.from_numpy(lens).to(dev)
n = torch.from_numpy(np.array([len(x) for x in lists], np.uint8)).to(dev)
z = torch.zeros(B, 1, dtype=torch.int8, device=dev)
ones = torch.ones(B, dtype=torch.uint8, device=dev)
t = ops.turn_struct(0, z, n, ones, 200, -0.1)
waves = (B * 16 + 63) // 64
st = torch.zeros(waves, 6, dtype=torch.int64, device=dev)
pst = torch.zeros(waves, 8, dtype=torch.int64, device=dev)
L = _lib.lib()
L.rmi_countdown_set_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
assert L.rmi_countdown_set_stamps(ctypes.c_void_p(st.data_ptr()), ctypes.c_void_p(pst.data_ptr())) == 0
s = cd.struct()
for _ in range(5):
    ops.countdown_step_turn(s, cd.ep, t, bt, lt)
torch.cuda.synchronize()
a = st.cpu().numpy().astype(np.float64)
ev = a[:, 2] != a[:, 1]
d = a - a[:, :1]
names = ["loads landed", "answer staged", "reward done", "turn done", "stores issued"]
print(f"B={B} p_empty={p_empty}: {int(ev.sum())} of {waves} waves evaluated an answer in row 0")
for sel, lab in ((ev, "evaluating"), (~ev, "no answer in row 0")):
    if sel.any():
        print(lab, "mean cycles from entry:", {nm: round(float(d[sel, i + 1].mean())) for i, nm in enumerate(names)},
              "max stores issued:", round(float(d[sel, 5].max())))
pa = pst.cpu().numpy().astype(np.float64)
ok = ev & (pa[:, 6] > 0)
pn = ["mask bytes read", "token parsed", "syntax ballots", "format", "tree", "evaluated", "result"]
if ok.any():
    base = a[ok, 2]
    print("par_reward phases, mean cycles after 'answer staged':",
          {nm: round(float((pa[ok, i] - base).mean())) for i, nm in enumerate(pn)})
