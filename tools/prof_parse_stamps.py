"""Where the time of one rmi_parse_actions launch goes (diagnostic, not product).
Builds parse.hip with RMI_PARSE_STAMPS into tools/_build/libparse_stamps.so (s_memtime per
phase per wave) and prints the mean cycles of each phase at a few batch shapes.
  0 entry | 1 text staged | 2 '<' events classified | 3 regex match | 4 cascade/strip |
  5 split + names | 6 stores; inside the split: 7 separator candidates collected, 8 separators
  selected"""
import ctypes, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch
from ragen_amd import ops, synthetic

OUT = os.path.join(ROOT, "tools", "_build")
SO = os.path.join(OUT, "libparse_stamps.so")
if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(os.path.join(ROOT, "ragen_amd", "csrc", "parse.hip")):
    os.makedirs(OUT, exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "-x", "hip", "--offload-arch=gfx950", "-O3",
                    "-std=c++17", "-ffp-contract=off", "-DRMI_PARSE_STAMPS", "-I", os.path.join(ROOT, "include"),
                    "-I", os.path.join(ROOT, "ragen_amd", "csrc"), os.path.join(ROOT, "ragen_amd", "csrc", "parse.hip"),
                    "-o", SO], check=True)
if len(sys.argv) > 1 and sys.argv[1] == "build":
    sys.exit(0)
L = ctypes.CDLL(SO)
from ragen_amd import _lib
f = L.rmi_parse_actions
f.restype = ctypes.c_int32
f.argtypes = _lib._SIGS["rmi_parse_actions"][1]
dev = torch.device("cuda", 0)
lk = {1: "Up", 2: "Down", 3: "Left", 4: "Right"}
names = ["stage", "events", "match", "strip", "split", "stores"]
for B, tw, think in ((1024, (8, 60), True), (8192, (8, 60), True), (8192, (0, 2), True), (8192, (200, 300), True),
                     (1024, (0, 2), False)):
    ids, n = synthetic.rollout_actions(B, 1, 5, 1, 4)
    texts = synthetic.responses_for_actions(ids[0], n[0], lk, think_words=tw)
    buf, lens = synthetic.encode_rows(texts)
    text, tl = torch.from_numpy(buf).to(dev), torch.from_numpy(lens).to(dev)
    st = torch.zeros(B, 12, dtype=torch.int64, device=dev)
    L.rmi_parse_set_stamps(ctypes.c_void_p(st.data_ptr()))
    cfg = ops.parse_config(think, 5, "||", lk)
    o = ops.parse_actions(cfg, text, tl)
    for _ in range(3):
        rc = f(ctypes.byref(cfg), text.data_ptr(), tl.data_ptr(), B, buf.shape[1], None, o["actions"].data_ptr(),
               o["n_actions"].data_ptr(), o["spans"].data_ptr(), None, None, 0, o["err"].data_ptr(),
               torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    s = st.cpu().numpy().astype(np.float64)
    d = np.diff(s[:, :7], axis=1)
    span = s[:, 6].max() - s[:, 0].min()
    print(f"B={B} words={tw} think={think}: wave span mean {np.mean(s[:, 6] - s[:, 0]):.0f} cyc, "
          f"grid span {span:.0f} cyc ({span / 2.4e3:.1f} us @2.4GHz)")
    print("   " + "  ".join(f"{nm}={d[:, i].mean():.0f}" for i, nm in enumerate(names)))
    sp = s[:, 7] > 0  # rows with a match: the split's separator collect / greedy selection / pieces
    if sp.any():
        print(f"   split: collect={np.mean(s[sp, 7] - s[sp, 4]):.0f}  select={np.mean(s[sp, 8] - s[sp, 7]):.0f}  "
              f"pieces={np.mean(s[sp, 5] - s[sp, 8]):.0f}")
