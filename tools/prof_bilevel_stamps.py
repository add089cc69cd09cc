"""Where the time of one rmi_bilevel_gae launch goes (diagnostic, not product).  Builds
advantage.hip with RMI_BL_STAMPS into tools/_build/libbilevel_stamps.so and prints each
wave's mean cycles in P1 (incl. the tile load wait), the P2+P3 walk and P4, summed over its
tiles, for the bench's bi-level rows (8192 rows, turn rewards at each turn's end).
The segment-parallel kernel (the default at these row lengths) stamps its tile loop (P1+P2),
the segment walks (P3) and the outputs (P4) instead; RAGEN_AMD_BILEVEL_TILED=1 selects the
tiled kernel's stamps."""
import ctypes, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch
from ragen_amd import synthetic, _lib

OUT = os.path.join(ROOT, "tools", "_build")
SO = os.path.join(OUT, "libbilevel_stamps.so")
SRC = os.path.join(ROOT, "ragen_amd", "csrc", "advantage.hip")
if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(SRC):
    os.makedirs(OUT, exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "-x", "hip", "--offload-arch=gfx950", "-O3",
                    "-std=c++17", "-ffp-contract=off", "-DRMI_BL_STAMPS", "-I", os.path.join(ROOT, "include"),
                    "-I", os.path.join(ROOT, "ragen_amd", "csrc"), SRC, "-o", SO], check=True)
if len(sys.argv) > 1 and sys.argv[1] == "build":
    sys.exit(0)
L = ctypes.CDLL(SO)
f = L.rmi_bilevel_gae
f.restype = ctypes.c_int32
f.argtypes = _lib._SIGS["rmi_bilevel_gae"][1]
dev = torch.device("cuda", 0)
rng = np.random.default_rng(3)
B = 8192
n_turns = rng.integers(1, 6, B).astype(np.int32)
score = rng.standard_normal(B).astype(np.float32)
tr = (rng.random((B, 5)) < 0.7).astype(np.float32) * 0.5 + 0.5
r, v, m = synthetic.token_rows(n_turns, score, seed=12, turn_scores=tr)
r, v, m = (torch.from_numpy(x).to(dev) for x in (r, v, m))
Bn, Ln = r.shape
adv = torch.empty_like(r)
ret = torch.empty_like(r)
err = torch.zeros(Bn, dtype=torch.uint8, device=dev)
waves = (Bn + 3) // 4
st = torch.zeros(waves, 4, dtype=torch.int64, device=dev)
L.rmi_bilevel_set_stamps(ctypes.c_void_p(st.data_ptr()))
s = torch.cuda.current_stream().cuda_stream
for _ in range(3):
    rc = f(r.data_ptr(), v.data_ptr(), m.data_ptr(), Bn, Ln, 1.0, 0.95, 0.95, adv.data_ptr(), ret.data_ptr(), None,
           err.data_ptr(), s)
    assert rc == 0
torch.cuda.synchronize()
a = st.cpu().numpy().astype(np.float64)
ntiles = (Ln + 63) // 64
print(f"B={Bn} L={Ln} tiles/wave={ntiles}: per wave mean cycles P1 {a[:,0].mean():.0f}  walk {a[:,1].mean():.0f}  "
      f"P4 {a[:,2].mean():.0f}  total {a[:,3].mean():.0f}  (per tile: {a[:,0].mean()/ntiles:.0f} / "
      f"{a[:,1].mean()/ntiles:.0f} / {a[:,2].mean()/ntiles:.0f})")
