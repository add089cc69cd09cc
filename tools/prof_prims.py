"""Host-side cost of the primitives the device turn loop is built from (diagnostic): a bare
synchronize, small device->host reads (pageable .cpu(), pinned non_blocking copy + event wait),
torch elementwise launches, torch.cat, and one of this library's ops (host time per call, and
per call + synchronize)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ragen_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
N = 8192
a = torch.zeros(N, dtype=torch.uint8, device=dev)
b = torch.ones(N, dtype=torch.uint8, device=dev)
c = torch.zeros(N, dtype=torch.int32, device=dev)
pin = torch.empty(3 * N, dtype=torch.uint8).pin_memory()
ev = torch.cuda.Event()


def t(label, f, reps=200):
    for _ in range(10):
        f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    dt = (time.perf_counter() - t0) / reps
    torch.cuda.synchronize()
    print(f"{label:60s} {dt * 1e6:8.2f} us")


t("synchronize (idle)", torch.cuda.synchronize)
t("torch.cat 3 x 8192 u8 (launch)", lambda: torch.cat([a, b, a]))
t("(a == 0) u8 (launch)", lambda: a == 0)
t("zeros 8192 u8 (launch)", lambda: torch.zeros(N, dtype=torch.uint8, device=dev))
t("empty 8192 u8", lambda: torch.empty(N, dtype=torch.uint8, device=dev))
t("c.max() (launch)", lambda: c.max())
t("int(c.max())  (launch + read)", lambda: int(c.max()))
t("a.cpu() 8 KB pageable", lambda: a.cpu())
t("cat(3 x 8 KB).cpu().numpy()", lambda: torch.cat([a, b, a]).cpu().numpy())


def pinned():
    pin.view(3, N)[0].copy_(a, non_blocking=True)
    pin.view(3, N)[1].copy_(b, non_blocking=True)
    pin.view(3, N)[2].copy_(a, non_blocking=True)
    ev.record()
    ev.synchronize()


t("3 x 8 KB pinned non_blocking copies + event wait", pinned)


def pinned1():
    torch.cat([a, b, a], out=ab)
    pin.copy_(ab, non_blocking=True)
    ev.record()
    ev.synchronize()


ab = torch.empty(3 * N, dtype=torch.uint8, device=dev)
t("cat(out=) + 1 pinned copy + event wait", pinned1)
t("torch.stack([c.max(), c.max()]).cpu().tolist()", lambda: torch.stack([c.max(), c.max()]).cpu().tolist())
import numpy as np  # noqa: E402
idx = np.arange(7000, dtype=np.int64)
t("from_numpy(7000 i64).to(dev) pageable", lambda: torch.from_numpy(idx).to(dev))
t("from_numpy(7000 i64).pin_memory().to(dev, non_blocking)", lambda: torch.from_numpy(idx).pin_memory().to(dev, non_blocking=True))
t("torch.cuda.current_stream(dev).cuda_stream", lambda: torch.cuda.current_stream(dev).cuda_stream)
t("np.unique(7000)", lambda: np.unique(idx))
x = torch.randn(1 << 20, device=dev)
t("x.sum() 1M f32 (launch)", lambda: x.sum())
# a ragen_amd op: the Sokoban render of 8192 envs
from ragen_amd.env import SokobanBatch  # noqa: E402
from ragen_amd.env.configs import SokobanEnvConfig  # noqa: E402
from ragen_amd import synthetic  # noqa: E402

env = SokobanBatch(SokobanEnvConfig(dim_x=6, dim_y=6, num_boxes=1, max_steps=100), N, 5, 5, dev)
env.reset(synthetic.env_seeds(N))
torch.cuda.synchronize()
t("env.render_rows() (launch)", lambda: env.render_rows())
t("env.render_rows() + synchronize", lambda: (env.render_rows(), torch.cuda.synchronize()))
print("done")
