"""Phase stamps of rmi_sokoban_token_turn (diagnostic): run with RAGEN_AMD_LIB pointing at a build of
sokoban.hip with -DRMI_TOK_STAMPS (tools/build_variant.sh tokstamps sokoban.hip -DRMI_TOK_STAMPS).
On the bench's token-rollout rows (tools/bench_token_turn.py's setup, plain turn form) it prints,
per wave (cycles): decode + parse, the wait at the first barrier, the turn (turn waves), the wait
at the second barrier, the render; per workgroup the slowest parse against the group's end; and
the grid span from the waves' s_memrealtime (100 MHz)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from ragen_amd import _lib, ops  # noqa: E402
from test_gpu_fused_render import _pair  # noqa: E402
from test_gpu_token_turn import _tokens  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    B = 8192
    (a, _), _ = _pair(dev, B, 6, 6, 1, seed=5)
    cfg, vt, toks, stride = _tokens(dev, B, 1, 5, 9)
    has = torch.ones(B, dtype=torch.uint8, device=dev)
    oa = ops.detok_parse(toks[0], vt, stride, cfg)
    tok = ops.token_rows_struct(toks[0], vt, cfg, oa)
    ts = ops.turn_struct(1, oa["actions"], oa["n_actions"], has, 255, -0.1)
    obs = ops.render_buffers(B, 6, 6, dev)
    r = ops.render_struct(a.config.grid_lookup, 6, 6, *obs)
    st = torch.zeros(B, 8, dtype=torch.int64, device=dev)
    L = _lib.lib()
    f = getattr(L, "rmi_tok_set_stamps")
    f.argtypes = [ctypes.c_void_p]
    f(ctypes.c_void_p(st.data_ptr()))  # before any launch: the stamps build writes through it
    for _ in range(4):
        ops.sokoban_token_turn(tok, a.struct(), a.ep, ts, r)
    torch.cuda.synchronize()
    s = st.cpu().numpy().astype(np.float64)
    parse = s[:, 2] - s[:, 1]
    wait_a = s[:, 3] - s[:, 2]
    turn = s[:, 4] - s[:, 3]
    wait_b = s[:, 5] - s[:, 4]
    render = s[:, 6] - s[:, 5]
    wv = np.arange(B) % 16
    tw = wv < 4
    print(f"per wave (cycles, mean / p90): parse {parse.mean():.0f} / {np.percentile(parse, 90):.0f} | "
          f"wait A {wait_a.mean():.0f} | turn (turn waves) {turn[tw].mean():.0f} / {np.percentile(turn[tw], 90):.0f} | "
          f"wait B (other waves) {wait_b[~tw].mean():.0f} (turn waves {wait_b[tw].mean():.0f}) | render {render.mean():.0f} / "
          f"{np.percentile(render, 90):.0f}")
    tl = oa["text_len"].cpu().numpy()
    for lo, hi in ((0, 128), (128, 192), (192, 256), (256, 320), (320, 4096)):
        m = (tl >= lo) & (tl < hi)
        if m.any():
            print(f"  text {lo}-{hi} B: {m.sum()} rows, parse mean {parse[m].mean():.0f} p90 {np.percentile(parse[m], 90):.0f}")
    g = s.reshape(-1, 16, 8)
    t_parse_max = (g[:, :, 2] - g[:, :, 1].min(1, keepdims=True)).max(1)
    t_end = (g[:, :, 6] - g[:, :, 1].min(1, keepdims=True)).max(1)
    print(f"per workgroup (cycles from its first wave's start): slowest parse end {t_parse_max.mean():.0f}, "
          f"group end {t_end.mean():.0f} (tail after the parse {np.mean(t_end - t_parse_max):.0f})")
    rt0, rt1 = s[:, 0], s[:, 7]
    print(f"grid span {(rt1.max() - rt0.min()) / 100:.1f} us | wave starts p50/p90/max "
          f"{np.percentile(rt0 - rt0.min(), 50) / 100:.1f}/{np.percentile(rt0 - rt0.min(), 90) / 100:.1f}/"
          f"{(rt0.max() - rt0.min()) / 100:.1f} us | wave duration mean {((rt1 - rt0) / 100).mean():.2f} us")


if __name__ == "__main__":
    main()
