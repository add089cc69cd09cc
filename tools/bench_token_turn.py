"""A/B timing of the token turn (diagnostic): on the bench's token-rollout rows (8192 6x6 envs, the
synthetic responses over the byte vocabulary), HIP-event times of 20 back-to-back launches of
  * rmi_detok_parse alone,
  * the three-launch turn: rmi_detok_parse + rmi_sokoban_step_turn + rmi_sokoban_render,
  * rmi_sokoban_token_turn (plain form),
on the library in RAGEN_AMD_LIB (variant builds of sokoban.hip: tools/build_variant.sh with
-DRMI_TOK_NO_TURN / -DRMI_TOK_NO_RENDER).  has_input is all ones and the action cap 255, so every
env steps in every launch.  Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from ragen_amd import ops  # noqa: E402
from test_gpu_fused_render import _pair  # noqa: E402
from test_gpu_token_turn import _tokens  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    torch.cuda._sleep(2_000_000)
    e[0].record()
    for _ in range(reps):
        fn()
    e[1].record()
    torch.cuda.synchronize()
    return e[0].elapsed_time(e[1]) * 1e3 / reps


def main():
    dev = torch.device("cuda", 0)
    B = 8192
    (a, b), _ = _pair(dev, B, 6, 6, 1, seed=5)
    cfg, vt, toks, stride = _tokens(dev, B, 1, 5, 9)
    lk = a.config.grid_lookup
    has = torch.ones(B, dtype=torch.uint8, device=dev)
    oa = ops.detok_parse(toks[0], vt, stride, cfg)
    tok = ops.token_rows_struct(toks[0], vt, cfg, oa)
    ts = ops.turn_struct(1, oa["actions"], oa["n_actions"], has, 255, -0.1)
    obs = ops.render_buffers(B, 6, 6, dev)
    r = ops.render_struct(lk, 6, 6, *obs)
    out = {"lib": os.path.basename(os.environ.get("RAGEN_AMD_LIB", "libragen_amd.so")), "B": B, "stride": stride}
    out["detok_parse_us"] = timed(lambda: ops.detok_parse(toks[0], vt, stride, cfg, out=oa))

    def three():
        ops.detok_parse(toks[0], vt, stride, cfg, out=oa)
        ops.sokoban_step_turn(b.struct(), b.ep, ts)
        ops.sokoban_render(b.struct(), B, lk, dev, out=obs)
    out["three_launches_us"] = timed(three)
    out["token_turn_us"] = timed(lambda: ops.sokoban_token_turn(tok, a.struct(), a.ep, ts, r))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
