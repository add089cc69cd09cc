"""Countdown turn kernel under different lanes-per-answer spreads (diagnostic).

    python tools/prof_countdown_lpa.py build     # variants of libragen_amd.so, -DRMI_CD_LPA=L
    python tools/prof_countdown_lpa.py           # bench.toytext_legs' Countdown rollout per variant

Each variant runs in its own process (RAGEN_AMD_LIB points ragen_amd at the variant)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tools", "_build")
LPAS = (1, 4, 16, 64)


def build():
    os.makedirs(OUT, exist_ok=True)
    objs_dir = os.path.join(ROOT, "ragen_amd", "_build")
    src = os.path.join(ROOT, "ragen_amd", "csrc", "countdown.hip")
    for L in LPAS:
        obj = os.path.join(OUT, f"countdown_lpa{L}.o")
        subprocess.run(["/opt/rocm/bin/hipcc", "-c", "-x", "hip", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                        "-ffp-contract=off", "-fvisibility=hidden", f"-DRMI_CD_LPA={L}", "-I",
                        os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "ragen_amd", "csrc"), src, "-o", obj],
                       check=True)
        others = [os.path.join(objs_dir, f) for f in os.listdir(objs_dir) if f.endswith(".o")
                  and not f.startswith("countdown.")]
        subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "--offload-arch=gfx950", "-o",
                        os.path.join(OUT, f"libragen_amd_cdlpa{L}.so"), obj] + others + ["-lpthread"], check=True)
        os.remove(obj)


def child():
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch
    import bench
    from ragen_amd import ops, synthetic
    from ragen_amd.env import CountdownBatch
    from ragen_amd.env.configs import CountdownEnvConfig
    from ragen_amd.env.countdown import synthetic_instances
    dev = torch.device("cuda", 0)
    r = bench.toytext_legs(dev)["countdown"]
    out = {"lib": os.path.basename(os.environ.get("RAGEN_AMD_LIB", "")), "ms_per_rollout": r["ms_per_rollout"]}
    inst = synthetic_instances(1024, 7)
    for B in (1024, 4096, 16384, 65536):  # one turn, half the envs answering, back-to-back launches
        cd = CountdownBatch(CountdownEnvConfig(data=inst), B, 1, 1, dev)
        cd.reset(synthetic.env_seeds(B))
        ans = synthetic.countdown_answers([inst[int(i)] for i in cd.index], 1, p_empty=0.5)[0]
        lists = [[a] if a is not None else [] for a in ans]
        buf, lens = cd.encode_answers(lists)
        bt, lt = torch.from_numpy(buf).to(dev), torch.from_numpy(lens).to(dev)
        n = torch.from_numpy(np.array([len(x) for x in lists], np.uint8)).to(dev)
        z = torch.zeros(B, 1, dtype=torch.int8, device=dev)
        ones = torch.ones(B, dtype=torch.uint8, device=dev)
        t = ops.turn_struct(0, z, n, ones, 200, -0.1)
        st = cd.struct()
        for _ in range(3):
            ops.countdown_step_turn(st, cd.ep, t, bt, lt)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            ops.countdown_step_turn(st, cd.ep, t, bt, lt)
        e1.record()
        torch.cuda.synchronize()
        out[f"turn_us_B{B}"] = round(e0.elapsed_time(e1) * 1000 / 50, 2)
    print(json.dumps(out))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        build()
    elif len(sys.argv) > 1 and sys.argv[1] == "child":
        child()
    else:
        for L in LPAS:
            env = dict(os.environ, RAGEN_AMD_LIB=os.path.join(OUT, f"libragen_amd_cdlpa{L}.so"))
            subprocess.run([sys.executable, __file__, "child"], env=env, check=True)
