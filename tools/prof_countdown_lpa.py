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
    import torch
    import bench
    r = bench.toytext_legs(torch.device("cuda", 0))["countdown"]
    print(json.dumps({"lib": os.environ.get("RAGEN_AMD_LIB"), "ms_per_rollout": r["ms_per_rollout"]}))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        build()
    elif len(sys.argv) > 1 and sys.argv[1] == "child":
        child()
    else:
        for L in LPAS:
            env = dict(os.environ, RAGEN_AMD_LIB=os.path.join(OUT, f"libragen_amd_cdlpa{L}.so"))
            subprocess.run([sys.executable, __file__, "child"], env=env, check=True)
