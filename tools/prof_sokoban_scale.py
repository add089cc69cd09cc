"""Sokoban turn kernel at scale under different lanes-per-env layouts (diagnostic).
Builds variants of libragen_amd.so into tools/_build/ (compile-time switches of sokoban.hip,
e.g. RMI_SOK_LATE_MIN, RMI_SOKOBAN_DWORD_STORES), then times 5 turn launches at B = 8192 * tile
in a child process each.
usage: python tools/prof_sokoban_scale.py [build]"""
import os, subprocess, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tools", "_build")
VARIANTS = {"default": [], "nolate": ["-DRMI_SOK_LATE_MIN=0x7fffffff"]}  # also: ["-DRMI_SOKOBAN_DWORD_STORES"]
TILES = (1, 16, 128, 512)  # 8192 .. 4 194 304 envs (the last one past the 256 MiB Infinity Cache)


def build():
    os.makedirs(OUT, exist_ok=True)
    objs_dir = os.path.join(ROOT, "ragen_amd", "_build")
    for name, flags in VARIANTS.items():
        so = os.path.join(OUT, f"libragen_amd_{name}.so")
        src = os.path.join(ROOT, "ragen_amd", "csrc", "sokoban.hip")
        obj = os.path.join(OUT, f"sokoban_{name}.o")
        subprocess.run(["/opt/rocm/bin/hipcc", "-c", "-x", "hip", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                        "-ffp-contract=off", "-fvisibility=hidden", "-I", os.path.join(ROOT, "include"), "-I",
                        os.path.join(ROOT, "ragen_amd", "csrc")] + flags + [src, "-o", obj], check=True)
        others = [os.path.join(objs_dir, f) for f in os.listdir(objs_dir) if f.endswith(".o") and not f.startswith("sokoban.")]
        subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "--offload-arch=gfx950", "-o", so, obj] + others
                       + ["-lpthread"], check=True)


def child(name):
    sys.path.insert(0, ROOT)
    from ragen_amd import _lib
    _lib.LIB_PATH = os.path.join(OUT, f"libragen_amd_{name}.so")
    import torch
    import bench
    dev = torch.device("cuda", 0)
    R = bench.Rollout(dev, 0)
    R.step()
    torch.cuda.synchronize()
    res = {}
    for tile in TILES:
        dur, B = bench.scale_leg(R, dev, tile=tile)
        n_turns = R.env.ep.n_turns.cpu().numpy()
        act = sum(int((n_turns > t).sum()) for t in range(bench.T_TURNS)) * tile
        res[B] = {"us_per_launch": dur / bench.T_TURNS * 1e6, "TBs": act * 141 / dur / 1e12}
    print(json.dumps({name: res}))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        build()
    elif len(sys.argv) > 2 and sys.argv[1] == "child":
        child(sys.argv[2])
    else:
        for name in VARIANTS:
            subprocess.run([sys.executable, __file__, "child", name], check=True)
