"""Build the gfx950 shared library ``ragen_amd/_build/libragen_amd.so`` (in-tree).

    python -m ragen_amd.build            # incremental
    python -m ragen_amd.build --force

hipcc cross-compiles for gfx950 without a GPU.  Device sources (*.hip) are compiled with
``-ffp-contract=off`` so the f32 recurrences keep the reference's rounding (no fused
multiply-add).  Host sources (*.cpp) are compiled with g++.
"""
import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OUT = os.path.join(PKG, "_build")
LIB = os.path.join(OUT, "libragen_amd.so")
ARCH = os.environ.get("RMI_OFFLOAD_ARCH", "gfx950")


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm required to build ragen_amd)")


def _deps():
    hdrs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hpp", ".h"))]
    hdrs.append(os.path.join(ROOT, "include", "ragen_amd.h"))
    return hdrs


def _stale(obj, src, deps):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(p) > t for p in [src] + deps)


def _compile(src, obj):
    inc = ["-I", os.path.join(ROOT, "include"), "-I", CSRC]
    if src.endswith(".hip"):
        cmd = [_hipcc(), "-c", "-x", "hip", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
               "-ffp-contract=off", "-fvisibility=hidden", "-Wall", "-Wno-unused-function"] + inc + [src, "-o", obj]
    else:
        cmd = ["g++", "-c", "-O2", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-pthread", "-Wall"] + inc + [
            src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


HOSTBOOK_SRC = os.path.join(CSRC, "hostbook.c")


def hostbook_path():
    import sysconfig
    return os.path.join(OUT, "_hostbook" + sysconfig.get_config_var("EXT_SUFFIX"))


def build_hostbook(force=False, verbose=False):
    """The CPython extension of the dict facade's host bookkeeping (csrc/hostbook.c), gcc."""
    import sysconfig
    so = hostbook_path()
    if not force and os.path.exists(so) and os.path.getmtime(so) >= os.path.getmtime(HOSTBOOK_SRC):
        return so
    tmp = so + ".tmp"
    cmd = ["gcc", "-O2", "-shared", "-fPIC", "-Wall", "-I", sysconfig.get_paths()["include"], HOSTBOOK_SRC, "-o", tmp]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, so)
    if verbose:
        print("built", so)
    return so


def build(force=False, verbose=False):
    os.makedirs(OUT, exist_ok=True)
    srcs = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp")))
    deps = _deps()
    jobs = []
    objs = []
    for s in srcs:
        o = os.path.join(OUT, os.path.basename(s) + ".o")
        objs.append(o)
        if force or _stale(o, s, deps):
            jobs.append((s, o))
    if jobs:
        with cf.ThreadPoolExecutor(max_workers=min(8, len(jobs))) as ex:
            for f in [ex.submit(_compile, s, o) for s, o in jobs]:
                o = f.result()
                if verbose:
                    print("built", o)
    if force or jobs or not os.path.exists(LIB) or any(os.path.getmtime(o) > os.path.getmtime(LIB) for o in objs):
        tmp = LIB + ".tmp"
        cmd = [_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + objs + ["-lpthread"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, LIB)
        if verbose:
            print("linked", LIB)
    build_hostbook(force, verbose)
    return LIB


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args(argv)
    print(build(force=a.force, verbose=True))


if __name__ == "__main__":
    sys.exit(main())
