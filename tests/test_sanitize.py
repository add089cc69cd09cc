"""ASan + UBSan builds of the host-side C++ / C: the Sokoban room generator
(ragen_amd/csrc/sokoban_gen.cpp, multi-threaded DFS with the 300 000-state cap) and the CPU
oracle (oracle/ragen_oracle.c), driven by tests/sanitize/san_driver.cpp over the golden
seeds — including the seeds the reference reseeds (3248, 3701) — and the generator's output
compared with the golden rooms.  Any sanitizer report aborts the driver (-fno-sanitize-recover)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from trace_util import load

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    if not (shutil.which("g++") and shutil.which("gcc")):
        pytest.skip("g++ / gcc not available")
    d = tmp_path_factory.mktemp("san")
    oobj = str(d / "ragen_oracle.o")
    subprocess.run(["gcc", "-c", "-std=c11", "-ffp-contract=off", *SAN, os.path.join(ROOT, "oracle", "ragen_oracle.c"),
                    "-o", oobj], check=True)
    exe = str(d / "san_driver")
    subprocess.run(["g++", "-std=c++17", "-pthread", *SAN, "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "sanitize", "san_driver.cpp"),
                    os.path.join(ROOT, "ragen_amd", "csrc", "sokoban_gen.cpp"), oobj, "-lm", "-o", exe], check=True)
    return exe, d


@pytest.mark.parametrize("tag,H,nb,sd", [("SimpleSokoban", 6, 1, 300), ("LargerSokoban", 8, 2, 10)])
def test_sanitized_generator_and_oracle(driver, tag, H, nb, sd):
    exe, d = driver
    g = load("sokoban_rooms")
    seeds0 = np.asarray(g[tag + "_seeds"], np.int64)
    if tag == "SimpleSokoban":
        assert {3248, 3701} <= set(seeds0.tolist())
    # the golden seeds, then the seeds the reference reseeded the failing ones with
    n0 = len(seeds0)
    reseed = np.asarray(g[tag + "_reseed"], np.int64)
    seeds = np.concatenate([seeds0, reseed])
    sf, of = str(d / f"{tag}_seeds.bin"), str(d / f"{tag}_out.bin")
    seeds.tofile(sf)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=86",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=87")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([exe, str(H), str(nb), str(sd), "4", sf, of], capture_output=True, text=True, env=env,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    n, HW = len(seeds), H * H
    out = np.fromfile(of, np.uint8)
    assert out.size == n * (2 * HW + 3)
    fixed = out[:n * HW].reshape(n, HW)
    state = out[n * HW:2 * n * HW].reshape(n, HW)
    player = out[2 * n * HW:2 * n * HW + 2 * n].view(np.int8).reshape(n, 2)
    status = out[2 * n * HW + 2 * n:]
    bad = np.nonzero(status[:n0])[0]
    if tag == "SimpleSokoban":
        assert set(seeds0[bad].tolist()) == {3248, 3701}  # the reference reseeds exactly these
    # a failed seed takes the room of its reseed (abs(hash(str(seed))) % 2**32, PYTHONHASHSEED=0)
    assert not status[n0 + bad].any()
    fa, sa, pa = fixed, state, player
    fixed, state, player = fa[:n0].copy(), sa[:n0].copy(), pa[:n0].copy()
    fixed[bad], state[bad], player[bad] = fa[n0 + bad], sa[n0 + bad], pa[n0 + bad]
    np.testing.assert_array_equal(fixed, g[tag + "_fixed"].reshape(n0, HW).astype(np.uint8))
    np.testing.assert_array_equal(state, g[tag + "_state"].reshape(n0, HW).astype(np.uint8))
    np.testing.assert_array_equal(player, g[tag + "_player"].astype(np.int8))
