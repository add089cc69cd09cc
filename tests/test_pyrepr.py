"""ragen_amd/csrc/pyrepr.hpp (the device's str(float) for the prompt's reward text,
ctx_manager.py:260-262) compiled for the host and compared with CPython's repr on sums of the
envs' rewards, random doubles over the supported range (1e-5 <= |x| < 2^53), powers of ten and
their neighbours, and halfway / boundary cases; values outside the range must return -1."""
import math
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    d = tmp_path_factory.mktemp("pyrepr")
    exe = str(d / "pyrepr")
    subprocess.run(["g++", "-O2", "-std=c++17", os.path.join(ROOT, "tests", "native", "pyrepr_driver.cpp"), "-o", exe],
                   check=True)
    return exe, d


def _values():
    rng = np.random.default_rng(0)
    v = []
    # RAGEN rewards: sums of -0.1 / 0.1 / 1 / -1 / 10 / 0.25 steps (es_manager.py:116-128)
    steps = [-0.1, 0.1, 1.0, -1.0, 10.0, 0.25, 0.5, -0.5, 0.3]
    for _ in range(20000):
        acc = 0
        for s in rng.choice(steps, size=int(rng.integers(1, 12))):
            acc += float(s)
        v.append(acc)
    mant = rng.random(200000) * 9 + 1
    ex = rng.integers(-5, 16, size=200000)
    v += list(mant * 10.0 ** ex)
    v += list(rng.random(50000) * 2 ** 53)
    v += list(np.frombuffer(rng.integers(0, 2 ** 63, size=100000, dtype=np.int64).tobytes(), np.float64))
    for k in range(-5, 17):
        p = 10.0 ** k
        v += [p, math.nextafter(p, 0), math.nextafter(p, math.inf), p * 5, p * 9.5, p * 0.5]
    for k in range(-16, 53):
        p = 2.0 ** k
        v += [p, math.nextafter(p, 0), math.nextafter(p, math.inf), p * 1.5]
    v += [0.0, -0.0, math.inf, -math.inf, math.nan, 1e-5, 9.999999999999999e-06, 2.0 ** 53, 2.0 ** 53 - 1, 1e16,
          123456789012345.6, 0.1 + 0.2, 1 / 3, 2 / 3, 5e-324, 1.7976931348623157e308]
    v = np.asarray(v, np.float64)
    return np.concatenate([v, -v])


def test_py_float_repr_matches_cpython(driver):
    exe, d = driver
    xs = _values()
    inp, out = str(d / "x.bin"), str(d / "x.txt")
    xs.tofile(inp)
    subprocess.run([exe, inp, out], check=True, timeout=300)
    got = open(out).read().split("\n")[:-1]
    assert len(got) == len(xs)
    n_checked = 0
    for x, g in zip(xs.tolist(), got):
        ax = abs(x)
        supported = x == 0 or math.isnan(x) or math.isinf(x) or (1e-5 <= ax < 2.0 ** 53)
        if not supported:
            assert g == "?", (x, g)
            continue
        assert g == repr(x), (x, g, repr(x))
        n_checked += 1
    assert n_checked > 500000
