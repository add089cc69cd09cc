"""ragen_amd/csrc/bigint.hpp (the Countdown evaluator's bounded Python ints, countdown/env.py:
16-21 evaluates answers with unbounded ints) compiled for the host and checked against Python's
own int arithmetic: + - * // % ** << >> & | ^, float(int) and int / int (correctly rounded,
subnormal results, OverflowError), decimal literals.  Results past 1024 bits of magnitude must
report RANGE (the evaluator flags those answers RMI_ERR_UNSUP)."""
import os
import random
import shutil
import struct
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BOUND = 1 << 1024


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    d = tmp_path_factory.mktemp("bigint")
    exe = str(d / "bigint")
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Werror", os.path.join(ROOT, "tests", "native",
                                                                                   "bigint_driver.cpp"), "-o", exe],
                   check=True)
    return exe, d


def _hex(v):
    return ("-" if v < 0 else "") + format(abs(v), "x")


def _values(rng, n):
    out = [0, 1, -1, 2, -2, 3, (1 << 32) - 1, 1 << 32, (1 << 63) - 1, -(1 << 63), 1 << 63, (1 << 64) - 1, 1 << 64,
           BOUND - 1, -(BOUND - 1), (BOUND - 1) >> 1, 1 << 1023, (1 << 1023) + 1, 10 ** 300, -(10 ** 300)]
    for _ in range(n):
        bits = rng.choice([rng.randint(0, 70), rng.randint(0, 1024), rng.randint(900, 1024), rng.randint(30, 32) * 32])
        v = rng.getrandbits(bits) if bits else 0
        kind = rng.random()
        if kind < 0.1 and bits:
            v = (1 << bits) - 1
        elif kind < 0.2 and bits:
            v = 1 << (bits - 1)
        elif kind < 0.25 and bits > 2:
            v = (1 << (bits - 1)) + rng.choice([-1, 1])
        out.append(-v if rng.random() < 0.5 else v)
    return out


def _bits(x):
    return struct.unpack("<Q", struct.pack("<d", x))[0]


def _expect(op, a, b):
    try:
        if op in ("add", "sub", "mul", "fdiv", "mod", "and", "or", "xor", "pow", "shl", "shr"):
            r = {"add": lambda: a + b, "sub": lambda: a - b, "mul": lambda: a * b, "fdiv": lambda: a // b,
                 "mod": lambda: a % b, "and": lambda: a & b, "or": lambda: a | b, "xor": lambda: a ^ b,
                 "pow": lambda: a ** b, "shl": lambda: a << b, "shr": lambda: a >> b}[op]()
            return "RANGE" if abs(r) >= BOUND else _hex(r)
        if op == "divmod":
            q, r = divmod(a, b)
            return _hex(q) + " " + _hex(r)
        if op == "todbl":
            return format(_bits(float(a)), "016x")
        if op == "tdiv":
            return format(_bits(a / b), "016x")
    except ZeroDivisionError:
        return "ZERODIV"
    except OverflowError:
        return "OVERFLOW"
    raise AssertionError(op)


def _run(driver, lines):
    exe, d = driver
    inp, out = str(d / "in.txt"), str(d / "out.txt")
    with open(inp, "w") as f:
        f.write("\n".join(lines) + "\n")
    subprocess.run([exe, inp, out], check=True, timeout=300)
    return open(out).read().split("\n")[:-1]


def test_bigint_matches_python(driver):
    rng = random.Random(7)
    vals = _values(rng, 400)
    cases = []
    for op in ("add", "sub", "mul", "fdiv", "mod", "divmod", "and", "or", "xor", "tdiv"):
        for _ in range(1500):
            a, b = rng.choice(vals), rng.choice(vals)
            if op == "mul" and rng.random() < 0.5:  # products near the bound
                a = rng.getrandbits(rng.randint(1, 600)) * rng.choice([1, -1])
                b = rng.getrandbits(rng.randint(1, 600)) * rng.choice([1, -1])
            if op in ("fdiv", "mod", "divmod") and rng.random() < 0.3:  # exact and near-exact quotients
                b = rng.choice(vals) or 1
                a = b * rng.getrandbits(rng.randint(0, 300)) * rng.choice([1, -1]) + rng.choice([0, 0, 1, -1])
                if abs(a) >= BOUND:
                    continue
            if op == "divmod" and b == 0:
                continue
            cases.append((op, a, b))
    for _ in range(1500):
        a = rng.choice(vals)
        cases.append(("todbl", a, 0))
    # float(int) at rounding boundaries: 53 significant bits + a half and sticky bits
    for e in (0, 1, 11, 53, 500, 969, 970, 971):
        for tail in (0b100, 0b101, 0b110, 0b011, 0b111):
            m = (rng.getrandbits(52) | (1 << 52)) << 3 | tail
            if (m << e) < BOUND:
                cases.append(("todbl", m << e, 0))
                cases.append(("todbl", -(m << e), 0))
    cases.append(("todbl", BOUND - 1, 0))                      # rounds to 2^1024: OverflowError
    cases.append(("todbl", BOUND - (1 << 970), 0))              # the largest finite double
    cases.append(("todbl", BOUND - (1 << 970) - 1, 0))
    # true division: subnormal and overflowing quotients, halfway cases
    for _ in range(1500):
        kind = rng.random()
        if kind < 0.3:
            a = rng.getrandbits(rng.randint(1, 60)) + 1
            b = rng.getrandbits(rng.randint(1000, 1024)) | 1
        elif kind < 0.5:
            a = rng.getrandbits(rng.randint(1000, 1024)) | 1
            b = rng.getrandbits(rng.randint(1, 5)) + 1
        elif kind < 0.8:  # quotient exactly halfway between two doubles
            q = (rng.getrandbits(52) | (1 << 52)) * 2 + 1
            b = rng.getrandbits(rng.randint(1, 400)) + 1
            sh = rng.randint(0, 400)
            a = q * b << sh
            b = b << (sh + 1)
            if a >= BOUND or b >= BOUND:
                continue
        else:
            a, b = rng.choice(vals), rng.choice(vals)
        cases.append(("tdiv", a * rng.choice([1, -1]), b * rng.choice([1, -1])))
    for a, b in ((BOUND - 1, 1), (-(BOUND - 1), 1), (BOUND - 1, -1), (BOUND - (1 << 970), 1),
                 (BOUND - (1 << 970) - 1, 1), (BOUND - (1 << 969), 1), ((BOUND - 1) >> 1, 1), (BOUND - 1, 2),
                 (1, BOUND - 1), (1, (BOUND - 1) >> 50), (3, 1 << 1023), (5, 0), (0, 7), (0, -7)):
        cases.append(("tdiv", a, b))
    for _ in range(500):
        a = rng.choice(vals)
        e = rng.choice([0, 1, 2, 3, rng.randint(0, 40), rng.randint(0, 1100)])
        if abs(a) > 1 << 70 and e > 20:
            e = rng.randint(0, 20)
        cases.append(("pow", a, e))
    for a in (0, 1, -1, 2, -2, 3, -3, 99, -99):
        for e in (0, 1, 2, 63, 64, 99, 150, 646, 1023, 1024, 1025, 10 ** 6):
            cases.append(("pow", a, e))
    for _ in range(800):
        a = rng.choice(vals)
        k = rng.choice([0, 1, 31, 32, 33, 63, 64, rng.randint(0, 1100)])
        cases.append((rng.choice(["shl", "shr"]), a, k))
    lines = []
    for op, a, b in cases:
        bb = str(b) if op in ("pow", "shl", "shr") else _hex(b)
        lines.append(f"{op} {_hex(a)} {bb}")
    got = _run(driver, lines)
    assert len(got) == len(cases)
    bad = [(c, g, _expect(*c)) for c, g in zip(cases, got) if g != _expect(*c)]
    assert not bad, bad[:5]
    assert sum(1 for c in cases if _expect(*c) == "RANGE") > 50
    assert sum(1 for c in cases if c[0] == "tdiv" and _expect(*c) == "OVERFLOW") >= 3
    assert sum(1 for c in cases if c[0] == "tdiv" and _expect(*c) == "ZERODIV") >= 1


def test_bigint_decimal_literals(driver):
    rng = random.Random(3)
    lits = ["0", "7", "1_000", "9" * 19, "9223372036854775808", "1" + "0" * 308, str(BOUND - 1), str(BOUND),
            "9" * 309, "9" * 400]
    lits += [str(rng.getrandbits(rng.randint(1, 1030))) for _ in range(300)]
    got = _run(driver, [f"dec {s} 0" for s in lits])
    for s, g in zip(lits, got):
        v = int(s)
        assert g == ("RANGE" if v >= BOUND else _hex(v)), s
