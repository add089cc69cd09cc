"""Countdown rewards with Python's unbounded ints (countdown/env.py:16-21 evaluates answers with
eval): intermediates past int64 -- literals, a**b, shifts, products -- continue in the device
evaluator's bounded big ints (csrc/bigint.hpp, magnitudes below 2^1024) and must give exactly
oracle.countdown_reward (Python's own eval); RMI_ERR_UNSUP is allowed only for an answer whose
Python evaluation makes an int of 2^1024 or more."""
import ast
import warnings

import numpy as np
import pytest
import torch

import oracle
from ragen_amd import _lib, ops
from ragen_amd.env import CountdownBatch
from ragen_amd.env.configs import CountdownEnvConfig

pytestmark = pytest.mark.gpu
BOUND = 1 << 1024


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def past_bound(expr):
    """True if Python's evaluation of expr makes an int of 2^1024 or more in magnitude (an AST
    walk with Python's own operators; a power is sized before it is computed)."""
    try:
        tree = ast.parse(expr, mode="eval")
    except SyntaxError:
        return False
    ops_ = {ast.Add: lambda a, b: a + b, ast.Sub: lambda a, b: a - b, ast.Mult: lambda a, b: a * b,
            ast.Div: lambda a, b: a / b, ast.FloorDiv: lambda a, b: a // b, ast.Mod: lambda a, b: a % b,
            ast.LShift: lambda a, b: a << b, ast.RShift: lambda a, b: a >> b, ast.BitAnd: lambda a, b: a & b,
            ast.BitOr: lambda a, b: a | b, ast.BitXor: lambda a, b: a ^ b}
    past = [False]

    class Past(Exception):
        pass

    def chk(v):
        if isinstance(v, int) and abs(v) >= BOUND:
            past[0] = True
            raise Past
        return v

    def ev(n):
        if isinstance(n, ast.Expression):
            return ev(n.body)
        if isinstance(n, ast.Constant):
            return chk(n.value)
        if isinstance(n, ast.UnaryOp):
            v = ev(n.operand)
            return chk(-v if isinstance(n.op, ast.USub) else (+v if isinstance(n.op, ast.UAdd) else ~v))
        if isinstance(n, ast.BinOp):
            a, b = ev(n.left), ev(n.right)
            if isinstance(n.op, ast.Pow):
                if isinstance(a, int) and isinstance(b, int) and b > 0 and abs(a) > 1 and \
                        b * (abs(a).bit_length() - 1) >= 1024:
                    past[0] = True
                    raise Past
                return chk(a ** b)
            if isinstance(n.op, ast.LShift) and isinstance(a, int) and isinstance(b, int) and b > 0 and a and \
                    abs(a).bit_length() + b > 1024:
                past[0] = True
                raise Past
            return chk(ops_[type(n.op)](a, b))
        raise ValueError
    try:
        ev(tree)
    except Past:
        pass
    except Exception:
        pass
    return past[0]


KATS = [  # answers with big intermediates; nums = their digit runs, target = Python's value
    "69 ** 80 - 81",                      # the golden trace's answer: a 489-bit int
    "(2 ** 80) // (2 ** 78) + 1",         # cancelling big intermediates
    "(99 ** 99) // (99 ** 98)",
    "(99 ** 99) % 100",
    "2 ** 64 - 2 ** 64 + 7",
    "(12 ** 30) // (12 ** 29) + 3",
    "(7 ** 40) / (7 ** 39)",              # int / int past 2^53: correctly rounded
    "(3 ** 100) / (3 ** 98) - 9",
    "1 / (10 ** 300)",                    # a tiny quotient
    "(10 ** 308) * 10.0",                 # float overflow -> inf, not an error
    "(2 ** 1023) * 2.0",
    "(2 ** 1024) * 1.0",                  # 2^1024: past the bound (flagged)
    "(10 ** 309) // (10 ** 308)",         # 10^309 > 2^1024: past the bound (flagged)
    "(2 ** 1000 + 1) % 7",
    "-(2 ** 63) // -1 - (2 ** 63) + 8",
    "-(2 ** 63) * -1 - (2 ** 62) - (2 ** 62) + 8",
    "((1 << 100) >> 98) + 2",
    "(1 << 200) - (1 << 200) + 5",
    "(-(2 ** 70)) >> 68",
    "((2 ** 90) | 5) & 7",
    "((2 ** 90) ^ (2 ** 90)) + 3",
    "~(2 ** 70) + (2 ** 70) + 2",
    "(-(2 ** 100)) % 3",
    "(2 ** 100) % -3",
    "(2 ** 100) // (3 ** 60) - 30",
    "(2 ** 200) ** 0 + 2",
    "(-1) ** (2 ** 100) + 1",
    "(2 ** 100) ** -1",                   # int ** negative int -> float
    "2 ** (2 ** 11)",                     # past the bound (flagged)
    "(2 ** 70) / 0",                      # ZeroDivisionError
    "(2 ** 70) // 0",
    "(2 ** 70) % 0",
    "(2 ** 70) << -1",                    # ValueError: negative shift count
    "(2 ** 1000) / (2 ** 999) + 13",
    "(5 ** 300) / (5 ** 301) * 5",
    "(2 ** 64) * (2 ** 64) // (2 ** 127)",
    "((3 ** 200) - 1) % (3 ** 2)",
    "(2 ** 512) * (2 ** 511) // (2 ** 1020)",  # 2^1023: inside the bound
    "(2 ** 512) * (2 ** 512) // (2 ** 1020)",  # 2^1024 intermediate: flagged
]


def _case(e):
    import re
    runs = [int(x) for x in re.findall(r"\d+", e)]
    try:
        v = None if past_bound(e) else eval(e, {"__builtins__": None}, {})
    except Exception:
        v = None
    t = int(round(v)) if isinstance(v, (int, float)) and v == v and abs(v) < 2 ** 31 else 7
    return e, runs, t


def _rewards(device, cases, max_bytes=256):
    n = len(cases)
    data = [{"nums": nums, "target": target} for _, nums, target in cases]
    env = CountdownBatch(CountdownEnvConfig(data=data), n, 1, 1, device, max_answer_bytes=max_bytes, max_nums=8)
    env.reset(np.arange(n, dtype=np.int64))
    buf, lens = env.encode_answers([[e] for e, _, _ in cases])
    r, fl, err = ops.countdown_reward(env.struct(), _t(buf[:, 0], device), _t(lens[:, 0].copy(), device))
    return r.cpu().numpy(), fl.cpu().numpy(), err.cpu().numpy()


def test_countdown_bigint_kats(device):
    cases = [_case(e) for e in KATS]
    assert all(len(n) <= 8 and max(n) < 2 ** 31 for _, n, _ in cases)
    r, fl, err = _rewards(device, cases)
    for i, (e, nums, t) in enumerate(cases):
        flagged = bool(err[i] & _lib.ERR_UNSUP)
        assert flagged == past_bound(e), (e, int(err[i]))
        if not flagged:  # (Python's eval of an answer past the bound may not finish: not evaluated)
            want = oracle.countdown_reward(e, nums, t)
            assert r[i] == want, (e, r[i], want)
    # the KATs reach every outcome without leaving the model
    ok = [i for i in range(len(cases)) if not err[i]]
    assert sum(r[i] == 1 for i in ok) >= 20 and sum(r[i] == 0.1 for i in ok) >= 3


def _gen(rng, nums, depth):
    """A random arithmetic expression over nums and big-int operators (** // % << >> & | ^ ~)."""
    if depth == 0 or rng.random() < 0.25:
        r = rng.random()
        if r < 0.05:
            return str(int(rng.integers(1, 10 ** 6)) * 10 ** int(rng.integers(15, 40)))  # a big literal
        return str(int(rng.choice(nums)))
    op = rng.choice(["+", "-", "*", "//", "%", "**", "**", "<<", ">>", "&", "|", "^", "/", "*"])
    a = _gen(rng, nums, depth - 1)
    if op == "**":
        b = str(int(rng.integers(0, 60)) if rng.random() < 0.8 else int(rng.integers(60, 400)))
    elif op in ("<<", ">>"):
        b = str(int(rng.integers(0, 200)))
    else:
        b = _gen(rng, nums, depth - 1)
    e = f"({a} {op} {b})"
    if rng.random() < 0.08:
        e = f"-{e}" if rng.random() < 0.7 else f"~{e}"
    return e


def test_countdown_bigint_fuzz(device):
    """20 000 random answers with big-int intermediates: the reward == Python's; the error bit
    exactly where Python's evaluation passes 2^1024."""
    rng = np.random.default_rng(5)
    n = 20000
    cases = []
    warnings.simplefilter("ignore", SyntaxWarning)
    while len(cases) < n:
        nums = [int(x) for x in rng.integers(1, 100, size=int(rng.integers(2, 5)))]
        e = _gen(rng, nums, int(rng.integers(1, 5)))
        if len(e.encode()) > 256:
            continue
        runs = [int(x) for x in __import__("re").findall(r"\d+", e)]
        if len(runs) > 8 or any(x >= 2 ** 31 for x in runs):
            runs = None
        try:
            v = None if past_bound(e) else eval(e, {"__builtins__": None}, {})
        except Exception:
            v = None
        target = int(v) if isinstance(v, int) and abs(v) < 2 ** 31 else int(rng.integers(-50, 50))
        cases.append((e, runs if runs is not None else nums, target))
    r, fl, err = _rewards(device, cases)
    past = np.array([past_bound(e) for e, _, _ in cases])
    want = np.array([-1.0 if p else oracle.countdown_reward(e, nums, t) for (e, nums, t), p in zip(cases, past)])
    flagged = (err & _lib.ERR_UNSUP) != 0
    assert not (flagged & ~past).any(), [cases[i][0] for i in np.nonzero(flagged & ~past)[0][:5]]
    bad = np.nonzero((r != want) & ~past)[0]
    assert bad.size == 0, [(cases[i], r[i], want[i]) for i in bad[:5]]
    assert (want == 1).sum() > n // 10 and (want == 0.1).sum() > n // 20
    assert past.sum() < n // 10


def test_countdown_golden_trace_no_unsupported(device):
    """The golden countdown_es trace through EnvStateManager: its two '69 ** 80 - 81' answers
    (a 489-bit intermediate) are now evaluated, so the step warns about no answer."""
    from ragen_amd.llm_agent import EnvStateManager
    from test_gpu_facade import _config
    from trace_util import load, strings
    d = load("countdown_es")
    S = strings()["countdown_es"]
    es = EnvStateManager(_config("countdown_es"), mode="train", device=device)
    es.reset(seed=int(d["seed"]))
    active = list(range(int(d["B"])))
    with warnings.catch_warnings():
        warnings.filterwarnings("error", message=".*outside the device evaluator.*")
        for t in range(int(d["T"])):
            inputs = [{"env_id": i, "llm_response": "r", "llm_raw_response": "r",
                       "actions": [] if S["answers"][t][i] is None else [S["answers"][t][i]]} for i in active]
            outs = es.step(inputs)
            active = [o["env_id"] for o in outs]
            if not active:
                break
    assert getattr(es.tags[0].batch, "unsupported_answers", 0) == 0
