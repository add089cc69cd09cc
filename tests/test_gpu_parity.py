"""GPU parity: the HIP kernels (through the C ABI) against the golden traces recorded from
the reference and against the pinned CPU oracle at the BASELINE sizes.

Bar: bit-exact for grid state, player, counters, flags, rewards (f64) and penalties;
returns/advantages: returns bit-exact, whitened advantages within 1e-5 (f32 whitening
uses a global reduction whose order torch does not define).
"""
import numpy as np
import pytest
import torch

import oracle
from ragen_amd import _lib, ops, synthetic
from ragen_amd.env import BanditBatch, CountdownBatch, FrozenLakeBatch, SokobanBatch
from ragen_amd.env.configs import BanditEnvConfig, CountdownEnvConfig, FrozenLakeEnvConfig, SokobanEnvConfig
from trace_util import load, strings, trace_inputs

pytestmark = pytest.mark.gpu


def _t(a, dev, dt=None):
    x = torch.from_numpy(np.ascontiguousarray(a))
    if dt is not None:
        x = x.to(dt)
    return x.to(dev)


def _host_ep(ep):
    return {k: getattr(ep, k).cpu().numpy() for k in ("num_actions", "flags", "n_turns", "penalty", "turn_reward",
                                                      "turn_info", "turn_exec")}


def _check_turn(ep, d, t):
    h = _host_ep(ep)
    np.testing.assert_array_equal(h["turn_reward"][t], d["turn_reward"][t])
    np.testing.assert_array_equal(h["turn_exec"][t], d["n_exec"][t])
    np.testing.assert_array_equal(h["turn_info"][t], d["info"][t])
    np.testing.assert_array_equal(h["penalty"], d["penalty"][t])
    np.testing.assert_array_equal(h["num_actions"], d["num_actions"][t])
    np.testing.assert_array_equal((h["flags"] & 1) > 0, d["term"][t] > 0)
    np.testing.assert_array_equal((h["flags"] & 2) > 0, d["trunc"][t] > 0)
    active = (d["act_in"][t] > 0) & ((h["flags"] & 4) == 0)
    np.testing.assert_array_equal(active, d["active_after"][t] > 0)


def _check_final(ep, d):
    m = ops.rollout_metrics(ep).cpu().numpy()
    for j, k in enumerate(["success", "num_actions", "action_is_effective", "action_is_valid"]):
        np.testing.assert_array_equal(m[:, j], d["metric_" + k])
    s, p = ops.trajectory_scores(ep)
    np.testing.assert_array_equal(s.cpu().numpy(), d["score_f32"])
    np.testing.assert_array_equal(p.cpu().numpy(), d["penalty_f32"])


@pytest.mark.parametrize("name", ["sokoban_es", "sokoban8_es"])
def test_sokoban_golden_trace(device, name):
    d, ids = trace_inputs(name)
    B, T, K = int(d["B"]), int(d["T"]), int(d["K"])
    H = int(np.sqrt(d["init_room_state"].shape[1]))
    cfg = SokobanEnvConfig(dim_x=H, dim_y=H, num_boxes=1 if H == 6 else 2, max_steps=100)
    env = SokobanBatch(cfg, B, T, K, device)
    env.load_state(d["init_room_fixed"].astype(np.uint8), d["init_room_state"].astype(np.uint8),
                   d["init_player"].astype(np.int8))
    err = torch.zeros(B, dtype=torch.uint8, device=device)
    for t in range(T):
        env.step_turn(t, _t(ids[t], device), _t(d["n_act"][t].astype(np.uint8), device),
                      _t(d["act_in"][t].astype(np.uint8), device), 10, -0.1, err)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(env.room_state.cpu().numpy(), d["turn_room_state"][t].astype(np.uint8))
        np.testing.assert_array_equal(env.player.cpu().numpy(), d["turn_player"][t].astype(np.int8))
        np.testing.assert_array_equal(env.num_env_steps.cpu().numpy(), d["turn_num_env_steps"][t])
        np.testing.assert_array_equal(env.boxes_on_target.cpu().numpy(), d["turn_boxes_on_target"][t])
        _check_turn(env.ep, d, t)
    assert not err.any()
    _check_final(env.ep, d)
    final = strings()[name]["final_obs"]
    assert [env.render(i) for i in range(B)] == final


def test_frozenlake_golden_trace(device):
    d, ids = trace_inputs("frozenlake_es")
    B, T, K = int(d["B"]), int(d["T"]), int(d["K"])
    env = FrozenLakeBatch(FrozenLakeEnvConfig(), B, T, K, device)
    env.reset(synthetic.env_seeds(B, int(d["seed"]), int(d["group_size"])))
    np.testing.assert_array_equal(env.desc.cpu().numpy(), d["init_desc"])
    np.testing.assert_array_equal(env.s.cpu().numpy(), d["init_s"])
    np.testing.assert_array_equal(env.rng.cpu().numpy().view(np.uint64).T, d["init_rng_state"])
    for t in range(T):
        env.step_turn(t, _t(ids[t], device), _t(d["n_act"][t].astype(np.uint8), device),
                      _t(d["act_in"][t].astype(np.uint8), device), 10, -0.1)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(env.s.cpu().numpy(), d["turn_s"][t])
        np.testing.assert_array_equal(env.rng.cpu().numpy().view(np.uint64).T, d["turn_rng_state"][t])
        _check_turn(env.ep, d, t)
    _check_final(env.ep, d)
    assert [env.render(i) for i in range(B)] == strings()["frozenlake_es"]["final_obs"]


def test_bandit_golden_trace(device):
    d, ids = trace_inputs("bandit_es")
    B, T, K = int(d["B"]), int(d["T"]), int(d["K"])
    env = BanditBatch(BanditEnvConfig(lo_arm_name="Phoenix", hi_arm_name="Dragon"), B, T, K, device)
    env.reset(synthetic.env_seeds(B, int(d["seed"]), int(d["group_size"])))
    np.testing.assert_array_equal(env.hi_is_first.cpu().numpy(), d["init_hi_is_first"])
    for t in range(T):
        env.step_turn(t, _t(ids[t], device), _t(d["n_act"][t].astype(np.uint8), device),
                      _t(d["act_in"][t].astype(np.uint8), device), 1, -0.1)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(env.rng.cpu().numpy().view(np.uint64).T, d["turn_rng_state"][t])
        _check_turn(env.ep, d, t)
    _check_final(env.ep, d)


def test_countdown_golden_trace(device):
    d = load("countdown_es")
    S = strings()
    B, T, K = int(d["B"]), int(d["T"]), int(d["K"])
    env = CountdownBatch(CountdownEnvConfig(data=S["countdown_data"]), B, T, K, device)
    env.reset(synthetic.env_seeds(B, int(d["seed"]), int(d["group_size"])))
    np.testing.assert_array_equal(env.target.cpu().numpy(), d["init_target"])
    np.testing.assert_array_equal(env.nums.cpu().numpy(), d["init_nums"])
    answers = S["countdown_es"]["answers"]
    for t in range(T):
        lists = [[a] if a is not None else [] for a in answers[t]]
        buf, lens = env.encode_answers(lists)
        n = np.array([len(x) for x in lists], np.uint8)
        env.step_turn(t, torch.zeros(B, K, dtype=torch.int8, device=device), _t(n, device),
                      _t(d["act_in"][t].astype(np.uint8), device), 1, -0.1, answers=_t(buf, device),
                      answer_len=_t(lens, device))
        torch.cuda.synchronize()
        _check_turn(env.ep, d, t)
    _check_final(env.ep, d)


def test_countdown_reward_kat(device):
    k = strings()["countdown_kat"]
    exprs = [c["expr"] for c in k["cases"]]
    n = len(exprs)
    env = CountdownBatch(CountdownEnvConfig(data=[{"nums": k["nums"], "target": k["target"]}]), n, 1, 1, device)
    env.reset(np.zeros(n, np.int64))
    buf, lens = env.encode_answers([[e] if e else [""] for e in exprs])
    r, fl, err = ops.countdown_reward(env.struct(), _t(buf[:, 0], device), _t(lens[:, 0].copy(), device))
    r = r.cpu().numpy()
    for i, c in enumerate(k["cases"]):
        assert r[i] == c["reward"], (c, r[i], int(err[i]))


def test_countdown_reward_grammar_full_size(device):
    """CD config size (16 384 answers) of the SURVEY §8(d) answer grammar ({digits + - * / ( )},
    correct / format-only / wrong numbers): rmi_countdown_reward == oracle.countdown_reward
    (countdown/env.py:69-78, Python eval) for every answer, no answer outside the model."""
    from ragen_amd.env.countdown import synthetic_instances
    n = 16384
    inst = synthetic_instances(1024, 7)
    env = CountdownBatch(CountdownEnvConfig(data=inst), n, 1, 1, device)
    env.reset(synthetic.env_seeds(n))
    mine = [inst[int(i)] for i in env.index]
    exprs = synthetic.countdown_answers(mine, 1, p_empty=0.0)[0]
    buf, lens = env.encode_answers([[e] for e in exprs])
    r, fl, err = ops.countdown_reward(env.struct(), _t(buf[:, 0], device), _t(lens[:, 0].copy(), device))
    r, err = r.cpu().numpy(), err.cpu().numpy()
    want = np.array([oracle.countdown_reward(e, list(m["nums"]), int(m["target"])) for e, m in zip(exprs, mine)])
    assert not err.any()
    bad = np.nonzero(r != want)[0]
    assert bad.size == 0, [(exprs[i], r[i], want[i]) for i in bad[:5]]
    assert (want == 1).sum() > n // 4 and (want == 0.1).sum() > n // 8 and (want == 0).sum() > n // 4


def _fuzz_answers(n, seed):
    """Random strings over the fast path's bytes "0-9 +-*/()" and ' ' (plus, rarely, bytes that
    leave it: '.', '%', '\\t', '**', '//', 'x'), each with nums = its digit runs and target =
    its Python value where that is an int32, so format and value hit both outcomes."""
    import re
    import warnings
    warnings.simplefilter("ignore", SyntaxWarning)  # "'int' object is not callable" from eval
    rng = np.random.default_rng(seed)
    alpha = list("0123456789+-*/() ") + ["12", "7", " + ", " - ", " * ", " / ", "(", ")"]
    rare = [".", "%", "\t", "//", "x", "05", "0"]
    def tree(depth):  # a valid expression: unary signs, nesting, all four operators
        if depth == 0 or rng.random() < 0.3:
            e = str(int(rng.choice([0, 1, 2, 7, 12, 99, 12345, 99999999999])))
        else:
            e = tree(depth - 1) + " " + "+-*/"[int(rng.integers(0, 4))] + " " + tree(depth - 1)
            if rng.random() < 0.5:
                e = "(" + e + ")"
        return "".join(rng.choice(["-", "+", "- "], int(rng.integers(0, 3)))) + e

    out, data = [], []
    for _ in range(n):
        if rng.random() < 0.5:
            e = tree(int(rng.integers(1, 5)))
            if len(e) > 60 or e.count("(") > 12:
                e = "((((((((((((((((((1))))))))))))))))))"  # nesting beyond the fast path
        else:
            toks = [alpha[int(j)] for j in rng.integers(0, len(alpha), int(rng.integers(0, 14)))]
            if rng.random() < 0.1:
                toks.insert(int(rng.integers(0, len(toks) + 1)), rare[int(rng.integers(0, len(rare)))])
            e = "".join(toks)[:58]
        if rng.random() < 0.02:
            e += "**2"  # at the end only: a random exponent could take Python forever
        runs = [int(x) for x in re.findall(r"\d+", e)][:4]
        try:
            v = eval(e, {"__builtins__": None}, {})
            tgt = int(v) if isinstance(v, (int, float)) and abs(v) < 2**31 and v == int(v) else 1
        except Exception:
            tgt = 1
        if rng.random() < 0.2:
            tgt += 1
        out.append(e)
        data.append({"nums": [x if x < 2**31 else 1 for x in runs] or [1], "target": tgt})
    return out, data


def test_countdown_reward_fuzz(device):
    """Random answers over the fast path's alphabet (syntax errors, unary chains, deep parens,
    division by zero, int overflow, bytes that leave the fast path) == oracle.countdown_reward;
    an answer flagged RMI_ERR_UNSUP (outside the evaluator's model) is only allowed where
    Python's value is beyond int64 / not modelled."""
    n = 20000
    exprs, data = _fuzz_answers(n, 7)
    env = CountdownBatch(CountdownEnvConfig(data=data), n, 1, 1, device, max_answer_bytes=64)
    env.reset(np.arange(n, dtype=np.int64))
    buf, lens = env.encode_answers([[e] for e in exprs])
    r, fl, err = ops.countdown_reward(env.struct(), _t(buf[:, 0], device), _t(lens[:, 0].copy(), device))
    r, err = r.cpu().numpy(), err.cpu().numpy()
    want = np.array([oracle.countdown_reward(e, d["nums"], d["target"]) for e, d in zip(exprs, data)])
    bad = [i for i in np.nonzero(r != want)[0] if not err[i]]
    assert not bad, [(exprs[i], r[i], want[i]) for i in bad[:5]]
    assert (err != 0).sum() < n // 50
    assert (want == 1).sum() > n // 20 and (want == 0.1).sum() > n // 20


def _tree_answers(n, seed):
    """Valid expressions shaped for the 16-lane evaluator's envelope edges: random binary trees
    over + - * / (left chains, ties of equal keys, groups on either side), redundant parens,
    signs on literals and on groups, 1..8 literals, depth up to 5, 14..18 tokens, ints around
    2**53, float results, zero divisors, 0 and -0 operands."""
    rng = np.random.default_rng(seed)
    lits = [0, 1, 2, 3, 7, 12, 99, 100, 12345, 94906265, 94906266, 99999999]

    def expr(nl, depth):
        if nl == 1:
            e = str(int(rng.choice(lits)))
        else:
            cut = int(rng.integers(1, nl))
            e = expr(cut, depth + 1) + rng.choice([" ", ""]) + "+-*/"[int(rng.integers(0, 4))] + \
                rng.choice([" ", ""]) + expr(nl - cut, depth + 1)
            if rng.random() < 0.45:
                e = "(" + e + ")"
        if rng.random() < 0.08:
            e = "(" + e + ")"  # redundant group
        if rng.random() < 0.15:
            e = "".join(rng.choice(["-", "+", "- "], int(rng.integers(1, 5)))) + e  # signs, some before '('
        return e

    out, data = [], []
    for _ in range(n):
        e = expr(int(rng.integers(1, 9)), 0)
        if len(e) > 64:
            e = e[:64]  # a cut expression: a syntax error (or > 64 bytes handled by the fallback)
        runs = [int(x) for x in __import__("re").findall(r"\d+", e)]
        try:
            v = eval(e, {"__builtins__": None}, {})
            tgt = int(v) if isinstance(v, (int, float)) and abs(v) < 2**31 and v == int(v) else 5
        except Exception:
            tgt = 5
        if rng.random() < 0.15:
            tgt += 1
        nums = [x if x < 2**31 else 1 for x in runs][:8] or [1]
        if rng.random() < 0.1:
            nums = nums[::-1] + [3]  # format mismatch
        out.append(e)
        data.append({"nums": nums[:8], "target": tgt})
    return out, data


def _past_int64(expr):
    """True if evaluating expr (+ - * / and unary signs) makes an int of 2**63 or more in
    magnitude (a Python big int: outside the device evaluator's int64 model)."""
    import ast
    try:
        tree = ast.parse(expr, mode="eval")
    except SyntaxError:
        return False
    seen = [False]

    def ev(n):
        if isinstance(n, ast.Expression):
            return ev(n.body)
        if isinstance(n, ast.Constant):
            return n.value
        if isinstance(n, ast.UnaryOp):
            v = ev(n.operand)
            v = -v if isinstance(n.op, ast.USub) else v
        else:
            a, b = ev(n.left), ev(n.right)
            op = type(n.op)
            v = a + b if op is ast.Add else a - b if op is ast.Sub else a * b if op is ast.Mult else a / b
        if isinstance(v, int) and abs(v) >= 2**63:
            seen[0] = True
        return v
    try:
        ev(tree)
    except ZeroDivisionError:
        pass
    return seen[0]


def test_countdown_reward_tree_shapes(device):
    """The 16-lane evaluator (one token per lane: syntax from neighbours, the Cartesian tree of
    operator keys, node-by-node f64 evaluation) and its fallbacks == oracle.countdown_reward
    (Python eval) on 20 000 tree-shaped answers, with no RMI_ERR_UNSUP (products past int64 are
    Python big ints, evaluated by the fallback's bounded big ints)."""
    n = 20000
    exprs, data = _tree_answers(n, 11)
    env = CountdownBatch(CountdownEnvConfig(data=data), n, 1, 1, device, max_answer_bytes=64, max_nums=8)
    env.reset(np.arange(n, dtype=np.int64))
    buf, lens = env.encode_answers([[e] for e in exprs])
    r, fl, err = ops.countdown_reward(env.struct(), _t(buf[:, 0], device), _t(lens[:, 0].copy(), device))
    r, fl, err = r.cpu().numpy(), fl.cpu().numpy(), err.cpu().numpy()
    want = np.array([oracle.countdown_reward(e, d["nums"], d["target"]) for e, d in zip(exprs, data)])
    big = np.array([_past_int64(e) for e in exprs])
    assert big.sum() > 0  # answers with Python big ints (past int64) are among them ...
    bad = np.nonzero(r != want)[0]
    assert bad.size == 0, [(exprs[i], data[i], r[i], want[i]) for i in bad[:5]]
    assert not err.any()  # ... and are evaluated too (bigint.hpp): no answer leaves the model
    ok = np.ones(n, bool)
    assert np.array_equal((fl & 1)[ok], (want[ok] > 0).astype(np.uint8))
    assert np.array_equal((fl >> 1 & 1)[ok], (want[ok] == 1).astype(np.uint8))
    assert (want == 1).sum() > n // 10 and (want == 0.1).sum() > n // 10


# ------------------------------------------------------------- BASELINE-size parity vs oracle
@pytest.mark.parametrize("B", [8192, 20000])
def test_sokoban_full_size_vs_oracle(device, B):
    """SK config: 8192 envs x 5 turns, K=5, cap 10 — kernel == oracle bit for bit each turn
    (20000 envs: the one-lane-per-env launch, partial last wave)."""
    T, K = 5, 5
    cfg = SokobanEnvConfig(dim_x=6, dim_y=6, num_boxes=1, max_steps=100)
    env = SokobanBatch(cfg, B, T, K, device)
    env.reset(synthetic.env_seeds(B))
    fixed = env.room_fixed.cpu().numpy()
    state = env.room_state.cpu().numpy()
    player = env.player.cpu().numpy()
    nes = np.zeros(B, np.int32)
    bot = np.zeros(B, np.int32)
    oep = oracle.Episode(B, T)
    ids, n = synthetic.rollout_actions(B, T, K, 1, 4)
    total_steps = 0
    for t in range(T):
        env.step_turn(t, _t(ids[t], device), _t(n[t], device), None, 10, -0.1)
        oracle.sokoban_turn(6, 6, 1, 100, fixed, state, player, nes, bot, oep, t, ids[t], n[t], None, 10, -0.1)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(env.room_state.cpu().numpy(), state)
        np.testing.assert_array_equal(env.player.cpu().numpy(), player)
        h = _host_ep(env.ep)
        for k in ("num_actions", "flags", "n_turns", "penalty", "turn_reward", "turn_info", "turn_exec"):
            np.testing.assert_array_equal(h[k], getattr(oep, k), err_msg=k)
        total_steps += int(oep.turn_exec[t].sum())
    assert total_steps > 6 * B
    np.testing.assert_array_equal(ops.rollout_metrics(env.ep).cpu().numpy(), oracle.rollout_metrics(oep))


def test_sokoban_big_batch_vs_oracle(device):
    """131 072 envs (the bench's 8192 rooms tiled 16x, 2048 one-wave workgroups: every CU holds
    several) — kernel == oracle bit for bit each turn, with has_input both given and derived
    from the done flags."""
    T, K, tile = 5, 5, 16
    cfg = SokobanEnvConfig(dim_x=6, dim_y=6, num_boxes=1, max_steps=100)
    small = SokobanBatch(cfg, 8192, T, K, device)
    small.reset(synthetic.env_seeds(8192))
    B = 8192 * tile
    env = SokobanBatch(cfg, B, T, K, device)
    fixed = np.tile(small.room_fixed.cpu().numpy(), (tile, 1))
    state = np.tile(small.room_state.cpu().numpy(), (tile, 1))
    player = np.tile(small.player.cpu().numpy(), (tile, 1))
    env.load_state(fixed, state, player)
    nes = np.zeros(B, np.int32)
    bot = np.zeros(B, np.int32)
    oep = oracle.Episode(B, T)
    ids, n = synthetic.rollout_actions(B, T, K, 1, 4, seed=9)
    has = (np.random.default_rng(4).random((T, B)) < 0.9).astype(np.uint8)
    for t in range(T):
        h_in = has[t] if t % 2 else None
        env.step_turn(t, _t(ids[t], device), _t(n[t], device), None if h_in is None else _t(h_in, device), 10, -0.1)
        oracle.sokoban_turn(6, 6, 1, 100, fixed, state, player, nes, bot, oep, t, ids[t], n[t], h_in, 10, -0.1)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(env.room_state.cpu().numpy(), state)
        np.testing.assert_array_equal(env.player.cpu().numpy(), player)
        h = _host_ep(env.ep)
        for k in ("num_actions", "flags", "n_turns", "penalty", "turn_reward", "turn_info", "turn_exec"):
            np.testing.assert_array_equal(h[k], getattr(oep, k), err_msg=k)
    assert (oep.flags & 4).any() and not (oep.flags & 4).all()


def test_frozenlake_full_size_vs_oracle(device):
    B, T, K = 4096, 8, 5
    env = FrozenLakeBatch(FrozenLakeEnvConfig(), B, T, K, device)
    env.reset(synthetic.env_seeds(B))
    desc = env.desc.cpu().numpy()
    s = env.s.cpu().numpy()
    rng = env.rng.cpu().numpy().view(np.uint64).copy()
    oep = oracle.Episode(B, T)
    ids, n = synthetic.rollout_actions(B, T, K, 1, 4, seed=5)
    for t in range(T):
        env.step_turn(t, _t(ids[t], device), _t(n[t], device), None, 10, -0.1)
        oracle.frozenlake_turn(4, 4, True, env.cs, desc, s, rng, oep, t, ids[t], n[t], None, 10, -0.1)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(env.s.cpu().numpy(), s)
        np.testing.assert_array_equal(env.rng.cpu().numpy().view(np.uint64), rng)
        h = _host_ep(env.ep)
        for k in ("num_actions", "flags", "penalty", "turn_reward", "turn_info", "turn_exec"):
            np.testing.assert_array_equal(h[k], getattr(oep, k), err_msg=k)


def test_bandit_full_size_vs_oracle(device):
    """BD at scale: 16384 envs x 3 turns (cap 2), ids 0..3 (unknown names and invalid ids
    included): kernel == oracle incl. PCG64 states and error flags."""
    B, T, K = 16384, 3, 2
    env = BanditBatch(BanditEnvConfig(lo_arm_name="Phoenix", hi_arm_name="Dragon"), B, T, K, device)
    env.reset(synthetic.env_seeds(B))
    hi = env.hi_is_first.cpu().numpy()
    rng = env.rng.cpu().numpy().view(np.uint64).copy()
    c = env.config
    oep = oracle.Episode(B, T)
    g = np.random.default_rng(8)
    bad = np.zeros(B, bool)
    for t in range(T):
        ids = g.integers(0, 4, size=(B, K)).astype(np.int8)
        n = g.integers(0, K + 1, size=B).astype(np.uint8)
        err = torch.zeros(B, dtype=torch.uint8, device=device)
        env.step_turn(t, _t(ids, device), _t(n, device), None, 2, -0.1, err)
        oerr = oracle.bandit_turn(int(c.action_space_start), c.lo_arm_score, c.hi_arm_loscore, c.hi_arm_hiscore,
                                  c.hi_arm_hiscore_prob, hi, rng, oep, t, ids, n, None, 2, -0.1)
        torch.cuda.synchronize()
        np.testing.assert_array_equal((err.cpu().numpy() != 0)[~bad], (oerr != 0)[~bad])
        bad |= oerr != 0
        ok = ~bad
        np.testing.assert_array_equal(env.rng.cpu().numpy().view(np.uint64)[:, ok], rng[:, ok])
        h = _host_ep(env.ep)
        for k in ("num_actions", "flags", "penalty"):
            np.testing.assert_array_equal(h[k][ok], getattr(oep, k)[ok], err_msg=k)
        for k in ("turn_reward", "turn_info", "turn_exec"):
            np.testing.assert_array_equal(h[k][:, ok], getattr(oep, k)[:, ok], err_msg=k)


def test_gae_full_size(device):
    """B=8192 rows ~1k tokens: legacy/masked GAE returns bit-exact vs oracle, whitened adv <= 1e-5."""
    B = 8192
    rng = np.random.default_rng(0)
    n_turns = rng.integers(1, 6, size=B)
    scores = rng.choice([-0.5, 0.9, 10.4, -1.2], size=B).astype(np.float32)
    r, v, m = synthetic.token_rows(n_turns, scores, seed=1)
    tr, tv, tm = _t(r, device), _t(v, device), _t(m, device)
    for variant, (g, lam) in (("legacy", (1.0, 1.0)), ("legacy", (1.0, 0.95)), ("masked", (0.99, 0.95))):
        stats = torch.zeros(B, 3, dtype=torch.float64, device=device)
        adv, ret = ops.gae(tr, tv, tm, g, lam, variant, row_stats=stats)
        oadv, oret = oracle.gae(r, v, m, g, lam, variant)
        np.testing.assert_array_equal(ret.cpu().numpy(), oret)
        np.testing.assert_array_equal(adv.cpu().numpy(), oadv)
        ops.masked_whiten_(adv, tm, stats)
        np.testing.assert_allclose(adv.cpu().numpy(), oracle.masked_whiten(oadv, m), rtol=0, atol=1e-5)


def test_gae_golden(device):
    d = load("gae")
    m = d["mask"]
    tm = _t(m, device)
    for gl in ("g1.0_l1.0", "g1.0_l0.95", "g0.99_l0.95"):
        g, lam = (float(x[1:]) for x in gl.split("_"))
        for rn in ("last", "turn"):
            r = _t(d["rew"] if rn == "last" else d["rew_turn"], device)
            v = _t(d["values"], device)
            for var, key in (("legacy", "gae"), ("masked", "gaem")):
                adv, ret = ops.gae(r, v, tm, g, lam, var)
                np.testing.assert_array_equal(ret.cpu().numpy(), d[f"{key}_{rn}_{gl}_ret"])
                ops.masked_whiten_(adv, tm)
                np.testing.assert_allclose(adv.cpu().numpy(), d[f"{key}_{rn}_{gl}_adv"], rtol=0, atol=1e-5)
            adv, ret = ops.bilevel_gae(r, v, tm, g, lam, 0.95)
            np.testing.assert_array_equal(ret.cpu().numpy(), d[f"bilevel_{rn}_{gl}_ret"])
            ops.masked_whiten_(adv, tm)
            np.testing.assert_allclose(adv.cpu().numpy(), d[f"bilevel_{rn}_{gl}_adv"], rtol=0, atol=1e-5)
    with pytest.raises(IndexError):
        ops.bilevel_gae(_t(np.array([[0, 1, 0, 0]], np.float32), device), torch.zeros(1, 4, device=device),
                        torch.ones(1, 4, dtype=torch.uint8, device=device), 1.0, 1.0, 0.95)


def test_grpo_golden(device):
    d = load("gae")
    B = d["mask"].shape[0]
    r, tm = _t(d["rew_turn"], device), _t(d["mask"], device)
    adv, ret = ops.grpo_outcome(r, tm, _t(np.arange(B + 1, dtype=np.int32), device))
    np.testing.assert_allclose(adv.cpu().numpy(), d["ca_grpo_0_adv"], rtol=1e-6, atol=1e-6)
    adv, ret = ops.grpo_outcome(r, tm, _t(np.arange(0, B + 1, 4, dtype=np.int32), device))
    np.testing.assert_allclose(adv.cpu().numpy(), d["grpo_g4_adv"], rtol=1e-5, atol=1e-5)


def test_normalize_golden(device):
    d = load("normalize")
    B = len(d["scores"])
    sc, pen = _t(d["scores"], device), _t(d["penalty"].astype(np.float32), device)
    segs = {"state": np.arange(0, B + 1, 16), "inductive": np.array([0, 48, 96]), "batch": np.array([0, B])}
    for grouping, seg in segs.items():
        for method in ("mean_std", "mean", "asym_clip", "identity"):
            out = ops.group_normalize(sc, pen, _t(seg.astype(np.int32), device), method)
            np.testing.assert_allclose(out.cpu().numpy(), d[f"norm_{grouping}_{method}"], rtol=0, atol=1e-5)


def test_filter_vs_oracle(device):
    d = load("filter")
    for key in ("r0.25_std", "r0.25_std_rev", "r1.0_std", "r0.5_std"):
        ratio = float(key.split("_")[0][1:])
        ftype = key.split("_", 1)[1]
        rows = ops.row_sum(_t(d[key + "_scores"], device))
        keep, met, (sd, mx, mn) = ops.filter_groups(rows, 64, 16, ratio, ftype)
        okeep, omet, (osd, omx, omn) = oracle.filter_groups(rows.cpu().numpy(), 64, 16, ratio, ftype)
        np.testing.assert_array_equal(keep.cpu().numpy(), okeep)
        np.testing.assert_allclose(met.cpu().numpy(), omet, rtol=1e-6)
        np.testing.assert_array_equal(sd.cpu().numpy(), osd)
    # large G with many ties: deterministic selection identical to the oracle's documented order
    G, gs = 4096, 16
    rng = np.random.default_rng(2)
    sc = np.repeat(rng.choice([0.0, 1.0, -0.5], size=G), gs).astype(np.float32)
    sc[rng.random(G * gs) < 0.05] = 10.0
    keep, met, _ = ops.filter_groups(_t(sc, device), G, gs, 0.25, "std")
    okeep, omet, _ = oracle.filter_groups(sc, G, gs, 0.25, "std")
    np.testing.assert_array_equal(keep.cpu().numpy(), okeep)


@pytest.mark.parametrize("G", [8193, 40000])
def test_filter_large_g_vs_oracle(device, G):
    """G above the LDS sort's 8192 groups: the radix-select path keeps the same groups (ties by
    ascending index) and reports the same metrics; a score count != G*gs raises as view() does."""
    gs = 16
    rng = np.random.default_rng(G)
    sc = np.repeat(rng.choice([0.0, 1.0, -0.5, 2.5], size=G), gs).astype(np.float32)
    sc[rng.random(G * gs) < 0.03] = 10.0
    sc[rng.random(G * gs) < 0.01] = rng.standard_normal(1)[0]
    for ratio, ftype in ((0.25, "std"), (0.25, "std_rev"), (0.5, "std"), (1.0, "std"), (0.0, "std")):
        keep, met, (sd, mx, mn) = ops.filter_groups(_t(sc, device), G, gs, ratio, ftype)
        okeep, omet, (osd, omx, omn) = oracle.filter_groups(sc, G, gs, ratio, ftype)
        np.testing.assert_array_equal(keep.cpu().numpy(), okeep, err_msg=f"{ratio} {ftype}")
        np.testing.assert_allclose(met.cpu().numpy(), omet, rtol=1e-6)
        np.testing.assert_array_equal(sd.cpu().numpy(), osd)
        np.testing.assert_array_equal(mx.cpu().numpy(), omx)
    with pytest.raises(RuntimeError):
        ops.filter_groups(_t(sc[:-gs], device), G, gs, 0.25, "std")


def test_whiten_errors_and_empty(device):
    x = torch.zeros(2, 3, device=device)
    ops.masked_whiten_(x, torch.zeros(2, 3, dtype=torch.uint8, device=device))  # status recorded, no crash
    e = ops.EpisodeState.empty(0, 1, device)
    assert ops.rollout_metrics(e).shape == (0, 4)


def test_fused_reset_and_finalize(device):
    """rmi_sokoban_reset == a fresh load; rmi_rollout_finalize == metrics + scores + normalize."""
    B, T, K = 1024, 5, 5
    env = SokobanBatch(SokobanEnvConfig(dim_x=6, dim_y=6, num_boxes=1, max_steps=100), B, T, K, device)
    env.reset(synthetic.env_seeds(B))
    s0 = env.room_state.clone()
    ids, n = synthetic.rollout_actions(B, T, K, 1, 4, seed=11)
    outs = []
    for rep in range(2):
        env.restore()
        assert torch.equal(env.room_state, s0)
        for t in range(T):
            env.step_turn(t, _t(ids[t], device), _t(n[t], device), None, 10, -0.1)
        outs.append(env.room_state.clone())
    assert torch.equal(outs[0], outs[1])
    seg = torch.arange(0, B + 1, 16, dtype=torch.int32, device=device)
    for method in ("identity", "mean", "mean_std", "asym_clip"):
        norm = torch.empty(B, dtype=torch.float32, device=device)
        met = torch.empty(B, 4, dtype=torch.float64, device=device)
        sc = torch.empty(B, dtype=torch.float32, device=device)
        pe = torch.empty(B, dtype=torch.float32, device=device)
        ops.rollout_finalize(env.ep, seg, method, norm, met, sc, pe)
        s2, p2 = ops.trajectory_scores(env.ep)
        assert torch.equal(sc, s2) and torch.equal(pe, p2)
        assert torch.equal(torch.nan_to_num(met, 7.0), torch.nan_to_num(ops.rollout_metrics(env.ep), 7.0))
        assert torch.equal(norm, ops.group_normalize(s2, p2, seg, method))


def _irregular_rooms(rng, B, H, W, fixed, state, player):
    """Overwrite some rooms with hand-made ones the generator never makes: open borders, a
    player on / outside the border (numpy wrap and IndexError), inconsistent state bytes."""
    hw = H * W
    kind = rng.integers(0, 4, size=B)
    for i in np.nonzero(kind == 0)[0]:          # random grids, anything goes
        f = rng.choice([0, 1, 2], size=hw, p=[0.3, 0.5, 0.2]).astype(np.uint8)
        s = f.copy()
        m = rng.random(hw) < 0.2
        s[m] = rng.choice([3, 4], size=int(m.sum()))
        fixed[i], state[i] = f, s
        player[i] = rng.integers(-H - 1, H + 1, size=2)
    for i in np.nonzero(kind == 1)[0]:          # regular room, player moved onto the border
        r, c = (0, int(rng.integers(0, W))) if rng.random() < 0.5 else (int(rng.integers(0, H)), W - 1)
        fixed[i].reshape(H, W)[r, c] = 1
        state[i].reshape(H, W)[r, c] = 5
        state[i][state[i] == 5] = fixed[i][state[i] == 5]
        state[i].reshape(H, W)[r, c] = 5
        player[i] = (r, c)
    for i in np.nonzero(kind == 2)[0]:          # one inconsistent byte
        state[i][int(rng.integers(0, hw))] = int(rng.integers(0, 6))


@pytest.mark.parametrize("frac_irregular,B", [(0.0, 2050), (0.01, 2050), (0.5, 2050), (0.5, 16500)])
def test_sokoban_irregular_rooms_vs_oracle(device, frac_irregular, B):
    """Waves mixing regular (bitboard path) and irregular rooms (exact LDS path), invalid and
    out-of-range action ids: kernel == oracle on every env the reference would not raise on,
    and the same error flags where it would.  B = 2050 runs 4 lanes per env (partial last
    wave), B = 16500 one lane per env."""
    rng = np.random.default_rng(int(frac_irregular * 1000) + B)
    T, K, H, W = 4, 6, 6, 6
    env = SokobanBatch(SokobanEnvConfig(dim_x=H, dim_y=W, num_boxes=1, max_steps=12), B, T, K, device)
    env.reset(synthetic.env_seeds(B))
    fixed = env.room_fixed.cpu().numpy().copy()
    state = env.room_state.cpu().numpy().copy()
    player = env.player.cpu().numpy().copy()
    sel = rng.random(B) < frac_irregular
    idx = np.nonzero(sel)[0]
    f2, s2, p2 = fixed[idx].copy(), state[idx].copy(), player[idx].copy()
    _irregular_rooms(rng, len(idx), H, W, f2, s2, p2)
    fixed[idx], state[idx], player[idx] = f2, s2, p2
    env.load_state(fixed, state, player)
    nes = np.zeros(B, np.int32)
    bot = np.zeros(B, np.int32)
    oep = oracle.Episode(B, T)
    bad = np.zeros(B, bool)
    for t in range(T):
        ids = rng.choice([0, 1, 2, 3, 4, 5, 6, 7, 8, 9, -1], size=(B, K),
                         p=[0.05] + [0.11] * 8 + [0.03, 0.04]).astype(np.int8)
        if frac_irregular == 0.0:
            ids = np.clip(ids, 1, 8).astype(np.int8)
        n = rng.integers(0, K + 1, size=B).astype(np.uint8)
        err = torch.zeros(B, dtype=torch.uint8, device=device)
        env.step_turn(t, _t(ids, device), _t(n, device), None, 9, -0.1, err)
        oerr = oracle.sokoban_turn(H, W, 1, 12, fixed, state, player, nes, bot, oep, t, ids, n, None, 9, -0.1)
        torch.cuda.synchronize()
        kerr = err.cpu().numpy()
        np.testing.assert_array_equal(kerr != 0, oerr != 0)
        bad |= oerr != 0
        ok = ~bad
        np.testing.assert_array_equal(env.room_state.cpu().numpy()[ok], state[ok])
        np.testing.assert_array_equal(env.player.cpu().numpy()[ok], player[ok])
        np.testing.assert_array_equal(env.num_env_steps.cpu().numpy()[ok], nes[ok])
        np.testing.assert_array_equal(env.boxes_on_target.cpu().numpy()[ok], bot[ok])
        h = _host_ep(env.ep)
        for k in ("num_actions", "flags", "n_turns", "penalty"):
            np.testing.assert_array_equal(h[k][ok], getattr(oep, k)[ok], err_msg=k)
        for k in ("turn_reward", "turn_info", "turn_exec"):
            np.testing.assert_array_equal(h[k][:, ok], getattr(oep, k)[:, ok], err_msg=k)
    if frac_irregular == 0.0:
        assert not bad.any()


def _chat_ids(rng, B, S, sp, rt, dup_rate=0.0):
    """Left-padded chat-shaped token rows: system, then user/assistant turns, each turn
    <sp> body <rt> [\\n]; some rows get a second reward token inside an assistant turn."""
    ids = np.full((B, S), 151643, np.int64)
    for b in range(B):
        row = [sp] + list(rng.integers(100, 1000, size=int(rng.integers(2, 6)))) + [rt, 198]
        for _ in range(int(rng.integers(0, 6))):
            row += [sp] + list(rng.integers(100, 1000, size=int(rng.integers(1, 7)))) + [rt, 198]
            body = list(rng.integers(100, 1000, size=int(rng.integers(1, 7))))
            if rng.random() < dup_rate:
                body.insert(int(rng.integers(0, len(body) + 1)), rt)
            row += [sp] + body + [rt]
            if rng.random() < 0.5:
                row += [198]
        row = row[-S:]
        ids[b, S - len(row):] = row
    return ids


@pytest.mark.parametrize("B,S,roll", [(257, 97, True), (300, 130, False), (64, 1, True), (33, 2, True)])
def test_masks_and_scores_vs_oracle(device, B, S, roll):
    rng = np.random.default_rng(B * 1000 + S)
    sp, rt = 151644, 151645
    ids = _chat_ids(rng, B, S, sp, rt, dup_rate=0.05)
    n = rng.integers(0, 6, size=B).astype(np.int32)
    T = 6
    tab = rng.standard_normal((T, B))
    for uts in (False, True):
        for erm in (False, True):
            for n_slots in (int(n.max()), T + 2):
                want = oracle.masks_and_scores(ids, sp, rt, tab, n, n_slots, uts, erm, roll)
                got = ops.masks_and_scores(_t(ids, device), sp, rt, _t(tab, device), _t(n, device), n_slots, uts,
                                           erm, roll)
                sc, lm, rm, err = (x.cpu().numpy() for x in got)
                np.testing.assert_array_equal(lm.astype(np.uint8), want[1])
                np.testing.assert_array_equal(rm.astype(np.uint8), want[2])
                if uts:
                    np.testing.assert_array_equal(err != 0, want[3] != 0)
                ok = want[3] == 0 if uts else np.ones(B, bool)
                np.testing.assert_array_equal(sc[ok], want[0][ok])


def test_masks_and_scores_full_size(device):
    """SK-sized token batch (8192 rows x 1024) against the oracle, turn scores + Qwen roll."""
    rng = np.random.default_rng(5)
    B, S, T = 8192, 1024, 5
    sp, rt = 151644, 151645
    ids = _chat_ids(rng, B, S, sp, rt)
    n = rng.integers(1, T + 1, size=B).astype(np.int32)
    tab = rng.standard_normal((T, B))
    want = oracle.masks_and_scores(ids, sp, rt, tab, n, T, True, True, True)
    got = ops.masks_and_scores(_t(ids, device), sp, rt, _t(tab, device), _t(n, device), T, True, True, True)
    for g, w in zip(got[:3], want[:3]):
        np.testing.assert_array_equal(g.cpu().numpy().astype(w.dtype), w)
    assert not got[3].any()


def test_render_vs_oracle(device):
    """Device text observations == the reference's render, incl. unknown
    codes ('?'), multi-byte glyphs and players on targets / holes / goals."""
    rng = np.random.default_rng(9)
    B = 777
    env = SokobanBatch(SokobanEnvConfig(dim_x=6, dim_y=6, num_boxes=1, max_steps=100), B, 2, 5, device)
    env.reset(synthetic.env_seeds(B))
    st = env.room_state.cpu().numpy()
    fx = env.room_fixed.cpu().numpy()
    st[:100] = rng.integers(0, 20, size=(100, 36))
    fx[:100] = rng.integers(0, 3, size=(100, 36))
    env.room_state.copy_(torch.from_numpy(st))
    env.room_fixed.copy_(torch.from_numpy(fx))
    env._invalidate()
    lk = env.config.grid_lookup
    got = env.render_all()
    assert got == [oracle.sokoban_render(st[i], fx[i], 6, 6, lk) for i in range(B)]
    fl = FrozenLakeBatch(FrozenLakeEnvConfig(), B, 2, 5, device)
    fl.reset(synthetic.env_seeds(B))
    s = rng.integers(0, 16, size=B).astype(np.int32)
    fl.s.copy_(torch.from_numpy(s))
    fl._invalidate()
    desc = fl.desc.cpu().numpy()
    assert fl.render_all() == [oracle.frozenlake_render(desc[i], int(s[i]), 4, fl.config.grid_lookup)
                               for i in range(B)]


@pytest.mark.parametrize("H,W", [(8, 8), (3, 5), (1, 64), (16, 4), (2, 3)])
def test_render_shapes_vs_oracle(device, H, W):
    """The 16-lanes-per-env render at other grid shapes (token runs of 1..8 per lane, rows of
    1..64 cells, one row without any newline), random codes incl. unknown ones, multi-byte
    glyphs, players on targets."""
    rng = np.random.default_rng(H * 100 + W)
    B = 300
    st = rng.integers(0, 9, size=(B, H * W)).astype(np.uint8)
    fx = rng.integers(0, 3, size=(B, H * W)).astype(np.uint8)
    lk = {0: "#", 1: "_", 2: "O", 3: "\u221a", 4: "X", 5: "P", 6: "S", 7: "\U0001F600"}
    gb, gl = ops.glyph_table(lk)
    out, n = torch.ops.ragen_amd.sokoban_render(_t(fx, device), _t(st, device), H, W, [int(x) for x in gb],
                                                [int(x) for x in gl])
    got = [bytes(out[i, :int(n[i])].cpu().numpy()).decode() for i in range(B)]
    assert got == [oracle.sokoban_render(st[i], fx[i], H, W, lk) for i in range(B)]


@pytest.mark.parametrize("B,T", [(1024, 5), (8192, 5), (2048, 10), (131072, 5)])
def test_fused_last_turn_finalize(device, B, T):
    """rmi_sokoban_step_turn_finalize == rmi_sokoban_step_turn + rmi_rollout_finalize, bit for bit
    (both lane layouts; groups that fit a wave, and the two-launch path for ones that do not;
    131072 envs: the large-batch form whose rows are loaded only for acting envs)."""
    K = 5
    cfg = SokobanEnvConfig(dim_x=6, dim_y=6, num_boxes=1, max_steps=100)
    ids, n = synthetic.rollout_actions(B, T, K, 1, 4, seed=23)
    ids, n = _t(ids, device), _t(n, device)
    big = B >= 131072
    for gs in ((16,) if big else (16, 4, 64)):
        for method in (("identity", "mean_std") if big else ("identity", "mean", "mean_std", "asym_clip")):
            outs = []
            for fused in (False, True):
                env = SokobanBatch(cfg, B, T, K, device)
                env.reset(synthetic.env_seeds(B))
                st = env.struct()
                norm = torch.full((B,), 7.0, dtype=torch.float32, device=device)
                met = torch.full((B, 4), 7.0, dtype=torch.float64, device=device)
                sc = torch.full((B,), 7.0, dtype=torch.float32, device=device)
                pe = torch.full((B,), 7.0, dtype=torch.float32, device=device)
                last = T - 2  # the rollout may end before the record is full
                for t in range(last + 1):
                    turn = ops.turn_struct(t, ids[t], n[t], None, 10, -0.1)
                    if fused and t == last:
                        fin = ops.finalize_struct(gs, method, norm, met, sc, pe)
                        ops.sokoban_step_turn_finalize(st, env.ep, turn, fin)
                    else:
                        ops.sokoban_step_turn(st, env.ep, turn)
                if not fused:
                    seg = torch.arange(0, B + 1, gs, dtype=torch.int32, device=device)
                    ops.rollout_finalize(env.ep, seg, method, norm, met, sc, pe)
                torch.cuda.synchronize()
                outs.append((env.room_state.clone(), env.ep.arena.clone(), norm, torch.nan_to_num(met, 9.0), sc, pe))
            for a, b in zip(*outs):
                assert torch.equal(a, b), (gs, method)


def test_frozenlake_restore(device):
    """rmi_frozenlake_reset == the post-reset state: desc, start state, PCG64 state, zeroed record;
    a rollout replayed after it is identical."""
    B, T, K = 1000, 4, 5
    fl = FrozenLakeBatch(FrozenLakeEnvConfig(), B, T, K, device)
    fl.reset(synthetic.env_seeds(B))
    snap = [x.clone() for x in (fl.desc, fl.s, fl.rng)]
    ids, n = synthetic.rollout_actions(B, T, K, 1, 4, seed=5)
    outs = []
    for rep in range(2):
        fl.restore()
        assert all(torch.equal(a, b) for a, b in zip((fl.desc, fl.s, fl.rng), snap))
        assert int(fl.ep.arena.count_nonzero()) == 0
        for t in range(T):
            fl.step_turn(t, _t(ids[t], device), _t(n[t], device), None, 10, -0.1)
        outs.append((fl.s.clone(), fl.rng.clone(), fl.ep.arena.clone()))
    assert all(torch.equal(a, b) for a, b in zip(*outs))


@pytest.mark.parametrize("B", [1000, 8192])
def test_bilevel_vs_oracle_large(device, B):
    """Bi-level GAE at SK-like shapes vs the C oracle: returns and pre-whitening advantages
    bit-exact, the IndexError rows identical; turn rewards with zeros, negative and NaN-free
    values, rows ending in mask-0 and in mask-1 without reward, ragged L % 4."""
    rng = np.random.default_rng(B)
    n_turns = rng.integers(1, 6, B).astype(np.int32)
    tr = rng.choice([0.0, 0.5, -1.1, 10.9], size=(B, 5), p=[0.2, 0.4, 0.2, 0.2]).astype(np.float32)
    r, v, m = synthetic.token_rows(n_turns, rng.standard_normal(B).astype(np.float32), seed=B, turn_scores=tr)
    pad = 1 if (r.shape[1] + 1) % 4 else 2  # trailing mask-0 columns, L % 4 != 0
    r, v, m = (np.pad(x, ((0, 0), (0, pad))) for x in (r, v, m))
    rd, vd, md = _t(r, device), _t(v, device), _t(m, device)
    for g, lam, hg in ((1.0, 1.0, 0.95), (0.99, 0.95, 0.9)):
        oa, oret, oerr = oracle.bilevel_gae(r, v, m, g, lam, hg)
        assert 0 < int((oerr != 0).sum()) < B  # rows whose last turn scored 0 raise IndexError
        adv, ret = ops.bilevel_gae(rd, vd, md, g, lam, hg, check_errors=False)
        ok = oerr == 0  # rows the reference completes
        np.testing.assert_array_equal(ret.cpu().numpy()[ok], oret[ok])
        np.testing.assert_array_equal(adv.cpu().numpy()[ok], oa[ok])
        stats = torch.empty(B, 3, dtype=torch.float64, device=device)
        errs = torch.empty(B, dtype=torch.uint8, device=device)
        check = ops.lib().rmi_bilevel_gae(ops._ptr(rd), ops._ptr(vd), ops._ptr(md), B, r.shape[1], g, lam, hg,
                                          ops._ptr(adv), ops._ptr(ret), ops._ptr(stats), ops._ptr(errs),
                                          ops._stream(device))
        assert check == 0
        np.testing.assert_array_equal(errs.cpu().numpy() != 0, oerr != 0)
        s1 = (oa.astype(np.float64) * m).sum(1)
        np.testing.assert_allclose(stats[:, 0].cpu().numpy()[ok], s1[ok], rtol=1e-12, atol=1e-9)
        np.testing.assert_array_equal(stats[:, 2].cpu().numpy(), m.sum(1).astype(np.float64))


@pytest.mark.parametrize("B,L,p_eos,p_valid", [
    (512, 700, 0.05, 0.6),   # ~20 segments per row: the segment-parallel walk
    (512, 700, 0.4, 0.7),    # > 64 segment starts in most rows: the serial fallback walk
    (300, 257, 0.02, 0.3),   # few segments, many rows without any (a tail segment: IndexError rows)
    (64, 9001, 0.01, 0.5),   # a row too long for the LDS row buffer: bilevel_tiled_kernel
])
def test_bilevel_segment_walks_vs_oracle(device, monkeypatch, B, L, p_eos, p_valid):
    """rmi_bilevel_gae's segment-parallel kernel and its tiled kernel (RAGEN_AMD_BILEVEL_TILED=1)
    both equal the oracle bit for bit on rows the reference completes: rewards (eos) at random
    columns inside and outside the mask, NaN-free, negative and -0.0 rewards among them."""
    rng = np.random.default_rng(L)
    r = np.where(rng.random((B, L)) < p_eos, rng.choice([0.5, -1.25, 3.0, -0.0], size=(B, L)), 0.0).astype(np.float32)
    m = (rng.random((B, L)) < p_valid).astype(np.uint8)
    v = rng.standard_normal((B, L)).astype(np.float32)
    last = L - 1 - np.argmax(m[:, ::-1], axis=1)  # each row's last valid column: a turn end in 80 % of rows
    pick = (rng.random(B) < 0.8) & (m.sum(1) > 0)
    r[np.nonzero(pick)[0], last[pick]] = 1.5
    rd, vd, md = _t(r, device), _t(v, device), _t(m, device)
    for g, lam, hg in ((1.0, 1.0, 0.95), (0.99, 0.95, 0.9)):
        oa, oret, oerr = oracle.bilevel_gae(r, v, m, g, lam, hg)
        ok = oerr == 0
        assert 0 < ok.sum() < B
        for tiled in ("0", "1"):
            monkeypatch.setenv("RAGEN_AMD_BILEVEL_TILED", tiled)
            adv, ret = ops.bilevel_gae(rd, vd, md, g, lam, hg, check_errors=False)
            np.testing.assert_array_equal(ret.cpu().numpy()[ok], oret[ok])
            np.testing.assert_array_equal(adv.cpu().numpy()[ok], oa[ok])
            stats = torch.empty(B, 3, dtype=torch.float64, device=device)
            errs = torch.empty(B, dtype=torch.uint8, device=device)
            assert ops.lib().rmi_bilevel_gae(ops._ptr(rd), ops._ptr(vd), ops._ptr(md), B, L, g, lam, hg, ops._ptr(adv),
                                             ops._ptr(ret), ops._ptr(stats), ops._ptr(errs), ops._stream(device)) == 0
            np.testing.assert_array_equal(errs.cpu().numpy() != 0, oerr != 0)
            np.testing.assert_array_equal(stats[:, 2].cpu().numpy(), m.sum(1).astype(np.float64))
            s1 = (oa.astype(np.float64) * m).sum(1)
            np.testing.assert_allclose(stats[:, 0].cpu().numpy()[ok], s1[ok], rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("B,frac_irregular,partial", [(8192, 0.0, False), (1000, 0.0, True), (2050, 0.3, False),
                                                       (16500, 0.3, True)])
def test_fused_first_turn(device, B, frac_irregular, partial):
    """rmi_sokoban_step_turn_first == rmi_sokoban_reset + rmi_sokoban_step_turn, bit for bit:
    rows, players, counters, the whole episode record and the error bits, starting from a
    dirty (mid-rollout) state; both lane layouts, irregular rooms, envs without input."""
    rng = np.random.default_rng(B + int(partial))
    T, K, H, W = 4, 6, 6, 6
    cfg = SokobanEnvConfig(dim_x=H, dim_y=W, num_boxes=1, max_steps=12)
    env0 = SokobanBatch(cfg, B, T, K, device)
    env0.reset(synthetic.env_seeds(B))
    fixed = env0.room_fixed.cpu().numpy().copy()
    state = env0.init_state.cpu().numpy().copy()
    player = env0.init_player.cpu().numpy().copy()
    idx = np.nonzero(rng.random(B) < frac_irregular)[0]
    f2, s2, p2 = fixed[idx].copy(), state[idx].copy(), player[idx].copy()
    _irregular_rooms(rng, len(idx), H, W, f2, s2, p2)
    fixed[idx], state[idx], player[idx] = f2, s2, p2
    turns = []
    for t in range(3):
        ids = rng.choice([0, 1, 2, 3, 4, 5, 6, 7, 8, 9], size=(B, K), p=[0.05] + [0.11] * 8 + [0.07]).astype(np.int8)
        n = rng.integers(0, K + 1, size=B).astype(np.uint8)
        turns.append((_t(ids, device), _t(n, device)))
    has = _t((rng.random(B) < 0.7).astype(np.uint8), device) if partial else None
    outs = []
    for fused in (False, True):
        env = SokobanBatch(cfg, B, T, K, device)
        env.load_state(fixed, state, player)
        for t in (0, 1):  # dirty the state and the record
            env.step_turn(t, turns[t][0], turns[t][1], None, 9, -0.1)
        err = torch.zeros(B, dtype=torch.uint8, device=device)
        turn = ops.turn_struct(0, turns[2][0], turns[2][1], has, 9, -0.1)
        if fused:
            ops.sokoban_step_turn_first(env.struct(), env.ep, turn, env.init_state, env.init_player, err)
        else:
            env.restore()
            ops.sokoban_step_turn(env.struct(), env.ep, turn, err)
        torch.cuda.synchronize()
        outs.append((env.room_state.clone(), env.player.clone(), env.num_env_steps.clone(),
                     env.boxes_on_target.clone(), env.ep.arena.clone(), err))
    for name, a, b in zip(("room_state", "player", "nes", "bot", "episode", "err"), *outs):
        assert torch.equal(a, b), name


@pytest.mark.parametrize("B,partial", [(4096, False), (1000, True)])
def test_frozenlake_fused_first_turn(device, B, partial):
    """rmi_frozenlake_step_turn_first == rmi_frozenlake_reset + rmi_frozenlake_step_turn, bit for
    bit (desc, s, the PCG64 state, the whole record, error bits), from a dirty state."""
    rng = np.random.default_rng(B)
    T, K = 4, 5
    ids, n = synthetic.rollout_actions(B, 3, K, 1, 4, seed=B)
    has = _t((rng.random(B) < 0.6).astype(np.uint8), device) if partial else None
    outs = []
    for fused in (False, True):
        fl = FrozenLakeBatch(FrozenLakeEnvConfig(), B, T, K, device)
        fl.reset(synthetic.env_seeds(B))
        for t in (0, 1):
            fl.step_turn(t, _t(ids[t], device), _t(n[t], device), None, 10, -0.1)
        err = torch.zeros(B, dtype=torch.uint8, device=device)
        turn = ops.turn_struct(0, _t(ids[2], device), _t(n[2], device), has, 10, -0.1)
        if fused:
            ops.frozenlake_step_turn_first(fl.struct(), fl.ep, turn, fl.init_desc, fl.init_s, fl.init_rng, err)
        else:
            fl.restore()
            ops.frozenlake_step_turn(fl.struct(), fl.ep, turn, err)
        torch.cuda.synchronize()
        outs.append((fl.desc.clone(), fl.s.clone(), fl.rng.clone(), fl.ep.arena.clone(), err))
    for name, a, b in zip(("desc", "s", "rng", "episode", "err"), *outs):
        assert torch.equal(a, b), name


@pytest.mark.parametrize("B,T", [(4096, 8), (1024, 5)])
def test_frozenlake_fused_last_turn_finalize(device, B, T):
    """rmi_frozenlake_step_turn_finalize == rmi_frozenlake_step_turn + rmi_rollout_finalize, bit for
    bit (groups inside the wave, and the two-launch fallback for groups of 128)."""
    K = 5
    ids, n = synthetic.rollout_actions(B, T, K, 1, 4, seed=31)
    ids, n = _t(ids, device), _t(n, device)
    for gs in (16, 4, 64, 128):
        for method in ("identity", "mean", "mean_std", "asym_clip"):
            outs = []
            for fused in (False, True):
                fl = FrozenLakeBatch(FrozenLakeEnvConfig(), B, T, K, device)
                fl.reset(synthetic.env_seeds(B))
                st = fl.struct()
                norm = torch.full((B,), 7.0, dtype=torch.float32, device=device)
                met = torch.full((B, 4), 7.0, dtype=torch.float64, device=device)
                sc = torch.full((B,), 7.0, dtype=torch.float32, device=device)
                pe = torch.full((B,), 7.0, dtype=torch.float32, device=device)
                last = T - 2
                for t in range(last + 1):
                    turn = ops.turn_struct(t, ids[t], n[t], None, 10, -0.1)
                    if fused and t == last:
                        ops.frozenlake_step_turn_finalize(st, fl.ep, turn,
                                                          ops.finalize_struct(gs, method, norm, met, sc, pe))
                    else:
                        ops.frozenlake_step_turn(st, fl.ep, turn)
                if not fused:
                    seg = torch.arange(0, B + 1, gs, dtype=torch.int32, device=device)
                    ops.rollout_finalize(fl.ep, seg, method, norm, met, sc, pe)
                torch.cuda.synchronize()
                outs.append((fl.s.clone(), fl.rng.clone(), fl.ep.arena.clone(), norm, torch.nan_to_num(met, 9.0),
                             sc, pe))
            for a, b in zip(*outs):
                assert torch.equal(a, b), (gs, method)


def test_pcg64_seed_matches_numpy(device):
    """rmi_pcg64_seed == numpy Generator(PCG64(SeedSequence(seed))) after `draws` random()
    calls (gymnasium seeding.np_random as BanditEnv / FrozenLakeEnv reset it), for seeds across
    the one-word / two-word entropy boundary and the 63-bit maximum."""
    rs = np.random.default_rng(5)
    seeds = np.concatenate([np.arange(0, 70), [2**32 - 1, 2**32, 2**32 + 1, 2**40 + 7, 2**63 - 1, 123, 1000000],
                            rs.integers(0, 2**63 - 1, 200, dtype=np.int64)]).astype(np.int64)
    for draws in (0, 1, 3):
        rng, last = ops.pcg64_seed(_t(seeds, device), draws)
        rng = rng.cpu().numpy().view(np.uint64)
        last = last.cpu().numpy()
        for i, sd in enumerate(seeds):
            g = np.random.Generator(np.random.PCG64(np.random.SeedSequence(int(sd))))
            u = 0.0
            for _ in range(draws):
                u = g.random()
            st = g.bit_generator.state["state"]
            got = (int(rng[0, i]) << 64 | int(rng[1, i]), int(rng[2, i]) << 64 | int(rng[3, i]))
            assert got == (st["state"], st["inc"]), (sd, draws)
            assert last[i] == u, (sd, draws)
    with pytest.raises(ValueError):
        ops.pcg64_seed(_t(np.array([3, -1], np.int64), device), 1)


NAME_CASES = [  # (answer, modelled); every answer's digit runs are exactly {12, 3}, so the
    # format check passes and the evaluation decides (0.1 = not correct, 1 = correct)
    ("x + 12 + 3", True), ("abs(12) + 3", True), ("a + 12 - 3", True), ("12 + x * 3", True), ("_ + 12 + 3", True),
    ("print(12, 3)", True), ("12 3 foo", True), ("(x) - 12 + 3", True), ("12+3 # x", True),
    ("match + 12 + 3", True),
    ("12if x else 3", False), ("(x := 12) + 3", False), ("True + 12 + 3", False), ("3 < 12 < x", False),
    ("x.real + 12 + 3", False), ("(12).real + 3", False), ("lambda: 12 + 3", False), ("12 if x else 3", False),
    ("not x + 12 + 3", False), ("x or 12 + 3", False), ("12 + 3j", False), ("\u210c + 12 + 3", False),
]


def test_countdown_bare_names(device):
    """countdown/env.py:16-21 evaluates under {"__builtins__": None}, where every name lookup
    raises: answers whose only non-arithmetic tokens are plain names are 'not correct' and
    are modelled (format_score or 0, no error flag); answers where a keyword, ':', '.', a
    comparison, a quote or a fused literal could bind or skip a name stay flagged."""
    n = len(NAME_CASES)
    data = [{"nums": [12, 3], "target": 15}] * n
    env = CountdownBatch(CountdownEnvConfig(data=data), n, 1, 1, device)
    env.reset(np.zeros(n, dtype=np.int64))
    buf, lens = env.encode_answers([[e] for e, _ in NAME_CASES])
    r, fl, err = ops.countdown_reward(env.struct(), _t(buf[:, 0], device), _t(lens[:, 0].copy(), device))
    r, err = r.cpu().numpy(), err.cpu().numpy()
    for i, (e, modelled) in enumerate(NAME_CASES):
        want = oracle.countdown_reward(e, [12, 3], 15)
        if modelled:
            assert err[i] == 0 and r[i] == want, (e, r[i], want, err[i])
        else:
            assert err[i] & _lib.ERR_UNSUP, (e, err[i])


@pytest.mark.parametrize("slippery,bad_waves", [(True, 0.0), (False, 0.0), (True, 0.3)])
def test_frozenlake_fast_and_generic_paths_vs_oracle(device, slippery, bad_waves):
    """The 4x4 straight-line turn (waves whose ids are all 0..4) and the generic turn (waves with
    an out-of-range id somewhere) against the oracle, slippery and not, K = 8 / 3 / 5."""
    B, T = 8192, 6
    rng = np.random.default_rng(int(slippery) * 10 + int(bad_waves * 10))
    for K in (8, 3, 5):
        env = FrozenLakeBatch(FrozenLakeEnvConfig(is_slippery=slippery), B, T, K, device)
        env.reset(synthetic.env_seeds(B, 2000 + K))
        desc = env.desc.cpu().numpy()
        s = env.s.cpu().numpy()
        st = env.rng.cpu().numpy().view(np.uint64).copy()
        oep = oracle.Episode(B, T)
        bad = np.zeros(B, bool)
        for t in range(T):
            ids = rng.integers(0, 5, size=(B, K)).astype(np.int8)
            n = rng.integers(0, K + 1, size=B).astype(np.uint8)
            waves = rng.random(B // 64) < bad_waves
            for w in np.nonzero(waves)[0]:
                ids[w * 64 + int(rng.integers(0, 64)), int(rng.integers(0, K))] = int(rng.choice([5, 9, -1]))
            err = torch.zeros(B, dtype=torch.uint8, device=device)
            env.step_turn(t, _t(ids, device), _t(n, device), None, 9, -0.1, err)
            oerr = oracle.frozenlake_turn(4, 4, slippery, env.cs, desc, s, st, oep, t, ids, n, None, 9, -0.1)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(err.cpu().numpy() != 0, oerr != 0)
            bad |= oerr != 0
            ok = ~bad
            np.testing.assert_array_equal(env.s.cpu().numpy()[ok], s[ok])
            np.testing.assert_array_equal(env.rng.cpu().numpy().view(np.uint64)[:, ok], st[:, ok])
            h = _host_ep(env.ep)
            for k in ("num_actions", "flags", "n_turns", "penalty"):
                np.testing.assert_array_equal(h[k][ok], getattr(oep, k)[ok], err_msg=f"K={K} t={t} {k}")
            for k in ("turn_reward", "turn_info", "turn_exec"):
                np.testing.assert_array_equal(h[k][:, ok], getattr(oep, k)[:, ok], err_msg=f"K={K} t={t} {k}")


@pytest.mark.parametrize("kind", ["gae", "bilevel_seg", "bilevel_tiled"])
def test_streamed_launches_vs_oracle(device, monkeypatch, kind):
    """Launches whose traffic passes 256 MiB (8192 x 2112 tokens, 294 MB) take the nontemporal
    load / store forms of the GAE and bi-level kernels (advantage.hip, kStreamBytes): the same
    results as the oracle, bit for bit."""
    B, L = 8192, 2112
    rng = np.random.default_rng(77)
    n_turns = rng.integers(1, 6, B).astype(np.int32)
    tr = rng.choice([0.5, -1.1, 10.9], size=(B, 5)).astype(np.float32)
    r, v, m = synthetic.token_rows(n_turns, rng.standard_normal(B).astype(np.float32), seed=5, turn_scores=tr,
                                   max_len=L)
    assert r.shape[1] * B * 17 > 256 * 1024 * 1024
    rd, vd, md = _t(r, device), _t(v, device), _t(m, device)
    if kind == "gae":
        for variant, (g, lam) in (("legacy", (1.0, 1.0)), ("masked", (0.99, 0.95))):
            adv, ret = ops.gae(rd, vd, md, g, lam, variant)
            oadv, oret = oracle.gae(r, v, m, g, lam, variant)
            np.testing.assert_array_equal(ret.cpu().numpy(), oret)
            np.testing.assert_array_equal(adv.cpu().numpy(), oadv)
        return
    if kind == "bilevel_tiled":
        monkeypatch.setenv("RAGEN_AMD_BILEVEL_TILED", "1")
    oa, oret, oerr = oracle.bilevel_gae(r, v, m, 0.99, 0.95, 0.9)
    adv, ret = ops.bilevel_gae(rd, vd, md, 0.99, 0.95, 0.9, check_errors=False)
    ok = oerr == 0
    np.testing.assert_array_equal(ret.cpu().numpy()[ok], oret[ok])
    np.testing.assert_array_equal(adv.cpu().numpy()[ok], oa[ok])
