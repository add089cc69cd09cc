"""Pin the CPU oracle (oracle/) against golden vectors recorded from the reference itself.

CPU-only (no GPU): these tests establish that the oracle the GPU parity tests compare
against reproduces the reference's outputs on the reference's own code paths.
"""
import numpy as np
import pytest
import torch

import oracle
from trace_util import load, strings, trace_inputs


def replay_sokoban(name):
    d, ids = trace_inputs(name)
    B, T = int(d["B"]), int(d["T"])
    H = W = int(np.sqrt(d["init_room_state"].shape[1]))
    num_boxes = 1 if H == 6 else 2
    fixed = d["init_room_fixed"].astype(np.uint8).copy()
    state = d["init_room_state"].astype(np.uint8).copy()
    player = d["init_player"].astype(np.int8).copy()
    nes = np.zeros(B, np.int32)
    bot = np.zeros(B, np.int32)
    ep = oracle.Episode(B, T)
    for t in range(T):
        err = oracle.sokoban_turn(H, W, num_boxes, 100, fixed, state, player, nes, bot, ep, t, ids[t], d["n_act"][t],
                                  d["act_in"][t], 10, -0.1)
        assert not err.any()
        np.testing.assert_array_equal(state, d["turn_room_state"][t].astype(np.uint8))
        np.testing.assert_array_equal(player, d["turn_player"][t].astype(np.int8))
        np.testing.assert_array_equal(nes, d["turn_num_env_steps"][t])
        np.testing.assert_array_equal(bot, d["turn_boxes_on_target"][t])
        check_episode_turn(ep, d, t)
    check_final(ep, d)


def check_episode_turn(ep, d, t):
    np.testing.assert_array_equal(ep.turn_reward[t], d["turn_reward"][t])  # bit-exact f64
    np.testing.assert_array_equal(ep.turn_exec[t], d["n_exec"][t])
    np.testing.assert_array_equal(ep.turn_info[t], d["info"][t])
    np.testing.assert_array_equal(ep.penalty, d["penalty"][t])
    np.testing.assert_array_equal(ep.num_actions, d["num_actions"][t])
    np.testing.assert_array_equal((ep.flags & oracle.FLAG_TERM) > 0, d["term"][t] > 0)
    np.testing.assert_array_equal((ep.flags & oracle.FLAG_TRUNC) > 0, d["trunc"][t] > 0)
    active = (d["act_in"][t] > 0) & ((ep.flags & oracle.FLAG_DONE) == 0)
    np.testing.assert_array_equal(active, d["active_after"][t] > 0)


def check_final(ep, d):
    m = oracle.rollout_metrics(ep)
    for j, k in enumerate(["success", "num_actions", "action_is_effective", "action_is_valid"]):
        np.testing.assert_array_equal(m[:, j], d["metric_" + k])
    s, p = oracle.trajectory_scores(ep)
    np.testing.assert_array_equal(s, d["score_f32"])
    np.testing.assert_array_equal(p, d["penalty_f32"])


def test_sokoban_trace():
    replay_sokoban("sokoban_es")


def test_sokoban8_trace():
    replay_sokoban("sokoban8_es")


def test_frozenlake_trace():
    d, ids = trace_inputs("frozenlake_es")
    B, T = int(d["B"]), int(d["T"])
    desc = d["init_desc"].astype(np.uint8).copy()
    s = d["init_s"].astype(np.int32).copy()
    rng = np.ascontiguousarray(d["init_rng_state"].T).astype(np.uint64)  # [4,B]
    ep = oracle.Episode(B, T)
    cs = tuple(np.cumsum([(1 - 1 / 3) / 2, 1 / 3, (1 - 1 / 3) / 2]).tolist())
    for t in range(T):
        err = oracle.frozenlake_turn(4, 4, True, cs, desc, s, rng, ep, t, ids[t], d["n_act"][t], d["act_in"][t], 10,
                                     -0.1)
        assert not err.any()
        np.testing.assert_array_equal(s, d["turn_s"][t])
        np.testing.assert_array_equal(rng.T, d["turn_rng_state"][t])
        check_episode_turn(ep, d, t)
    check_final(ep, d)


def test_bandit_trace():
    d, ids = trace_inputs("bandit_es")
    B, T = int(d["B"]), int(d["T"])
    rng = np.ascontiguousarray(d["init_rng_state"].T).astype(np.uint64)
    ep = oracle.Episode(B, T)
    hi = d["init_hi_is_first"].astype(np.uint8)
    for t in range(T):
        oracle.bandit_turn(1, 0.1, 0.0, 1.0, 0.25, hi, rng, ep, t, ids[t], d["n_act"][t], d["act_in"][t], 1, -0.1)
        np.testing.assert_array_equal(rng.T, d["turn_rng_state"][t])
        check_episode_turn(ep, d, t)
    check_final(ep, d)


def test_bandit_kat():
    """bandit/env.py:87-104 self-check: seeds 500..1499, action 1."""
    k = strings()["bandit_kat"]
    seeds = np.arange(*k["seeds"])
    B = len(seeds)
    st = []
    hi = []
    for s in seeds:
        g = np.random.Generator(np.random.PCG64(np.random.SeedSequence(int(s))))
        hi.append(0 if g.random() < 0.5 else 1)
        x = g.bit_generator.state["state"]
        st.append([x["state"] >> 64, x["state"] & (2**64 - 1), x["inc"] >> 64, x["inc"] & (2**64 - 1)])
    np.testing.assert_array_equal(hi, k["hi_is_first"])
    rng = np.ascontiguousarray(np.array(st, np.uint64).T)
    ep = oracle.Episode(B, 1)
    oracle.bandit_turn(1, 0.1, 0.0, 1.0, 0.25, np.array(hi, np.uint8), rng, ep, 0, np.ones((B, 1), np.int8),
                       np.ones(B, np.uint8))
    np.testing.assert_array_equal(ep.turn_reward[0], k["rewards"])
    assert abs(ep.turn_reward[0].mean() - 0.175) < 1e-12 and abs(k["mean"] - 0.175) < 1e-12


def test_pcg64_matches_numpy():
    for seed in (0, 1, 123, 2**31 + 7, 99999):
        g = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))
        x = g.bit_generator.state["state"]
        st = np.array([x["state"] >> 64, x["state"] & (2**64 - 1), x["inc"] >> 64, x["inc"] & (2**64 - 1)],
                      np.uint64)
        for _ in range(20):
            u, st = oracle.pcg64_random(st)
            assert u == g.random()


def test_countdown_kat():
    k = strings()["countdown_kat"]
    for c in k["cases"]:
        assert oracle.countdown_reward(c["expr"], k["nums"], k["target"]) == c["reward"], c


def test_countdown_trace():
    """oracle.countdown_turn (es_manager.py:149-169 over countdown/env.py:58-62) replays the
    reference-run 64 x 4 trace: rewards, penalties, caps, flags, metrics and scores."""
    d = load("countdown_es")
    S = strings()
    B, T = int(d["B"]), int(d["T"])
    answers = S["countdown_es"]["answers"]
    nums = [list(d["init_nums"][b, :d["init_n_nums"][b]]) for b in range(B)]
    ep = oracle.Episode(B, T)
    for t in range(T):
        lists = [[a] if a is not None else [] for a in answers[t]]
        oracle.countdown_turn(lists, nums, d["init_target"], ep, t, d["act_in"][t], 1, -0.1)
        check_episode_turn(ep, d, t)
    check_final(ep, d)


def test_normalize_golden():
    d = load("normalize")
    B = len(d["scores"])
    pen32 = d["penalty"].astype(np.float32)
    segs = {"state": np.arange(0, B + 1, 16), "inductive": np.array([0, 48, 96]), "batch": np.array([0, B])}
    for grouping, seg in segs.items():
        for method in ("mean_std", "mean", "asym_clip", "identity"):
            out = oracle.group_normalize(d["scores"], pen32, seg, method)
            np.testing.assert_allclose(out, d[f"norm_{grouping}_{method}"], rtol=0, atol=1e-5)


def test_gae_golden():
    d = load("gae")
    m = d["mask"]
    for gl in ("g1.0_l1.0", "g1.0_l0.95", "g0.99_l0.95"):
        g, lam = (float(x[1:]) for x in gl.split("_"))
        for rn in ("last", "turn"):
            r = d["rew"] if rn == "last" else d["rew_turn"]
            for var, key in (("legacy", "gae"), ("masked", "gaem")):
                adv, ret = oracle.gae(r, d["values"], m, g, lam, var)
                np.testing.assert_array_equal(ret, d[f"{key}_{rn}_{gl}_ret"])  # returns: bit-exact
                w = oracle.masked_whiten(adv, m)
                np.testing.assert_allclose(w, d[f"{key}_{rn}_{gl}_adv"], rtol=0, atol=1e-5)
            adv, ret, err = oracle.bilevel_gae(r, d["values"], m, g, lam, 0.95)
            assert not err.any()
            np.testing.assert_array_equal(ret, d[f"bilevel_{rn}_{gl}_ret"])
            w = oracle.masked_whiten(adv, m)
            np.testing.assert_allclose(w, d[f"bilevel_{rn}_{gl}_adv"], rtol=0, atol=1e-5)


def test_bilevel_main_example_and_error():
    d = load("gae")
    r = np.array([[0, 0, 0, 0, 1, 0, 0, 0, 0, 1]], np.float32)
    v = np.array([[0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7, 0.8, 0.9, 1.0]], np.float32)
    m = np.ones((1, 10), np.uint8)
    adv, ret, err = oracle.bilevel_gae(r, v, m, 1.0, 1.0, 0.95)
    np.testing.assert_array_equal(ret, d["main_example_ret"])
    np.testing.assert_allclose(oracle.masked_whiten(adv, m), d["main_example_adv"], atol=1e-6)
    _, _, err = oracle.bilevel_gae(np.array([[0, 1, 0, 0]], np.float32), np.zeros((1, 4), np.float32),
                                   np.ones((1, 4), np.uint8), 1.0, 1.0, 0.95)
    assert err[0] and int(d["bilevel_zero_last_raises"]) == 1


def test_compute_advantage_golden():
    d = load("gae")
    m = d["mask"]
    B = m.shape[0]
    adv, ret = oracle.grpo(d["rew_turn"], m, np.arange(B + 1))
    np.testing.assert_allclose(adv, d["ca_grpo_0_adv"], rtol=1e-6, atol=1e-6)
    adv, ret = oracle.grpo(d["rew_turn"], m, np.arange(0, B + 1, 4))
    np.testing.assert_allclose(adv, d["grpo_g4_adv"], rtol=1e-5, atol=1e-5)
    adv, ret = oracle.gae(d["rew_turn"], d["values"], m, 1.0, 0.95)
    np.testing.assert_array_equal(ret, d["ca_gae_0_ret"])
    np.testing.assert_allclose(oracle.masked_whiten(adv, m), d["ca_gae_0_adv"], atol=1e-5)
    adv, ret, _ = oracle.bilevel_gae(d["rew_turn"], d["values"], m, 1.0, 0.95, 0.95)
    np.testing.assert_array_equal(ret, d["ca_gae_1_ret"])


def test_filter_golden():
    d = load("filter")
    for key in ("r0.25_std", "r0.25_std_rev", "r1.0_std", "r0.5_std"):
        ratio = float(key.split("_")[0][1:])
        ftype = key.split("_", 1)[1]
        sc = d[key + "_scores"]
        rows = torch.from_numpy(sc).sum(-1).numpy()
        keep, met, (sd, mx, mn) = oracle.filter_groups(rows, 64, 16, ratio, ftype)
        names = ["in_group_std", "in_group_max", "in_group_mean", "chosen_in_group_std", "chosen_in_group_max",
                 "chosen_in_group_mean"]
        ref = [float(d[f"{key}_rollout__{n}"]) for n in names]
        # tie-invariant parts match the reference: the per-group stats, the chosen std mean and
        # the multiset of selected std values
        np.testing.assert_allclose(met[:4], ref[:4], rtol=1e-6, atol=1e-6)
        kept = np.unique(d[key + "_kept_env_ids"] // 16)
        np.testing.assert_array_equal(np.sort(sd[keep > 0]), np.sort(sd[kept]))
        # documented deviation: torch.topk's choice among tied std values is
        # implementation-defined; we pick ties by ascending group index.  chosen max/mean then
        # match the reference exactly whenever the k-th and (k+1)-th std differ.
        order = np.lexsort((np.arange(64), -sd if ftype == "std" else sd))
        np.testing.assert_array_equal(np.nonzero(keep)[0], np.sort(order[:int(keep.sum())]))
        np.testing.assert_allclose(met[4:], [mx[keep > 0].mean(), mn[keep > 0].mean()], rtol=1e-6)
        k = int(keep.sum())
        if k == 64 or sd[order[k - 1]] != sd[order[k]]:
            np.testing.assert_allclose(met[4:], ref[4:], rtol=1e-6, atol=1e-6)


def test_host_sokoban_generator_golden():
    """The product's host-side C++ generator (exact CPython/numpy MT19937 streams) vs the
    rooms generate_room produced in the reference (sokoban/utils.py:221-278)."""
    from ragen_amd import ops
    d = load("sokoban_rooms")
    for tag, (H, nb, sd) in {"SimpleSokoban": (6, 1, 300), "LargerSokoban": (8, 2, 10)}.items():
        seeds = d[tag + "_seeds"]
        fixed, state, player, status = ops.generate_sokoban_rooms(seeds, H, H, nb, sd)
        bad = np.nonzero(status)[0]
        if len(bad):  # the reference reseeded these with abs(hash(str(seed))) % 2**32
            f2, s2, p2, st2 = ops.generate_sokoban_rooms(d[tag + "_reseed"][bad], H, H, nb, sd)
            assert not st2.any()
            fixed[bad], state[bad], player[bad] = f2, s2, p2
        np.testing.assert_array_equal(fixed, d[tag + "_fixed"].astype(np.uint8))
        np.testing.assert_array_equal(state, d[tag + "_state"].astype(np.uint8))
        np.testing.assert_array_equal(player, d[tag + "_player"].astype(np.int8))
    assert set(d["SimpleSokoban_seeds"][np.nonzero(ops.generate_sokoban_rooms(
        d["SimpleSokoban_seeds"], 6, 6, 1, 300)[3])[0]]) == {3248, 3701}


def test_masks_and_scores_golden():
    """oracle.masks_and_scores == get_masks_and_scores run by the reference (Qwen ids, roll)."""
    d = load("masks_scores")
    lens = d["scores_len"]
    flat = d["scores_flat"]
    B = len(lens)
    T = int(lens.max())
    tab = np.zeros((T, B), np.float64)
    o = 0
    for b, n in enumerate(lens):
        tab[:n, b] = flat[o:o + n]
        o += n
    for uts in (False, True):
        for erm in (False, True):
            sc, lm, rm, err = oracle.masks_and_scores(d["input_ids"], 151644, 151645, tab, lens, T, uts, erm, True)
            key = f"uts{int(uts)}_erm{int(erm)}"
            np.testing.assert_array_equal(sc, d[key + "_score"])
            np.testing.assert_array_equal(lm, d[key + "_loss_mask"])
            np.testing.assert_array_equal(rm, d[key + "_response_mask"])
            assert not err.any()


def test_masks_and_scores_llama3_golden():
    """The Llama-3 branch (ctx_manager.py:27-29: ids 128006 / 128009, and no roll at :60-62):
    oracle.masks_and_scores with roll off == get_masks_and_scores run by the reference on
    Llama-3 chat rows (tests/golden/make_golden_llama.py), both score placements and both mask
    modes; rows with fewer turns than the batch keep zip_longest's fill 0 on their own last
    column, which the roll would have carried off.  The facade's get_special_tokens takes the
    same branch."""
    from fake_tok import FakeLlama3Tok
    from ragen_amd.llm_agent.ctx_manager import get_special_tokens
    d = load("masks_scores_llama")
    sp, rt = (int(x) for x in d["special"])
    assert get_special_tokens(FakeLlama3Tok()) == (sp, rt) == (128006, 128009)
    lens, flat = d["scores_len"], d["scores_flat"]
    B, T = len(lens), int(lens.max())
    tab = np.zeros((T, B), np.float64)
    o = 0
    for b, n in enumerate(lens):
        tab[:n, b] = flat[o:o + n]
        o += n
    for uts in (False, True):
        for erm in (False, True):
            sc, lm, rm, err = oracle.masks_and_scores(d["input_ids"], sp, rt, tab, lens, T, uts, erm, False)
            key = f"uts{int(uts)}_erm{int(erm)}"
            np.testing.assert_array_equal(sc, d[key + "_score"])
            np.testing.assert_array_equal(lm, d[key + "_loss_mask"])
            np.testing.assert_array_equal(rm, d[key + "_response_mask"])
            assert not err.any()
    # the fixture holds the case the roll hides: a shorter row whose last turn's score was overwritten
    last = d["uts1_erm0_score"][:, -1]
    ends_on_eot = d["input_ids"][:, -1] == rt
    assert ((lens < T) & ends_on_eot & (last == 0)).any()
