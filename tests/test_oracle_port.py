"""The timed CPU baseline (oracle/port.py) computes what the pinned C oracle computes."""
import numpy as np

import oracle
from oracle import port
from ragen_amd import ops, synthetic


def test_port_matches_c_oracle():
    B, T, K = 256, 5, 5
    seeds = synthetic.env_seeds(B)
    uniq, inv = np.unique(seeds, return_inverse=True)
    f, s, p, st = ops.generate_sokoban_rooms(uniq, 6, 6, 1, 300)
    assert not st.any()
    fixed, state, player = f[inv], s[inv], p[inv]
    ids, n = synthetic.rollout_actions(B, T, K, 1, 4)
    envs = port.make_sokoban_envs(fixed, state, player)
    steps = port.sokoban_rollout(envs, ids, n, 10)
    ep = oracle.Episode(B, T)
    st_ = state.copy()
    pl = player.copy()
    nes = np.zeros(B, np.int32)
    bot = np.zeros(B, np.int32)
    for t in range(T):
        oracle.sokoban_turn(6, 6, 1, 100, fixed, st_, pl, nes, bot, ep, t, ids[t], n[t])
    assert steps == int(ep.turn_exec.sum()) == int(nes.sum())
    for i, e in enumerate(envs):
        np.testing.assert_array_equal(e["env"].room_state.ravel(), st_[i])
        assert e["status"]["num_actions"] == ep.num_actions[i]
        assert np.float64(e["cache"]["penalty"]) == ep.penalty[i]
        rw = e["status"]["rewards"]
        np.testing.assert_array_equal(np.array(rw + [0.0] * (T - len(rw))), ep.turn_reward[:, i])


def test_port_gae_matches_c_oracle():
    """The timed GAE baseline (torch column loop) == the C oracle's legacy GAE + whitening."""
    import torch
    rng = np.random.default_rng(5)
    n_turns = rng.integers(1, 6, 48).astype(np.int32)
    r, v, m = synthetic.token_rows(n_turns, rng.standard_normal(48).astype(np.float32), seed=3)
    for gamma, lam in ((1.0, 1.0), (1.0, 0.95)):
        adv, ret = port.verl_gae_whiten(torch.from_numpy(r), torch.from_numpy(v), torch.from_numpy(m), gamma, lam)
        oa, oret = oracle.gae(r, v, m, gamma, lam)
        np.testing.assert_allclose(ret.numpy(), oret, rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(adv.numpy(), oracle.masked_whiten(oa, m), rtol=1e-4, atol=1e-4)
