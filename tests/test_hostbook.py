"""The dict facade's host bookkeeping in C (ragen_amd/csrc/hostbook.c) against its Python
definition (EnvStateManager._book_py, es_manager.py:130-169 of the reference): the same
EnvStatus fields, penalties, history entries (values and types: Countdown's int rewards, the
int 0 of a turn without a step), note callbacks and active sets, over random turns of every
branch.  CPU only: the turn's device results are given as the lists _book receives."""
import copy
import random

import pytest

from ragen_amd import _lib
from ragen_amd.llm_agent import es_manager as em


class _Batch:
    def __init__(self, B, with_note):
        self.calls = []
        self.B = B
        if with_note:
            self.note_executed = lambda t, i, ex: self.calls.append((t, i, list(ex)))

    def render(self, i):
        return f"state of {i}"


class _Tag:
    def __init__(self, env_type, batch):
        self.env_type = env_type
        self.batch = batch


class _Es:
    def __init__(self, B, lo, max_actions):
        self.env_lo = lo
        self.envs = [{"status": em.EnvStatus(seed=lo + i), "max_actions_per_traj": max_actions} for i in range(B)]
        self._rc = [{"env_id": lo + i, "history": [{"state": "s0", "actions_left": max_actions}], "penalty": 0}
                    for i in range(B)]


def _turn(rng, B, lo, K, is_cd, pre_rendered):
    rows = sorted(rng.sample(range(B), rng.randint(1, B)))
    gids = [lo + i for i in rows]
    inputs = [{"env_id": g, "llm_response": f"resp {g}", "llm_raw_response": f"<think>{g}</think>",
               "actions": []} for g in gids]
    acts_l = [[rng.choice(["Up", "Down", "x"]) for _ in range(rng.randint(0, K))] for _ in rows]
    m_l = [[rng.choice([0, 1, 2, 3, 4]) for _ in a] for a in acts_l]
    F = [_lib.FLAG_TERMINATED, _lib.FLAG_TRUNCATED, _lib.FLAG_DONE]
    flags = [sum(f for f in F if rng.random() < 0.3) for _ in range(B)]
    num_actions = [rng.randint(0, 10) for _ in range(B)]
    I = [_lib.INFO_PRESENT, _lib.INFO_EFFECTIVE, _lib.INFO_VALID, _lib.INFO_SUCCESS]
    info = [sum(b for b in I if rng.random() < 0.5) for _ in range(B)]
    n_exec = [rng.randint(0, K) for _ in range(B)]
    vals = [0.0, 1.0, -0.1, 0.1, -0.30000000000000004, 10.9] if not is_cd else [0.0, 1.0, 0.1]
    rw = [rng.choice(vals) for _ in range(B)]
    pen = [rng.choice([0.0, -0.1]) for _ in range(B)]
    obs = [f"obs {i}" for i in range(B)] if pre_rendered else None
    return inputs, gids, rows, acts_l, m_l, flags, num_actions, info, n_exec, rw, pen, obs


def _snapshot(es, batch, still):
    st = [(e["status"].num_actions, [(type(r).__name__, r) for r in e["status"].rewards], e["status"].terminated,
           e["status"].truncated) for e in es.envs]
    hist = repr(es._rc)  # values and types (1 vs 1.0) of every entry
    return st, hist, sorted(still), list(batch.calls)


@pytest.mark.parametrize("is_cd,with_note,pre_rendered", [(False, False, True), (False, True, False),
                                                          (True, True, True), (True, False, False)])
def test_hostbook_equals_python(is_cd, with_note, pre_rendered):
    hb = em._hostbook()
    assert hb is not None, "the extension must be built (ragen_amd.build)"
    rng = random.Random(7 + 2 * is_cd + with_note)
    B, lo, K = 40, 1000, 5
    es_c, es_p = _Es(B, lo, 10), _Es(B, lo, 10)
    b_c, b_p = _Batch(B, with_note), _Batch(B, with_note)
    tg_c, tg_p = _Tag("countdown" if is_cd else "sokoban", b_c), _Tag("countdown" if is_cd else "sokoban", b_p)
    for t in range(6):
        args = _turn(rng, B, lo, K, is_cd, pre_rendered)
        still_c = em.EnvStateManager._book(es_c, tg_c, t, *copy.deepcopy(args))
        still_p = em.EnvStateManager._book_py(es_p, tg_p, t, *copy.deepcopy(args))
        assert _snapshot(es_c, b_c, still_c) == _snapshot(es_p, b_p, still_p), t
