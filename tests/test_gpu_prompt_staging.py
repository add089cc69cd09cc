"""rmi_prompt_text's staging (csrc/prompt.hip): the row's pool, observation and response are
copied into LDS before the piece loop when they are dword-sized and aligned, and read in place
otherwise.  The same program over the same rows must give the same bytes either way: a pool
whose length is a multiple of 4 (staged) against one that is not, response rows at a dword
stride against an odd stride, observation rows past 256 bytes (the staging's second loop),
rewards whose repr needs the exact search (17 significant digits), INT / TAG_CONST / IF pieces.
The expected text of the simple pieces is also checked directly."""
import numpy as np
import pytest
import torch

from ragen_amd import _lib
import ragen_amd.torch_ops  # noqa: F401  (registers torch.ops.ragen_amd)

pytestmark = pytest.mark.gpu


def _program(pieces, n_tags, obs_stride, resp_stride, enable_think=1, K=5):
    flat = [len(pieces)] + [x for p in pieces for x in p] + [n_tags, obs_stride, resp_stride, enable_think, K]
    return flat


def _run(pool_bytes, pool_pad, resp, resp_len, obs, obs_len, ints, reward, reward_int, spans, cond, tag, tag_const,
         pieces, B, stride, dev):
    pool = torch.frombuffer(bytearray(pool_bytes) + b"\0" * pool_pad, dtype=torch.uint8).to(dev)
    prog = _program(pieces, tag_const.shape[0] // 2 if tag_const is not None else 1, obs.shape[1], resp.shape[1])
    return torch.ops.ragen_amd.prompt_text(prog, list(b"||"), B, stride, pool, tag_const, tag, obs, obs_len, ints,
                                           reward, reward_int, resp, resp_len, spans, cond, None)


def test_prompt_text_staged_equals_in_place():
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(5)
    B, stride = 256, 2048
    consts = ["<|im_start|>user\nTurn 2:\nState:\n", "\nYou have ", " actions left.", "Reward:\n", "\n", "A:", "B:"]
    pool_bytes = b"".join(c.encode() for c in consts)
    offs = np.cumsum([0] + [len(c.encode()) for c in consts])
    C = lambda j: (_lib.PT_CONST, int(offs[j]), int(offs[j + 1] - offs[j]))  # noqa: E731
    # two tags: TAG_CONST 0 is "A:" for tag 0 and "B:" for tag 1
    tag_const = torch.tensor([int(offs[5]), 2, int(offs[6]), 2], dtype=torch.int32, device=dev)
    tag = torch.from_numpy(rng.integers(0, 2, B).astype(np.uint8)).to(dev)
    # observations: rows up to 300 bytes (past the first 256-byte batch)
    obs_stride = 300
    obs_np = np.zeros((B, obs_stride), np.uint8)
    obs_len_np = rng.integers(0, obs_stride + 1, B).astype(np.int32)
    for i in range(B):
        obs_np[i, :obs_len_np[i]] = rng.choice(list(b"#_PXO\n"), obs_len_np[i])
    # responses "<think>..</think><answer>Up || Down</answer>" after the "<think>" prefix
    texts = [f"t{i} </think><answer> Up || Down || Left </answer>".encode() for i in range(B)]
    rs = 4 * ((max(len(t) for t in texts) + 3) // 4) + 4
    resp_np = np.zeros((B, rs), np.uint8)
    for i, t in enumerate(texts):
        resp_np[i, :len(t)] = np.frombuffer(t, np.uint8)
    resp_len = torch.tensor([len(t) for t in texts], dtype=torch.int32, device=dev)
    spans = []
    for t in texts:  # think [7, te), answer [as, ae) in the prefixed text
        s = "<think>" + t.decode()
        te = s.index("</think>")
        a0 = s.index("<answer>") + len("<answer>")
        spans.append([7, te, a0, s.index("</answer>")])
    spans = torch.tensor(spans, dtype=torch.int32, device=dev)
    ints = torch.from_numpy(rng.integers(0, 12, (1, B)).astype(np.int32)).to(dev)
    rw = rng.choice([-0.1, 0.9, -0.30000000000000004, 10.8, 0.0, -1.2000000000000002], B)
    reward = torch.from_numpy(rw).to(dev)
    reward_int = torch.from_numpy((rng.random(B) < 0.2).astype(np.uint8)).to(dev)
    cond = torch.from_numpy((rng.random(B) < 0.8).astype(np.uint8)).to(dev)
    pieces = [(_lib.PT_RESPONSE, 0, 0), (_lib.PT_MARK, 0, 0), (_lib.PT_IF, 0, 0), C(3), (_lib.PT_REWARD, 0, 0), C(0),
              (_lib.PT_OBS, 0, 0), C(1), (_lib.PT_INT, 0, 0), C(2), (_lib.PT_TAG_CONST, 0, 0), C(4)]
    obs = torch.from_numpy(obs_np).to(dev)
    obs_len = torch.from_numpy(obs_len_np).to(dev)
    pad = (-len(pool_bytes)) % 4
    outs = []
    for pool_pad, resp_t in ((pad + 4, torch.from_numpy(resp_np).to(dev)),              # staged pool and rows
                             (pad + 5, torch.from_numpy(resp_np).to(dev)),              # pool in place
                             (pad + 4, torch.from_numpy(np.pad(resp_np, ((0, 0), (0, 1)))).to(dev))):  # odd stride
        text, tlen, mark, err = _run(pool_bytes, pool_pad, resp_t, resp_len, obs, obs_len, ints, reward, reward_int,
                                     spans, cond, tag, tag_const, pieces, B, stride, dev)
        torch.cuda.synchronize()
        outs.append((text.cpu().numpy(), tlen.cpu().numpy(), mark.cpu().numpy(), err.cpu().numpy()))
    ref = outs[0]
    assert not ref[3].any()
    for o in outs[1:]:
        np.testing.assert_array_equal(o[1], ref[1])
        np.testing.assert_array_equal(o[2], ref[2])
        for i in range(B):
            assert bytes(o[0][i, :o[1][i]]) == bytes(ref[0][i, :ref[1][i]]), i
    # the simple pieces, spelled out
    for i in range(B):
        row = bytes(ref[0][i, :ref[1][i]]).decode()
        assert row.startswith("<think>")
        if not cond[i]:
            assert row.endswith("</answer>")
            continue
        r = float(rw[i])
        rtxt = str(int(r)) if reward_int[i] else repr(r)
        tail = ("Reward:\n" + rtxt + consts[0] + bytes(obs_np[i, :obs_len_np[i]]).decode() + consts[1] +
                str(int(ints[0, i])) + consts[2] + ("A:" if int(tag[i]) == 0 else "B:") + "\n")
        assert row.endswith(tail), (i, row[-120:], tail)


def test_prompt_text_turn_form_equals_explicit():
    """The turn form (turn_exec, flags, int_reward_tags, last_turn: reward_int and cond derived
    on the device) against the same rows with reward_int / cond given: identical bytes, marks and
    errors, for both tags (tag 1 = Countdown's integer 0 / 1 rewards), done and running envs, the
    last turn and an earlier one."""
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(11)
    B, stride = 512, 1024
    consts = ["Reward:\n", "\nTurn 3:\n", "A:", "B:", "\n"]
    pool_bytes = b"".join(c.encode() for c in consts)
    offs = np.cumsum([0] + [len(c.encode()) for c in consts])
    C = lambda j: (_lib.PT_CONST, int(offs[j]), int(offs[j + 1] - offs[j]))  # noqa: E731
    tag_const = torch.tensor([int(offs[2]), 2, int(offs[3]), 2], dtype=torch.int32, device=dev)
    tag_np = rng.integers(0, 2, B).astype(np.uint8)
    tag = torch.from_numpy(tag_np).to(dev)
    obs_np = np.zeros((B, 8), np.uint8)
    obs_np[:, :4] = np.frombuffer(b"#P_#", np.uint8)
    obs = torch.from_numpy(obs_np).to(dev)
    obs_len = torch.full((B,), 4, dtype=torch.int32, device=dev)
    ints = torch.from_numpy(rng.integers(0, 9, (1, B)).astype(np.int32)).to(dev)
    rw = rng.choice([0.0, 1.0, -0.1, 0.9, 10.0, -1.0], B)
    reward = torch.from_numpy(rw).to(dev)
    ne_np = rng.integers(0, 3, B).astype(np.uint8)
    fl_np = (rng.random(B) < 0.3).astype(np.uint8) * _lib.FLAG_DONE | (rng.random(B) < 0.3).astype(np.uint8)
    ne, fl = torch.from_numpy(ne_np).to(dev), torch.from_numpy(fl_np).to(dev)
    pieces = [(_lib.PT_MARK, 0, 0), (_lib.PT_IF, 0, 0), C(0), (_lib.PT_REWARD, 0, 0), C(1), (_lib.PT_OBS, 0, 0),
              (_lib.PT_INT, 0, 0), (_lib.PT_TAG_CONST, 0, 0), C(4)]
    prog = _program(pieces, 2, obs.shape[1], 0)
    pad = (-len(pool_bytes)) % 4 + 4
    pool = torch.frombuffer(bytearray(pool_bytes) + b"\0" * pad, dtype=torch.uint8).to(dev)
    R = torch.ops.ragen_amd
    for last in (0, 1):
        rint = ((ne_np == 0) | ((tag_np == 1) & ((rw == 0.0) | (rw == 1.0)))).astype(np.uint8)
        cond = (((fl_np & _lib.FLAG_DONE) == 0) & (not last)).astype(np.uint8)
        want = R.prompt_text(prog, list(b"||"), B, stride, pool, tag_const, tag, obs, obs_len, ints, reward,
                             torch.from_numpy(rint).to(dev), None, None, None, torch.from_numpy(cond).to(dev), None)
        got = R.prompt_text(prog, list(b"||"), B, stride, pool, tag_const, tag, obs, obs_len, ints, reward, None,
                            None, None, None, None, None, ne, fl, 0b10, last)
        torch.cuda.synchronize()
        for w, g in zip(want[1:], got[1:]):  # lengths, marks, errors
            assert torch.equal(w, g), last
        lens = got[1].cpu().numpy()
        tw, tg = want[0].cpu().numpy(), got[0].cpu().numpy()
        for i in range(B):  # the bytes of each row (the buffer past a row's length is not written)
            assert bytes(tw[i, :lens[i]]) == bytes(tg[i, :lens[i]]), (last, i)
        assert (lens[cond == 0] == 0).all() and (lens[cond == 1] > 0).all()
