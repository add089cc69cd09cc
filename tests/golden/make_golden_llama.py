"""Golden vectors for the Llama-3 branch of get_special_tokens (ctx_manager.py:24-33) and the
un-rolled score placement of get_masks_and_scores (ctx_manager.py:35-70, the roll at :60-62 is
Qwen-only), by RUNNING THE READ-ONLY REFERENCE.

TEST INFRASTRUCTURE.  Run in the build container only:

    PYTHONHASHSEED=0 python tests/golden/make_golden_llama.py

It imports make_golden (which installs refshim's restatements of the absent third-party code) and
calls the reference's own ``get_special_tokens`` and ``get_masks_and_scores`` on Llama-3-shaped
chat rows.  Only data is written: tests/golden/masks_scores_llama.npz.

Rows: <|begin_of_text|>, then a system header block, then (user, assistant) blocks, each
``<|start_header_id|> role <|end_header_id|> \\n\\n content <|eot_id|>``; rows end on the last
assistant's <|eot_id|> or on one trailing token, and hold 1..4 turns, so rows with fewer turns than
the batch maximum get zip_longest's fill 0 written at their last column (ctx_manager.py:58-59):
without the Qwen roll that write lands on the row's own last token.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import ctxm  # noqa: E402  (installs refshim)

BOT, SH, EH, EOT, NL2, PAD = 128000, 128006, 128007, 128009, 271, 128001


class FakeLlama3Tok:
    """Only what get_special_tokens reads: name_or_path (no encode call on this branch)."""
    name_or_path = "meta-llama/Meta-Llama-3-8B-Instruct"


def block(rng, role_id, lo, hi):
    return [SH, role_id, EH, NL2] + list(int(x) for x in rng.integers(100, 1000, size=int(rng.integers(lo, hi)))) + [EOT]


def cases():
    rng = np.random.default_rng(11)
    tok = FakeLlama3Tok()
    sp, rt = ctxm.get_special_tokens(tok)
    B = 32
    rows, all_scores = [], []
    for b in range(B):
        n_turns = int(rng.integers(1, 5))
        ids = [BOT] + block(rng, 9125, 3, 8)  # system
        sc = []
        for t in range(n_turns):
            ids += block(rng, 882, 2, 9)  # user
            ids += block(rng, 78191, 2, 9)  # assistant
            sc.append(float(rng.choice([-0.1, 0.9, 0.0, 10.9, -1.1, 1.0])))
        if rng.random() < 0.4:
            ids += [int(rng.integers(100, 1000))]  # a trailing token after the last <|eot_id|>
        rows.append(ids)
        all_scores.append(sc)
    S = max(len(r) for r in rows) + 3
    input_ids = np.full((B, S), PAD, np.int64)
    for b, r in enumerate(rows):
        input_ids[b, S - len(r):] = r  # left padding
    out = {"special": np.array([sp, rt], np.int64), "input_ids": input_ids,
           "scores_flat": np.array([s for sc in all_scores for s in sc], np.float64),
           "scores_len": np.array([len(sc) for sc in all_scores], np.int32)}
    for uts in (False, True):
        for erm in (False, True):
            st, lm, rm = ctxm.get_masks_and_scores(torch.from_numpy(input_ids), tok, all_scores,
                                                   use_turn_scores=uts, enable_response_mask=erm)
            key = f"uts{int(uts)}_erm{int(erm)}"
            out[key + "_score"] = st.numpy()
            out[key + "_loss_mask"] = lm.numpy().astype(np.uint8)
            out[key + "_response_mask"] = rm.numpy().astype(np.uint8)
    return out


if __name__ == "__main__":
    np.savez_compressed(os.path.join(HERE, "masks_scores_llama.npz"), **cases())
    print("written", os.path.join(HERE, "masks_scores_llama.npz"))
