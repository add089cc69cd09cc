"""Helpers turning the recorded golden traces (tests/golden/*_es.npz) into kernel inputs."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

SOKOBAN_LOOKUP = {1: "Up", 2: "Down", 3: "Left", 4: "Right"}
FROZEN_LOOKUP = {1: "Left", 2: "Down", 3: "Right", 4: "Up"}


def load(name):
    d = np.load(os.path.join(GOLDEN, name + ".npz"))
    return {k: d[k] for k in d.files}


_STRINGS = None


def strings():
    global _STRINGS
    if _STRINGS is None:
        with open(os.path.join(GOLDEN, "strings.json")) as f:
            _STRINGS = json.load(f)
    return _STRINGS


def map_codes(codes, vocab, lookup_for_env):
    """codes[T,B,K] vocab indices (-1 = none) -> ids[T,B,K] i8 via case-insensitive lookup."""
    T, B, K = codes.shape
    ids = np.zeros((T, B, K), np.int8)
    for t in range(T):
        for b in range(B):
            rev = {v.lower(): k for k, v in lookup_for_env(b).items()}
            for k in range(K):
                c = codes[t, b, k]
                if c >= 0:
                    ids[t, b, k] = rev.get(vocab[c].lower(), 0)
    return ids


def trace_inputs(name):
    d = load(name)
    env = name.split("_")[0]
    vocab = strings()[name]["vocab"]
    if env.startswith("sokoban"):
        ids = map_codes(d["codes"], vocab, lambda b: SOKOBAN_LOOKUP)
    elif env == "frozenlake":
        ids = map_codes(d["codes"], vocab, lambda b: FROZEN_LOOKUP)
    elif env == "bandit":
        hi = d["init_hi_is_first"]
        ids = map_codes(d["codes"], vocab,
                        lambda b: {1: "Dragon", 2: "Phoenix"} if hi[b] else {1: "Phoenix", 2: "Dragon"})
    else:
        ids = None
    return d, ids
