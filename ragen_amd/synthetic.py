"""Synthetic, fixed-seed workloads of SURVEY.md §8(d) (no LLM / dataset offline).

Actions stand in for parsed LLM responses: per env per turn n ~ U{0..K} actions, each a
known action id U{lo..hi} or, with probability p_unknown, an unknown name (id 0, dropped
by the name->id map and charged the format penalty).  GAE inputs are token rows shaped
like StarPO transcripts: a 150-token prompt (mask 0), then per executed turn a state block
U[32,96] (mask 0) and a response block U[16,128] (mask 1); rows left-padded to the batch
max length; V ~ N(0,1)*mask; reward = trajectory score at the last column.
"""
import numpy as np

ACTION_SEED = 20250704
ENV_SEED = 1000
GROUP_SIZE = 16


def turn_actions(rng: np.random.Generator, B: int, K: int, lo: int, hi: int, p_unknown: float = 0.1):
    """-> (ids i8[B,K], n_actions u8[B])"""
    n = rng.integers(0, K + 1, size=B).astype(np.uint8)
    ids = rng.integers(lo, hi + 1, size=(B, K)).astype(np.int8)
    unk = rng.random((B, K)) < p_unknown
    ids[unk] = 0
    ids[np.arange(K)[None, :] >= n[:, None]] = 0
    return ids, n


def rollout_actions(B: int, T: int, K: int, lo: int, hi: int, seed: int = ACTION_SEED, p_unknown: float = 0.1):
    """Pre-generated actions for T turns: (ids i8[T,B,K], n_actions u8[T,B])."""
    rng = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))
    ids = np.zeros((T, B, K), np.int8)
    n = np.zeros((T, B), np.uint8)
    for t in range(T):
        ids[t], n[t] = turn_actions(rng, B, K, lo, hi, p_unknown)
    return ids, n


def env_seeds(B: int, base: int = ENV_SEED, group_size: int = GROUP_SIZE, first_group: int = 0):
    """env i -> base + i // group_size (es_manager.py:80-82)."""
    return (base + first_group + np.arange(B) // group_size).astype(np.int64)


def token_rows(n_turns, scores, seed: int = 7, prompt: int = 150, turn_scores=None, max_len=None):
    """Token-level GAE inputs for trajectories with n_turns[b] executed turns.

    -> r f32[B,L], v f32[B,L], mask u8[B,L] (left padded).  With ``turn_scores`` [B,T] the
    reward of turn t sits on the last response token of that turn (bi-level / turn-score
    variant); otherwise scores[b] sits at the last column (StarPO default)."""
    rng = np.random.default_rng(seed)
    B = len(n_turns)
    lens, blocks = [], []
    for b in range(B):
        segs = [(prompt, 0)]
        for _ in range(max(int(n_turns[b]), 1)):
            segs.append((int(rng.integers(32, 97)), 0))
            segs.append((int(rng.integers(16, 129)), 1))
        blocks.append(segs)
        lens.append(sum(s for s, _ in segs))
    L = max(lens) if max_len is None else int(max_len)
    r = np.zeros((B, L), np.float32)
    mask = np.zeros((B, L), np.uint8)
    for b in range(B):
        pos = L - lens[b]
        t = 0
        for size, m in blocks[b]:
            if m:
                mask[b, pos:pos + size] = 1
                if turn_scores is not None:
                    r[b, pos + size - 1] = turn_scores[b, t]
                t += 1
            pos += size
        if turn_scores is None:
            r[b, L - 1] = scores[b]
    v = (rng.standard_normal((B, L)).astype(np.float32) * mask).astype(np.float32)
    return r, v, mask


def countdown_answers(instances, T: int, seed: int = ACTION_SEED, p_empty: float = 0.5):
    """Per env per turn a Countdown answer: with p_empty no parsed answer (the
    turn only costs the format penalty), else an expression over {digits + - * / ( )} and the
    instance's numbers that is
    * correct (1/3): the signed sum reaching the target, a left prefix of it parenthesised
      half of the time ("(-12 + 40) - 7");
    * format-only (1/3): every number once, in a random order, joined by random + - * / with
      random parentheses (evaluates to the target only by chance);
    * wrong numbers (1/3): the same grammar with one number off by one (reward 0).
    -> [T][B] str or None."""
    rng = np.random.default_rng(seed)
    out = [[None] * len(instances) for _ in range(T)]

    def grammar(vals):  # a random binary tree over vals in order, fully parenthesised inside
        if len(vals) == 1:
            return str(vals[0])
        cut = int(rng.integers(1, len(vals)))
        op = "+-*/"[int(rng.integers(0, 4))]
        left, right = grammar(vals[:cut]), grammar(vals[cut:])
        if cut > 1:
            left = "(" + left + ")"
        if len(vals) - cut > 1:
            right = "(" + right + ")"
        return left + " " + op + " " + right

    for t in range(T):
        for i, inst in enumerate(instances):
            if rng.random() < p_empty:
                continue
            nums, target = list(inst["nums"]), int(inst["target"])
            kind = int(rng.integers(0, 3))
            signs = None
            for m in range(1 << len(nums)):  # a sign pattern reaching the target (it exists)
                sg = [1 if (m >> j) & 1 else -1 for j in range(len(nums))]
                if sum(s * v for s, v in zip(sg, nums)) == target:
                    signs = sg
                    break
            if kind == 0 and signs is not None:
                terms = [("-" if signs[0] < 0 else "") + str(nums[0])]
                terms += [("+ " if s > 0 else "- ") + str(v) for s, v in zip(signs[1:], nums[1:])]
                cut = int(rng.integers(2, len(terms) + 1)) if rng.random() < 0.5 and len(terms) > 2 else 0
                if cut:
                    terms = ["(" + " ".join(terms[:cut]) + ")"] + terms[cut:]
                out[t][i] = " ".join(terms)
                continue
            if kind == 2:
                nums[int(rng.integers(0, len(nums)))] += 1
            out[t][i] = grammar([nums[j] for j in rng.permutation(len(nums))])
    return out


UNKNOWN_NAMES = ("Jump", "Wait", "north", "Stay", "upp")
THINK_WORDS = ("the", "box", "is", "left", "of", "target", "so", "I", "should", "push", "it", "right", "then",
               "move", "up", "avoid", "wall", "corner", "player", "at", "row", "column", "2", "3", "—", "→")


def responses_for_actions(ids: np.ndarray, n_actions: np.ndarray, lookup, seed: int = 11, think_words=(8, 60),
                          enable_think: bool = True):
    """LLM-shaped responses (the generation after the '<think>' tag, ctx_manager.py:338) whose
    answer lists the given actions: ids i8[B,K] (0 = an unknown name), n_actions u8[B].
    Names in random case and spacing, " || "-separated.  -> list[str]."""
    rng = np.random.default_rng(seed)
    out = []
    for b in range(ids.shape[0]):
        acts = []
        for k in range(int(n_actions[b])):
            i = int(ids[b, k])
            nm = lookup[i] if i else UNKNOWN_NAMES[int(rng.integers(len(UNKNOWN_NAMES)))]
            c = int(rng.integers(4))
            nm = nm.lower() if c == 1 else (nm.upper() if c == 2 else nm)
            acts.append(nm)
        seps = [" || ", "||", " ||", "|| "]
        body = ""
        for k, a in enumerate(acts):
            body += (seps[int(rng.integers(4))] if k else "") + a
        nw = int(rng.integers(think_words[0], think_words[1] + 1))
        think = " ".join(THINK_WORDS[int(j)] for j in rng.integers(len(THINK_WORDS), size=nw))
        gap = ["", " ", "\n"][int(rng.integers(3))]
        pad = [" ", ""][int(rng.integers(2))]
        if enable_think:
            out.append(f"{think}</think>{gap}<answer>{pad}{body}{pad}</answer>")
        else:
            out.append(f"{pad}{body}{pad}</answer>")
    return out


def encode_rows(texts, stride: int = 0):
    """list[str] -> (u8[B, stride] UTF-8 rows, i32[B] byte lengths); stride rounded up to 4."""
    bs = [t.encode("utf-8") for t in texts]
    L = max([len(b) for b in bs] + [1, stride])
    L = (L + 3) // 4 * 4
    buf = np.zeros((len(bs), L), np.uint8)
    for i, b in enumerate(bs):
        buf[i, :len(b)] = np.frombuffer(b, np.uint8)
    return buf, np.array([len(b) for b in bs], np.int32)


def byte_vocab(extra_words=()):
    """A byte-level vocabulary for synthetic token ids: one token per byte, whole words of the
    synthetic responses, and a special pad token (last id).  -> (table list[bytes], skip u8[V])."""
    words = ["</think>", "<answer>", "</answer>", " || ", "||", " ||", "|| "]
    for nm in ("Up", "Down", "Left", "Right") + UNKNOWN_NAMES:
        words += [nm, nm.lower(), nm.upper()]
    words += [" " + w for w in THINK_WORDS] + list(extra_words)
    table = [bytes([i]) for i in range(256)] + [w.encode("utf-8") for w in dict.fromkeys(words)] + [b"<|endoftext|>"]
    skip = np.zeros(len(table), np.uint8)
    skip[-1] = 1
    return table, skip


def tokenize_greedy(texts, table, R=None):
    """Longest-match tokenisation of UTF-8 texts over `table` (the byte tokens guarantee
    coverage), right-padded with the last (special) id.  -> i64[B, R]."""
    by_first = {}
    for i, t in enumerate(table[:-1]):
        if len(t) > 1:
            by_first.setdefault(t[0], []).append((t, i))
    for k in by_first:
        by_first[k].sort(key=lambda x: -len(x[0]))
    rows = []
    for txt in texts:
        b, i, row = txt.encode("utf-8"), 0, []
        while i < len(b):
            for t, tid in by_first.get(b[i], ()):
                if b.startswith(t, i):
                    row.append(tid)
                    i += len(t)
                    break
            else:
                row.append(b[i])
                i += 1
        rows.append(row)
    R = R or max(len(r) for r in rows)
    out = np.full((len(rows), R), len(table) - 1, np.int64)
    for j, r in enumerate(rows):
        out[j, :len(r)] = r[:R]
    return out


class ByteChatTokenizer:
    """Offline stand-in for the Qwen2.5 tokenizer (a hub download, unavailable here) for the
    benchmark's end-to-end rollout: Qwen's chat template and <|im_start|> / <|im_end|> /
    <|endoftext|> ids, every other byte its own id (0..255).  Vectorised (numpy per text), so
    formulating an 8192-env batch takes well under a second."""
    name_or_path = "Qwen/Qwen2.5-0.5B-Instruct (byte-level stand-in)"
    IM_START, IM_END, PAD = 151644, 151645, 151643
    pad_token_id = 151643
    _SPECIAL = {"<|im_start|>": 151644, "<|im_end|>": 151645, "<|endoftext|>": 151643}

    def encode(self, text):
        return [self._SPECIAL[text]] if text in self._SPECIAL else list(text.encode("utf-8"))

    def apply_chat_template(self, messages, add_generation_prompt, tokenize):
        s = "".join(f"<|im_start|>{m['role']}\n{m['content']}<|im_end|>\n" for m in messages)
        return s + ("<|im_start|>assistant\n" if add_generation_prompt else "")

    def _ids(self, text):
        import re
        parts = re.split(r"(<\|im_start\|>|<\|im_end\|>|<\|endoftext\|>)", text)
        out = [np.array([self._SPECIAL[p]], np.int64) if p in self._SPECIAL else
               np.frombuffer(p.encode("utf-8"), np.uint8).astype(np.int64) for p in parts if p]
        return np.concatenate(out) if out else np.zeros(0, np.int64)

    def __call__(self, texts, return_tensors="pt", padding=True, padding_side="left", truncation=False):
        import torch
        rows = [self._ids(t) for t in texts]
        if not padding:  # ragged rows, as a HF tokenizer's padding=False
            o = type("Enc", (), {})()
            o.input_ids = rows
            return o
        L = max(len(r) for r in rows)
        ids = np.full((len(rows), L), self.PAD, np.int64)
        am = np.zeros((len(rows), L), np.int64)
        for b, r in enumerate(rows):
            ids[b, L - len(r):] = r
            am[b, L - len(r):] = 1

        class Enc:
            pass
        e = Enc()
        e.input_ids, e.attention_mask = torch.from_numpy(ids), torch.from_numpy(am)
        return e

    def batch_decode(self, rows, skip_special_tokens=True):
        out = []
        for r in rows:
            r = np.asarray(r.tolist() if hasattr(r, "tolist") else r, np.int64)
            keep = r[r < 256] if skip_special_tokens else r
            out.append(bytes(keep.astype(np.uint8).tolist()).decode("utf-8", errors="replace"))
        return out


# --------------------------------------------------------- a Qwen2-style BPE tokenizer
QWEN_CHAT_TEMPLATE = (
    "{%- if messages[0]['role'] == 'system' %}"
    "{{- '<|im_start|>system\\n' + messages[0]['content'] + '<|im_end|>\\n' }}"
    "{%- else %}"
    "{{- '<|im_start|>system\\nYou are Qwen, created by Alibaba Cloud. You are a helpful assistant.<|im_end|>\\n' }}"
    "{%- endif %}"
    "{%- for message in messages %}"
    "{%- if (message.role == 'user') or (message.role == 'system' and not loop.first) or "
    "(message.role == 'assistant') %}"
    "{{- '<|im_start|>' + message.role + '\\n' + message.content + '<|im_end|>' + '\\n' }}"
    "{%- endif %}"
    "{%- endfor %}"
    "{%- if add_generation_prompt %}{{- '<|im_start|>assistant\\n' }}{%- endif %}")


def _tokenizer_corpus(n_docs: int, seed: int):
    """Text of the kind RAGEN's prompts and responses hold: the env instructions, grids,
    'Turn k' blocks, rewards, think / answer tags, words, numbers and some non-ASCII."""
    from .env import REGISTERED_ENV_CONFIGS
    rng = np.random.default_rng(seed)
    words = list(THINK_WORDS) + ["Up", "Down", "Left", "Right", "box", "target", "wall", "player", "State", "Turn",
                                 "Reward", "actions", "left", "answer", "think", "You", "have", "Always", "output",
                                 "format", "Strictly", "follow", "response", "length", "words", "tokens", "Target",
                                 "nums", "hole", "goal", "Phoenix", "Dragon", "café", "naïve", "über", "中文", "日本",
                                 "Привет", "мир", "ελληνικά", "√", "→", "…", "don't", "it's", "we're", "I'll"]
    # pseudo-words with a Zipf-like frequency: a vocabulary with many merges, as a real one
    syl = ["ka", "re", "to", "mi", "sa", "lo", "ne", "pu", "ti", "ga", "ber", "con", "ing", "tion", "er", "st", "an",
           "th", "ou", "pre", "ex", "al", "ly", "ment", "ous", "ive", "de", "un", "ch", "qu", "sh", "ph", "or", "es"]
    lex = ["".join(rng.choice(syl) for _ in range(int(rng.integers(1, 4)))) for _ in range(3000)]
    zipf = 1.0 / np.arange(1, len(lex) + 1)
    zipf /= zipf.sum()
    docs = [" ".join(lex[int(i)] if rng.random() > 0.1 else lex[int(i)].capitalize()
                     for i in rng.choice(len(lex), size=200, p=zipf)) for _ in range(n_docs // 3)]
    for cls in REGISTERED_ENV_CONFIGS.values():
        c = cls()
        docs.append(str(getattr(c, "env_instruction", "")))
        for k in ("grid_vocab", "action_lookup"):
            v = getattr(c, k, None)
            if v:
                docs.append(", ".join(f"{a}: {b}" for a, b in v.items()))
    for _ in range(n_docs):
        k = int(rng.integers(8, 60))
        toks = [words[int(i)] for i in rng.integers(0, len(words), size=k)]
        for i in range(k):
            r = rng.random()
            if r < 0.08:
                toks[i] = str(int(rng.integers(0, 1000)))
            elif r < 0.12:
                toks[i] = f"{rng.normal():.4g}"
            elif r < 0.16:
                toks[i] = rng.choice(["||", " || ", "\n", "\n\n", ":", ".", ",", "!", "?", "  ", "\t", "(", ")"])
        grid = "\n".join("".join(rng.choice(list("#_OXP√")) for _ in range(6)) for _ in range(6))
        docs.append(f"<think>{' '.join(toks)}</think><answer>{rng.choice(words)} || {rng.choice(words)}</answer>\n"
                    f"Turn {int(rng.integers(1, 9))}:\nState:\n{grid}\nYou have {int(rng.integers(0, 11))} actions "
                    f"left.\nReward:\n{rng.choice([0, -0.1, 1.0, -0.30000000000000004, 10.9])}\n")
    return docs


def qwen_like_tokenizer(vocab_size: int = 6000, n_docs: int = 1500, seed: int = 7):
    """A byte-level BPE with the Qwen2 / Qwen2.5 tokenizer's pipeline (NFC normalizer, the Qwen2
    pre-tokenizer regex + ByteLevel, <|endoftext|> / <|im_start|> / <|im_end|> added tokens, the
    Qwen chat template), trained deterministically on RAGEN-like text.  The Qwen2.5 tokenizer is
    a hub download (unavailable offline); this is its pipeline with a smaller vocabulary."""
    from tokenizers import Regex, Tokenizer, decoders, models, normalizers, pre_tokenizers, trainers
    from transformers import PreTrainedTokenizerFast
    from .tokenizer import QWEN2_PATTERN
    tok = Tokenizer(models.BPE())
    tok.normalizer = normalizers.NFC()
    tok.pre_tokenizer = pre_tokenizers.Sequence([
        pre_tokenizers.Split(Regex(QWEN2_PATTERN), behavior="isolated", invert=False),
        pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False)])
    tok.decoder = decoders.ByteLevel()
    tr = trainers.BpeTrainer(vocab_size=vocab_size, initial_alphabet=pre_tokenizers.ByteLevel.alphabet(),
                             show_progress=False)
    tok.train_from_iterator(_tokenizer_corpus(n_docs, seed), tr)
    tok.add_special_tokens(["<|endoftext|>", "<|im_start|>", "<|im_end|>"])
    return PreTrainedTokenizerFast(tokenizer_object=tok, name_or_path="Qwen/Qwen2.5-0.5B-Instruct (synthetic BPE)",
                                   eos_token="<|im_end|>", pad_token="<|endoftext|>", chat_template=QWEN_CHAT_TEMPLATE,
                                   clean_up_tokenization_spaces=False)


def qwen_scale_tokenizer(n_merges: int = 151000, seed: int = 11, base=None):
    """qwen_like_tokenizer's pipeline with a merge table of Qwen2's size (~151 k merges; the real
    table is a hub download): the trained tokenizer's merges, then random merges of two tokens
    already in the vocabulary (ranked after every trained one, words up to 16 bytes) until the
    table holds ``n_merges``.  A stand-in for the merge-table SIZE (hash-table footprint and
    lookups); which pairs merge is arbitrary.  Deterministic in ``seed``."""
    import json
    from tokenizers import Tokenizer
    from transformers import PreTrainedTokenizerFast
    base = base if base is not None else qwen_like_tokenizer()
    j = json.loads(base.backend_tokenizer.to_str())
    m = j["model"]
    vocab, merges = m["vocab"], [list(x) for x in m["merges"]]
    special = {t["id"] for t in j.get("added_tokens", [])}
    toks = [t for t, i in sorted(vocab.items(), key=lambda x: x[1]) if i not in special]
    nxt = max(vocab.values()) + 1
    rng = np.random.default_rng(seed)
    seen = {(a, b) for a, b in merges}
    by_len = [[] for _ in range(17)]  # tokens by their byte length (a new word stays <= 16 bytes)
    for t in toks:
        n = len(t.encode())
        if n <= 16:
            by_len[n].append(t)
    draws = rng.random((2 * n_merges, 2))
    k = 0
    while len(merges) < n_merges:
        if k == len(draws):
            draws, k = rng.random((2 * n_merges, 2)), 0
        la = 1 + int(draws[k, 0] * 8)  # a: 1..8 bytes, b: what is left of 16
        lb = 1 + int(draws[k, 1] * (16 - la))
        k += 1
        if not by_len[la] or not by_len[lb]:
            continue
        a = by_len[la][int(rng.integers(len(by_len[la])))]
        b = by_len[lb][int(rng.integers(len(by_len[lb])))]
        w = a + b
        if (a, b) in seen or w in vocab:
            continue
        seen.add((a, b))
        merges.append([a, b])
        vocab[w] = nxt
        by_len[la + lb].append(w)
        nxt += 1
    # the added tokens keep their ids: move them past the new ones
    for t in j.get("added_tokens", []):
        t["id"] = nxt
        vocab.pop(t["content"], None)
        nxt += 1
    m["merges"] = merges
    tk = Tokenizer.from_str(json.dumps(j))
    # (no name at construction: above 100 k tokens transformers looks the name up on the hub)
    out = PreTrainedTokenizerFast(tokenizer_object=tk, eos_token="<|im_end|>", pad_token="<|endoftext|>",
                                  chat_template=base.chat_template, clean_up_tokenization_spaces=False)
    out.name_or_path = base.name_or_path + f", {n_merges} merges"
    return out
