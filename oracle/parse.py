"""Parse oracle — TEST INFRASTRUCTURE (checker for rmi_parse_actions / rmi_detokenize).

Python restatement of the response -> action path of ContextManager.get_env_inputs
(ctx_manager.py:332-352) and EnvStateManager._extract_map_valid_actions
(es_manager.py:230-240).  It works on Python ``str`` with ``re`` exactly as the reference does,
so it is the semantic contract the byte-level kernel must meet.  Pinned against vectors
recorded by running the reference's own ``_parse_response`` (tests/golden/parse_response.json,
made by tests/golden/make_golden_parse.py) in tests/test_oracle.py.

``detokenize`` restates the tokenizers ByteLevel decoder (third-party; the reference calls it
through ``tokenizer.batch_decode(..., skip_special_tokens=True)``, ctx_manager.py:334-337):
per-token byte strings concatenated, then ``bytes.decode("utf-8", "replace")``.  Pinned in
tests against the installed ``tokenizers`` library on a synthetic byte-level BPE vocabulary
(the Qwen tokenizer itself is a hub download, absent offline).
"""
import re
from typing import Dict, List, Optional, Sequence, Tuple

SPECIAL_TOKENS = ["<think>", "</think>", "<answer>", "</answer>", "<|im_start|>", "<|im_end|>"]  # ctx_manager.py:94


def parse_response(response: str, enable_think: bool, max_actions: int, action_sep: str = "||"
                   ) -> Tuple[str, List[str]]:
    """ctx_manager.py:148-173 (``_parse_response``)."""
    pattern = r"<think>(.*?)</think>\s*<answer>(.*?)</answer>" if enable_think else r"<answer>(.*?)</answer>"
    m = re.search(pattern, response, re.DOTALL)
    if not m:
        return response, []
    think, content = (m.group(1), m.group(2)) if enable_think else ("", m.group(1))
    for tok in SPECIAL_TOKENS:
        content = content.replace(tok, "").strip()
        think = think.replace(tok, "").strip()
    actions = [a.strip() for a in content.split(action_sep) if a.strip()]
    if len(actions) > max_actions:
        actions = actions[:max_actions]
        content = (" " + action_sep + " ").join(actions)
    if enable_think:
        return f"<think>{think}</think><answer>{content}</answer>", actions
    return f"<answer>{content}</answer>", actions


def prefixed(response: str, enable_think: bool) -> str:
    """ctx_manager.py:338-339: the generation lacks the opening tag; it is added back."""
    return ("<think>" if enable_think else "<answer>") + response


def match_spans(response: str, enable_think: bool) -> Tuple[int, int, int, int]:
    """(think start, think end, answer start, answer end) in UTF-8 byte offsets of the
    prefixed response; all -1 when the pattern does not match."""
    pattern = r"<think>(.*?)</think>\s*<answer>(.*?)</answer>" if enable_think else r"<answer>(.*?)</answer>"
    m = re.search(pattern, response, re.DOTALL)
    if not m:
        return -1, -1, -1, -1

    def off(i):
        return len(response[:i].encode("utf-8"))

    if enable_think:
        return off(m.start(1)), off(m.end(1)), off(m.start(2)), off(m.end(2))
    return -1, -1, off(m.start(1)), off(m.end(1))


def map_actions(actions: Sequence[str], action_lookup: Optional[Dict[int, str]]) -> List:
    """es_manager.py:230-240 (``_extract_map_valid_actions``)."""
    if action_lookup is None:
        return list(actions)
    rev = {v.lower(): k for k, v in action_lookup.items()}
    return [rev[a.lower()] for a in actions if a.lower() in rev]


def action_ids(actions: Sequence[str], action_lookup: Optional[Dict[int, str]]) -> List[int]:
    """Per-action id in the kernels' turn-input convention: the lookup id, 0 when the name is
    not in the lookup (so ``[i for i in ids if i]`` == ``map_actions``), 1 without a lookup."""
    if action_lookup is None:
        return [1] * len(actions)
    rev = {v.lower(): k for k, v in action_lookup.items()}
    return [rev.get(a.lower(), 0) for a in actions]


# ------------------------------------------------------------------ byte-level decoding
def bytes_to_unicode() -> Dict[int, str]:
    """GPT-2 byte <-> printable-char map used by ByteLevel pre-tokenizers / decoders."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, map(chr, cs)))


def token_bytes(token: str, char_to_byte: Dict[str, int]) -> bytes:
    """ByteLevel decoder for one token: every char mapped back to its byte, or — when some
    char is outside the map (added tokens) — the token's own UTF-8 bytes."""
    try:
        return bytes(char_to_byte[c] for c in token)
    except KeyError:
        return token.encode("utf-8")


def detokenize(ids: Sequence[int], table: Sequence[bytes], skip: Sequence[bool]) -> str:
    """batch_decode row: skip special ids, concatenate the byte strings, lossy UTF-8 decode."""
    raw = b"".join(table[i] for i in ids if not skip[i])
    return raw.decode("utf-8", "replace")
