"""A byte-level stand-in for the Qwen2.5 tokenizer (the hub model is unavailable offline):
the chat template and the <|im_start|> / <|im_end|> ids of Qwen, one id per other character."""
import torch


class FakeQwenTok:
    name_or_path = "Qwen/Qwen2.5-0.5B-Instruct"
    IM_START, IM_END, PAD = 151644, 151645, 151643
    pad_token_id = 151643
    ADDED = {"<|im_start|>": IM_START, "<|im_end|>": IM_END}

    def encode(self, text):
        return {"<|im_start|>": [self.IM_START], "<|im_end|>": [self.IM_END]}[text]

    def apply_chat_template(self, messages, add_generation_prompt, tokenize):
        s = "".join(f"<|im_start|>{m['role']}\n{m['content']}<|im_end|>\n" for m in messages)
        return s + ("<|im_start|>assistant\n" if add_generation_prompt else "")

    def _ids(self, text):
        out, i = [], 0
        while i < len(text):
            hit = next((t for t in self.ADDED if text.startswith(t, i)), None)
            if hit is not None:
                out.append(self.ADDED[hit])
                i += len(hit)
            else:
                out.append(ord(text[i]) % 150000)
                i += 1
        return out

    def __call__(self, texts, return_tensors="pt", padding=True, padding_side="left", truncation=False):
        rows = [self._ids(t) for t in texts]
        if not padding:  # ragged rows, as a HF tokenizer's padding=False
            o = type("Enc", (), {})()
            o.input_ids = rows
            return o
        L = max(len(r) for r in rows)
        ids = torch.full((len(rows), L), self.PAD, dtype=torch.long)
        am = torch.zeros((len(rows), L), dtype=torch.long)
        for b, r in enumerate(rows):
            ids[b, L - len(r):] = torch.tensor(r)
            am[b, L - len(r):] = 1

        class O:
            pass
        o = O()
        o.input_ids, o.attention_mask = ids, am
        return o

    def decode(self, ids, skip_special_tokens=True):
        drop = set(self.ADDED.values()) | {self.PAD} if skip_special_tokens else set()
        return "".join(chr(int(i)) for i in ids if int(i) not in drop)

    def batch_decode(self, rows, skip_special_tokens=True):
        return [self.decode(r.tolist() if hasattr(r, "tolist") else r, skip_special_tokens) for r in rows]

    def byte_table(self, V=151646):
        """(table, skip) for ops.VocabTable.from_bytes: id -> UTF-8 of chr(id), as decode() does."""
        table = []
        for i in range(V):
            try:
                table.append(chr(i).encode("utf-8"))
            except UnicodeEncodeError:  # surrogates
                table.append(b"")
        special = set(self.ADDED.values()) | {self.PAD}
        skip = [1 if i in special else 0 for i in range(V)]
        return table, skip

    _backend = None

    @property
    def backend_tokenizer(self):
        """The same encoding as a `tokenizers` byte-level BPE (what the device prompt path reads,
        ragen_amd.tokenizer.DeviceTokenizer.from_hf): one pre-token per character, merges that
        rebuild every Basic-Multilingual-Plane character from its UTF-8 bytes into the id
        ord(c) % 150000, and <|im_start|> / <|im_end|> as added tokens.  Checked against _ids by
        tests/test_tokenizer.py."""
        if type(self)._backend is None:
            type(self)._backend = _char_bpe(self.ADDED)
        return type(self)._backend


def _char_bpe(added):
    """added: {token text: id} of the added (special) tokens."""
    import json

    from tokenizers import Tokenizer
    from ragen_amd.tokenizer import bytes_to_unicode
    b2u = bytes_to_unicode()
    vocab, merges = {}, []
    for b in range(256):
        vocab[b2u[b]] = b if b < 0x80 else 150000 + b
    nxt = 150256
    for c in range(0x80, 0x10000):
        if 0xD800 <= c <= 0xDFFF:
            continue
        bs = chr(c).encode("utf-8")
        syms = [b2u[x] for x in bs]
        cur = syms[0]
        for k, s in enumerate(syms[1:], 1):
            tok = cur + s
            if tok not in vocab:
                vocab[tok] = (c % 150000) if k == len(syms) - 1 else nxt
                if k < len(syms) - 1:
                    nxt += 1
                merges.append([cur, s])
            cur = tok
    # the added tokens hold their Qwen ids in the model vocabulary too (else tokenizers renumbers
    # them past the vocabulary); unused ids get placeholder tokens (no holes in the id space)
    vocab.update(added)
    used = set(vocab.values())
    for i in range(max(used) + 1):
        if i not in used:
            vocab[f"<unused_{i}>"] = i
    j = {"version": "1.0", "truncation": None, "padding": None,
         "added_tokens": [{"id": i, "content": t, "single_word": False, "lstrip": False, "rstrip": False,
                           "normalized": False, "special": True}
                          for t, i in added.items()],
         "normalizer": None,
         "pre_tokenizer": {"type": "Sequence", "pretokenizers": [
             {"type": "Split", "pattern": {"Regex": "."}, "behavior": "Isolated", "invert": False},
             {"type": "ByteLevel", "add_prefix_space": False, "trim_offsets": False, "use_regex": False}]},
         "post_processor": None, "decoder": {"type": "ByteLevel", "add_prefix_space": False, "trim_offsets": False,
                                             "use_regex": False},
         "model": {"type": "BPE", "dropout": None, "unk_token": None, "continuing_subword_prefix": None,
                   "end_of_word_suffix": None, "fuse_unk": False, "byte_fallback": False, "ignore_merges": False,
                   "vocab": vocab, "merges": merges}}
    return Tokenizer.from_str(json.dumps(j))


class FakeLlama3Tok(FakeQwenTok):
    """The same byte-level stand-in under a Llama-3 name: get_special_tokens' second branch
    (ctx_manager.py:27-29, ids 128006 / 128009, no Qwen roll), the Llama-3 chat layout
    (<|begin_of_text|>, <|start_header_id|> role <|end_header_id|> \\n\\n content <|eot_id|>) and its
    special ids; other characters keep the id ord(c) % 150000 (below 128000 for the BMP text of
    these tests)."""
    name_or_path = "meta-llama/Meta-Llama-3-8B-Instruct"
    BOT, IM_START, EH, IM_END, PAD = 128000, 128006, 128007, 128009, 128001
    pad_token_id = 128001
    ADDED = {"<|begin_of_text|>": BOT, "<|start_header_id|>": IM_START, "<|end_header_id|>": EH,
             "<|eot_id|>": IM_END}
    _backend = None

    def encode(self, text):
        raise AssertionError("the Llama-3 branch of get_special_tokens calls no encode")

    def apply_chat_template(self, messages, add_generation_prompt, tokenize):
        s = "<|begin_of_text|>" + "".join(
            f"<|start_header_id|>{m['role']}<|end_header_id|>\n\n{m['content']}<|eot_id|>" for m in messages)
        return s + ("<|start_header_id|>assistant<|end_header_id|>\n\n" if add_generation_prompt else "")
