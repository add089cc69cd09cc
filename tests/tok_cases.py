"""Text cases for the device tokenizer tests: the pre-tokenizer regex's corners, added tokens,
Unicode classes, runs longer than the kernel's 64-byte view, and fuzz."""
import numpy as np

EDGE = [
    "", "a", " ", "  ", "\n", "\n\n", "\r\n", " \n", "\n ", "  x", " x", "x  ", "x \n y", "\t\tword", "a\tb",
    "it's", "IT'S", "we're", "they've", "I'm", "you'll", "he'd", "'s", "''s", "'", "x'", "'ſ", "'ST", "'LL'Ve",
    "hello world", "hello  world", "hello   world  ", "end.", "(word)", "!word", ".\nx", "a.b", "a..b", " ...\n\n",
    " -0.30000000000000004", "10.9", "-0.1", "0", "12345", "٣٤", "Ⅻ", "½", "x²",
    "café", "naïve", "中文字符", "日本語のテキスト", "Привет, мир!", "ελληνικά", "√√ √", "#_P_O#\n#__X_#",
    "😀", "a😀b", "😀😀 😀", "�", "\xa0x", "x\xa0", "　　a", "a\x85b", "\x1c\x1d", "\x00\x01",
    "<|im_start|>", "<|im_end|>", "<|endoftext|>", "<|im_start|>user\nhi<|im_end|>\n", "<|im_", "<|im_start",
    "x<|im_end|>y", "<|im_start|><|im_start|>", " <|im_end|> ", "\n<|im_start|>\n", "<think>a</think><answer>b</answer>",
    "Up || Down", "up||down||LEFT", "a" * 70, " " * 100, "-" * 90, "\n" * 70, " " * 63 + "x", "x" * 200 + " y",
    ("word " * 30).strip(), "\t" * 80 + "z", "é" * 50, "中" * 40, " " * 65 + "\n",
]


def fuzz(n: int, seed: int = 0):
    rng = np.random.default_rng(seed)
    atoms = ["a", "Z", "word", "Word", " ", "  ", "\t", "\n", "\r", "\r\n", "'s", "'t", "'re", "'LL", "'", "0", "42",
             "3.5", "-", "--", "!", "?", ".", ",", ":", "(", ")", "||", "<", ">", "/", "é", "中", "Ж", "√", "😀",
             "\xa0", "　", "\x85", "_", "#", "<|im_start|>", "<|im_end|>", "<think>", "</answer>", "٣", "½"]
    out = []
    for _ in range(n):
        k = int(rng.integers(1, 40))
        out.append("".join(atoms[int(i)] for i in rng.integers(0, len(atoms), size=k)))
    return out


def nfc_unsafe():
    return ["é", "Café au lait", "가", "Å", "Å"]
