"""Timing probe for rmi_parse_actions / rmi_detokenize under varied inputs (HIP events)."""
import sys, os, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from ragen_amd import ops, synthetic

dev = torch.device("cuda", 0)
lk = {1: "Up", 2: "Down", 3: "Left", 4: "Right"}


def t_us(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda._sleep(2_000_000)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


res = {}
for B in (1024, 8192, 32768):
    for tw in ((8, 60), (0, 2), (200, 300)):
        ids, n = synthetic.rollout_actions(B, 1, 5, 1, 4)
        texts = synthetic.responses_for_actions(ids[0], n[0], lk, think_words=tw)
        buf, lens = synthetic.encode_rows(texts)
        text, tl = torch.from_numpy(buf).to(dev), torch.from_numpy(lens).to(dev)
        for name, cfg in (("think+lookup", ops.parse_config(True, 5, "||", lk)),
                          ("think nolookup", ops.parse_config(True, 5, "||", None)),
                          ("nothink", ops.parse_config(False, 5, "||", lk))):
            out = ops.parse_actions(cfg, text, tl)
            us = t_us(lambda: ops.parse_actions(cfg, text, tl, out=out))
            res[f"B={B} words={tw} {name} stride={buf.shape[1]} bytes/row={lens.mean():.0f}"] = round(us, 2)
for k, v in res.items():
    print(f"{v:9.2f} us  {k}")
