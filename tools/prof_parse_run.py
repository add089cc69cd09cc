"""Driver for PMC passes over rmi_parse_actions / rmi_detokenize / rmi_detok_parse
(8192 SK-shaped rows, 20 launches each)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ragen_amd import ops, synthetic

dev = torch.device("cuda", 0)
lk = {1: "Up", 2: "Down", 3: "Left", 4: "Right"}
ids, n = synthetic.rollout_actions(8192, 1, 5, 1, 4)
texts = synthetic.responses_for_actions(ids[0], n[0], lk)
buf, lens = synthetic.encode_rows(texts)
text, tl = torch.from_numpy(buf).to(dev), torch.from_numpy(lens).to(dev)
cfg = ops.parse_config(True, 5, "||", lk)
out = ops.parse_actions(cfg, text, tl)
table, skip = synthetic.byte_vocab()
vt = ops.VocabTable.from_bytes(table, skip, dev)
tok = torch.from_numpy(synthetic.tokenize_greedy(texts, table)).to(dev)
dec = ops.detokenize(tok, vt, buf.shape[1])
fused = ops.detok_parse(tok, vt, buf.shape[1], cfg)
for _ in range(20):
    ops.parse_actions(cfg, text, tl, out=out)
    ops.detokenize(tok, vt, buf.shape[1], out=dec)
    ops.detok_parse(tok, vt, buf.shape[1], cfg, out=fused)
torch.cuda.synchronize()
print("ok")
