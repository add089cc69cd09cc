"""Diagnostic: rmi_bpe_encode alone on the API rollout's real turn text (bench.api_leg's setup:
8192 envs, the Qwen2-pipeline BPE): the prompt text rows one chained turn wrote (slot --turn),
encoded into a scratch arena with HIP events around back-to-back launches, at the launch's own
row bound and at tighter ones (the LDS a wave takes grows with the bound: fewer waves per CU).
Also the word cache cold vs warm.  Prints one JSON line."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import prof_api_cprofile as base  # noqa: E402  (the proxy, warmed up)
import torch  # noqa: E402

from ragen_amd import _lib, ops  # noqa: E402

TURN = int(sys.argv[1]) if len(sys.argv) > 1 else 2
PMC = len(sys.argv) > 2 and sys.argv[2] == "pmc"  # (rocprofv3 --pmc: 10 launches at the bound only)
base.run()
es = base.proxy.train_es_manager
ch = es._chain
s = ch.slots[TURN]
pr = ch.pr
n = es.n_envs
text, tlen = s.ptext, s.ptext_len
bound = s.prompt[3]
longest = int(tlen.max())
pr.dt.ensure_two_pass(es.n_envs, 3072)  # (both forms timed below)
tok = pr.dt.bpe_struct(True)
dev = text.device
out = torch.zeros(n, 2048, dtype=torch.int64, device=dev)
out_len = torch.zeros(n, dtype=torch.int32, device=dev)
mark_tok = torch.empty(n, dtype=torch.int32, device=dev)
err = torch.empty(n, dtype=torch.uint8, device=dev)
L = _lib.lib()
stream = ops._stream(dev)


def launch(stride, st=None):
    out_len.zero_()
    ops.check(L.rmi_bpe_encode(ctypes.addressof(st or tok), text.data_ptr(), int(text.shape[1]), int(stride),
                               tlen.data_ptr(), n, out.data_ptr(), 2048, out_len.data_ptr(), None,
                               s.pmark.data_ptr(), mark_tok.data_ptr(), err.data_ptr(), stream), "rmi_bpe_encode")


def timed(stride, reps=20, st=None):
    launch(stride, st)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(1_000_000)
    e0.record()
    for _ in range(reps):
        launch(stride, st)
    e1.record()
    torch.cuda.synchronize()
    # (each launch also zeroes out_len: a 32 KB fill, ~2 us)
    return e0.elapsed_time(e1) * 1e3 / reps


if PMC:  # (the one-kernel form, as the turn chain runs it)
    one_pmc = pr.dt.bpe_struct(False)
    torch.cuda.synchronize()
    for _ in range(10):
        launch(bound, one_pmc)
    torch.cuda.synchronize()
    print(json.dumps({"turn": TURN, "rows": n, "bound": bound, "text_bytes": int(tlen.sum()), "launches": 10}))
    sys.exit(0)
ref_ids = None
res = {"turn": TURN, "rows": n, "bound": bound, "longest_row": longest, "mean_row": float(tlen.float().mean()),
       "text_bytes": int(tlen.sum()), "n_added": int(tok.n_added), "n_exp": int(tok.n_exp),
       "n_exp_ids": int(tok.n_exp_ids)}
launch(bound)
torch.cuda.synchronize()
ref = (out.clone(), out_len.clone(), err.clone())
strides = sorted({bound, (longest + 3) // 4 * 4, 448, 384, 320})
res["us_at_stride"] = {}
for st in strides:
    us = timed(st)
    launch(st)
    torch.cuda.synchronize()
    ok = int((err == 0).sum())
    same = bool(torch.equal(out_len[err == 0], ref[1][err == 0]))
    res["us_at_stride"][st] = {"us": us, "rows_encoded": ok, "same_lengths": same}
# the one-kernel form at the bound (the struct without the two-pass scratch), same outputs
one = pr.dt.bpe_struct(False)
res["two_pass"] = tok.pre is not None and tok.pre_cap > 0
res["us_one_kernel_at_bound"] = timed(bound, st=one)
launch(bound, one)
torch.cuda.synchronize()
res["one_kernel_same_ids"] = bool(torch.equal(out_len, ref[1]) and torch.equal(err, ref[2]) and all(
    torch.equal(out[i, :int(ref[1][i])], ref[0][i, :int(ref[1][i])]) for i in range(0, n, 97)))
# the word cache cold (cleared) for one launch at the bound
if pr.dt.word_cache is not None:
    wc = pr.dt.word_cache
    saved = wc.clone()
    wc.zero_()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    launch(bound)
    e1.record()
    torch.cuda.synchronize()
    res["us_cold_cache_one_launch"] = e0.elapsed_time(e1) * 1e3
    wc.copy_(saved)
print(json.dumps(res))
