"""Diagnostic: rmi_prompt_text alone on the API rollout's turn-``turn`` rows (bench.api_leg's
setup, 8192 envs; the chain's own program and buffers), HIP events over back-to-back launches;
the library from RAGEN_AMD_LIB (A/B variants).  Prints one JSON line."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import prof_api_cprofile as base  # noqa: E402  (the proxy, warmed up)
import torch  # noqa: E402

from ragen_amd import _lib, ops  # noqa: E402

TURN = int(sys.argv[1]) if len(sys.argv) > 1 else 2
base.run()
es = base.proxy.train_es_manager
s = es._chain.slots[TURN]
n = es.n_envs
_, _, pstride, _, _, held = s.prompt
P = ctypes.byref(held[0])
L = _lib.lib()
stream = ops._stream(s.ptext.device)


def launch():
    ops.check(L.rmi_prompt_text(P, n, s.ptext.data_ptr(), pstride, s.ptext_len.data_ptr(), s.pmark.data_ptr(),
                                s.pterr.data_ptr(), stream), "rmi_prompt_text")


launch()
torch.cuda.synchronize()
ref = (s.ptext.clone(), s.ptext_len.clone())
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda._sleep(1_000_000)
e0.record()
for _ in range(20):
    launch()
e1.record()
torch.cuda.synchronize()
print(json.dumps({"turn": TURN, "rows": n, "pstride": pstride, "us": e0.elapsed_time(e1) * 1e3 / 20,
                  "same_text": bool(torch.equal(s.ptext, ref[0]) and torch.equal(s.ptext_len, ref[1]))}))
