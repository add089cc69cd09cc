"""Wave timelines of rmi_detokenize and rmi_parse_actions (diagnostic, not product).

Builds parse.hip with RMI_PARSE_STAMPS into tools/_build/libparse_stamps.so and runs both kernels
on the bench's shapes (text_leg: 8192 responses; detokenize of [8192, 128] random ids over a
151 646-token vocabulary, and of the greedy byte-vocab tokenization of the responses).  Per
launch it prints the event time, the grid span from the waves' s_memrealtime stamps (100 MHz),
the spread of the wave start times, the mean wave duration, and the mean s_memtime cycles of
each phase:
  detok: ids landed | offsets landed | bytes placed | validity | stored
  parse: stage | events | match | strip | split | stores"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from ragen_amd import _lib, ops, synthetic  # noqa: E402

OUT = os.path.join(ROOT, "tools", "_build")
SO = os.path.join(OUT, "libparse_stamps.so")
SRC = os.path.join(ROOT, "ragen_amd", "csrc", "parse.hip")
if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(SRC):
    os.makedirs(OUT, exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "-x", "hip", "--offload-arch=gfx950", "-O3",
                    "-std=c++17", "-ffp-contract=off", "-DRMI_PARSE_STAMPS", "-I", os.path.join(ROOT, "include"),
                    "-I", os.path.join(ROOT, "ragen_amd", "csrc"), SRC, "-o", SO], check=True)
if len(sys.argv) > 1 and sys.argv[1] == "build":
    sys.exit(0)
L = ctypes.CDLL(SO)
fp = L.rmi_parse_actions
fp.restype = ctypes.c_int32
fp.argtypes = _lib._SIGS["rmi_parse_actions"][1]
fd = L.rmi_detokenize
fd.restype = ctypes.c_int32
fd.argtypes = _lib._SIGS["rmi_detokenize"][1]
dev = torch.device("cuda", 0)
stream = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731


def timeline(st, n_phase, names, rt_cols, label, ev_us):
    s = st.cpu().numpy().astype(np.float64)
    rt0, rt1 = s[:, rt_cols[0]], s[:, rt_cols[1]]
    span_us = (rt1.max() - rt0.min()) / 100.0
    starts = (rt0 - rt0.min()) / 100.0
    dur = (rt1 - rt0) / 100.0
    d = np.diff(s[:, :n_phase + 1], axis=1)
    print(f"{label}: event {ev_us:.1f} us | grid span {span_us:.1f} us | wave starts p10/p50/p90/max "
          f"{np.percentile(starts, 10):.1f}/{np.percentile(starts, 50):.1f}/{np.percentile(starts, 90):.1f}/"
          f"{starts.max():.1f} us | wave duration mean {dur.mean():.2f} us (p90 {np.percentile(dur, 90):.2f})")
    print("   cycles: " + "  ".join(f"{nm}={d[:, i].mean():.0f}" for i, nm in enumerate(names)))


def timed(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    torch.cuda._sleep(2_000_000)
    e[0].record()
    for _ in range(reps):
        fn()
    e[1].record()
    torch.cuda.synchronize()
    return e[0].elapsed_time(e[1]) * 1e3 / reps


def run_detok(tok, vt, stride, label):
    B, R = tok.shape
    out = torch.zeros(B, stride, dtype=torch.uint8, device=dev)
    ln = torch.zeros(B, dtype=torch.int32, device=dev)
    err = torch.zeros(B, dtype=torch.uint8, device=dev)
    st = torch.zeros(B, 8, dtype=torch.int64, device=dev)
    L.rmi_detok_set_stamps(ctypes.c_void_p(st.data_ptr()))

    def go():
        rc = fd(tok.data_ptr(), B, R, None, vt.packed.data_ptr(), vt.data.data_ptr(), vt.data.numel(),
                vt.packed.shape[0], out.data_ptr(), stride, ln.data_ptr(), err.data_ptr(), stream())
        assert rc == 0, rc
    us = timed(go)
    go()
    torch.cuda.synchronize()
    timeline(st, 5, ["ids", "offsets", "bytes", "validity", "stored"], (6, 7), label, us)
    return out, ln


def run_parse(text, tl, think, label):
    B = text.shape[0]
    lk = {1: "Up", 2: "Down", 3: "Left", 4: "Right"}
    cfg = ops.parse_config(think, 5, "||", lk)
    o = ops.parse_actions(cfg, text, tl)
    st = torch.zeros(B, 12, dtype=torch.int64, device=dev)
    L.rmi_parse_set_stamps(ctypes.c_void_p(st.data_ptr()))

    def go():
        rc = fp(ctypes.byref(cfg), text.data_ptr(), tl.data_ptr(), B, text.shape[1], None, o["actions"].data_ptr(),
                o["n_actions"].data_ptr(), o["spans"].data_ptr(), None, None, 0, o["err"].data_ptr(), stream())
        assert rc == 0, rc
    us = timed(go)
    go()
    torch.cuda.synchronize()
    timeline(st, 6, ["stage", "events", "match", "strip", "split", "stores"], (10, 11), label, us)


def main():
    B, K = 8192, 5
    lk = {1: "Up", 2: "Down", 3: "Left", 4: "Right"}
    ids, n = synthetic.rollout_actions(B, 1, K, 1, 4)
    texts = synthetic.responses_for_actions(ids[0], n[0], lk, seed=100)
    buf, lens = synthetic.encode_rows(texts)
    text, tl = torch.from_numpy(buf).to(dev), torch.from_numpy(lens).to(dev)
    for B_ in (1024, 8192):
        run_parse(text[:B_].contiguous(), tl[:B_].contiguous(), True, f"parse B={B_} stride={buf.shape[1]}")
    # detokenize: the bench's Qwen-sized random vocabulary, and the byte vocab of the token rollout
    V, Rt = 151646, 128
    rng = np.random.default_rng(5)
    lens_v = rng.integers(1, 9, size=V)
    data = rng.integers(97, 123, size=int(lens_v.sum())).astype(np.uint8)
    off = np.zeros(V + 1, np.int64)
    np.cumsum(lens_v, out=off[1:])
    skip = np.zeros(V, np.uint8)
    skip[151643:] = 1
    vt = ops.VocabTable(torch.from_numpy(off).to(dev), torch.from_numpy(data).to(dev), torch.from_numpy(skip).to(dev))
    tok = torch.from_numpy(rng.integers(0, 151643, size=(B, Rt)).astype(np.int64)).to(dev)
    for B_ in (1024, 8192):
        run_detok(tok[:B_].contiguous(), vt, 2048, f"detok random B={B_} R={Rt}")
    table, sk = synthetic.byte_vocab()
    tv = ops.VocabTable.from_bytes(table, sk, dev)
    tt = torch.from_numpy(synthetic.tokenize_greedy(texts, table)).to(dev)
    out, ln = run_detok(tt, tv, buf.shape[1], f"detok byte-vocab B={B} R={tt.shape[1]}")
    assert torch.equal(ln, tl)
    # the fused kernel (library build, no stamps) on the same token rows
    cfg = ops.parse_config(True, K, "||", lk)
    fo = ops.detok_parse(tt, tv, buf.shape[1], cfg)
    us = timed(lambda: ops.detok_parse(tt, tv, buf.shape[1], cfg, out=fo))
    print(f"detok_parse byte-vocab B={B} R={tt.shape[1]}: event {us:.1f} us")


if __name__ == "__main__":
    main()
