"""Micro-bench (diagnostic) of rmi_pad_rows: the generation batch (input_ids, attention_mask,
position_ids i64[8192, S]) from arena rows + a tail, at the S of the API rollout's turns.
Library from RAGEN_AMD_LIB (tools/build_variant.sh variants).  Prints us per launch and GB/s."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ragen_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
n, cap = 8192, 2048
g = torch.Generator(device="cpu").manual_seed(0)
arena = torch.randint(0, 150000, (n, cap), generator=g, dtype=torch.int64).to(dev)
tail = torch.tensor([151644, 77091, 198], dtype=torch.int64, device=dev)
rows = torch.arange(n, dtype=torch.int64, device=dev)
out = {}
for S in (160, 500, 700, 1001, 1100):
    alen = (S - 3 - torch.randint(0, 40, (n,), generator=g)).clamp(min=1).to(torch.int32).to(dev)
    for _ in range(3):
        ops.pad_rows(arena, alen, rows, tail, S, 151643)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    keep = []
    ev[0].record()
    for _ in range(20):
        keep.append(ops.pad_rows(arena, alen, rows, tail, S, 151643))
        if len(keep) > 2:
            keep.pop(0)
    ev[1].record()
    torch.cuda.synchronize()
    us = ev[0].elapsed_time(ev[1]) * 1e3 / 20
    byt = n * S * 24 + int(alen.sum()) * 8
    out[S] = (round(us, 1), round(byt / us / 1e3, 0))
print(os.path.basename(os.environ.get("RAGEN_AMD_LIB", "default")), json.dumps(out))
