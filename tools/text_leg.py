"""Run bench.text_leg alone (the response boundary on the bench's workload: parse, decode, fused
decode + parse, the SK rollout from text and from token ids) and print its JSON.
RAGEN_AMD_PARSE1=1 selects the one-response-per-wave parse kernels."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    R = bench.Rollout(dev, 0)
    R.step()
    torch.cuda.synchronize()
    print(json.dumps(bench.text_leg(R, dev)))
