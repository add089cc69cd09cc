"""Where the bench rollout with the board cache differs from the one without: eager R.step()
on both (the same rooms and actions), then the arenas, the state and the finalize outputs
compared; the first differing rows printed."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402

dev = torch.device("cuda", 0)
Rs = [bench.Rollout(dev, 0, boards=b) for b in (False, True)]
for rep in range(2):
    for R in Rs:
        R.step()
    torch.cuda.synchronize()
    a, b = Rs
    print("rep", rep, "arena equal", torch.equal(a.env.ep.arena, b.env.ep.arena),
          "state equal", torch.equal(a.env.room_state, b.env.room_state), "norm equal", torch.equal(a.norm, b.norm),
          flush=True)
    ma, mb = a.metrics.cpu().numpy(), b.metrics.cpu().numpy()
    diff = ~((ma == mb) | (np.isnan(ma) & np.isnan(mb)))
    rows = np.nonzero(diff.any(1))[0]
    print("  metric rows differing", len(rows), "nan rows", int(np.isnan(ma).any(1).sum()), int(np.isnan(mb).any(1).sum()),
          flush=True)
    for r in rows[:5]:
        print("   ", r, ma[r].tolist(), mb[r].tolist(), "n_turns", int(a.env.ep.n_turns[r]), flush=True)
