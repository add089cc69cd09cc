#!/bin/bash
# A/B (diagnostic): the bench's at-scale leg (the turn kernel on 4 194 304 envs, bench.scale_leg)
# with the default library and a variant build (RAGEN_AMD_LIB), alternating three times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VAR=$1
for i in 1 2 3; do
  for v in default $VAR; do
    if [ $v = default ]; then L=""; else L=variants/libragen_amd_$v.so; fi
    RAGEN_AMD_LIB=$L timeout -k 10 200 python3 - $v <<'PY' || exit 1
import sys, torch, bench
dev = torch.device("cuda", 0)
R = bench.Rollout(dev, 0)
R.step()
d, n = bench.scale_leg(R, dev)
print(sys.argv[1], "at_scale us/launch", round(d / bench.T_TURNS * 1e6, 1), flush=True)
PY
  done
done
