#!/bin/bash
# A/B (diagnostic): bench.toytext_legs (FrozenLake 4096 x 8, Countdown 16384 x 4) with the default
# library and variant builds (variants/libragen_amd_NAME.so), alternating three times.
#   tools/ab_toytext.sh OUT NAME [NAME ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-abtoy}; shift; mkdir -p $OUT
for i in 1 2 3; do
  for v in default "$@"; do
    if [ $v = default ]; then L=""; else L=$PWD/variants/libragen_amd_$v.so; fi
    RAGEN_AMD_LIB=$L timeout -k 10 120 python -c "
import json, torch, bench
d = bench.toytext_legs(torch.device('cuda', 0))
print('$v', round(d['frozenlake']['ms_per_rollout'] * 1e3, 2), round(d['countdown']['ms_per_rollout'] * 1e3, 2), flush=True)
" 2>> $OUT/err.log | tee -a $OUT/ab.txt || exit 1
  done
done
