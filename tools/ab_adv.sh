#!/bin/bash
# A/B (diagnostic): the bench's advantage legs with the default library and a variant build
# (RAGEN_AMD_LIB), alternating twice; prints GAE / bi-level in- and out-of-cache times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-abadv}; VAR=$2; mkdir -p $OUT
for i in 1 2; do
  for v in default $VAR; do
    if [ $v = default ]; then L=""; else L=variants/libragen_amd_$v.so; fi
    RAGEN_AMD_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/$v.$i.log 2>&1 || exit 1
    python3 - $OUT/$v.$i.log $v <<'PY'
import json, sys
l = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); a = l["advantage"]
print(sys.argv[2], "gae", round(a["gae_us"], 1), "gae_ooc", round(a["out_of_cache"]["gae_us"], 1),
      "bl", round(a["bilevel_gae"]["us"], 1), "bl_ooc", round(a["bilevel_gae"]["out_of_cache"]["us"], 1),
      "grpo", round(a["grpo"]["us"], 1), "masks", round(a["masks_and_scores"]["us"], 1), flush=True)
PY
  done
done
