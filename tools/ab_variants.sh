#!/bin/bash
# A/B of the headline step between variant builds of libragen_amd.so (tools/prof_sokoban_scale.py
# build) and the round-1 tree, alternated on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-abv}; shift; mkdir -p $OUT
VARS=${*:-"default bytestore"}
for i in 1 2; do
  (cd tools/_build/r01 && timeout -k 10 300 python bench.py --steps 1000 --warmup 40 --no-cpu-baseline --no-extras) \
    > $OUT/r01_$i.log 2>&1 || { echo r01 failed; tail -5 $OUT/r01_$i.log; exit 1; }
  for v in $VARS; do
    RAGEN_AMD_LIB=$PWD/tools/_build/libragen_amd_$v.so timeout -k 10 300 python bench.py --steps 1000 --warmup 40 \
      --no-cpu-baseline --no-extras > $OUT/${v}_$i.log 2>&1 || { echo $v failed; tail -5 $OUT/${v}_$i.log; exit 1; }
  done
done
for f in $OUT/*_[12].log; do
  python3 -c "import json; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); print('$f', round(d['ms_per_step']*1e3,2), 'us/step', round(d['roofline']['avg_launch_us'],2), 'us/launch')"
done
