#!/bin/bash
# A/B of the headline step on one box: the round-1 tree (tools/_build/r01, built from commit
# 73f88e2) against the current tree, alternated, --no-extras each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-ab}; mkdir -p $OUT
for i in 1 2; do
  (cd tools/_build/r01 && timeout -k 10 300 python bench.py --steps 1000 --warmup 40 --no-cpu-baseline --no-extras) \
    > $OUT/r01_$i.log 2>&1 || { echo r01 failed; tail -5 $OUT/r01_$i.log; exit 1; }
  timeout -k 10 300 python bench.py --steps 1000 --warmup 40 --no-cpu-baseline --no-extras > $OUT/cur_$i.log 2>&1 \
    || { echo cur failed; tail -5 $OUT/cur_$i.log; exit 1; }
done
for f in $OUT/r01_1.log $OUT/cur_1.log $OUT/r01_2.log $OUT/cur_2.log; do
  python3 -c "import json,sys; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); print('$f', round(d['ms_per_step']*1e3,2), 'us/step', round(d['roofline']['avg_launch_us'],2), 'us/launch')"
done
