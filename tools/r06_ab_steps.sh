#!/bin/bash
# Round 6: the slot-vector turn block (board_step.hpp) against the previous sokoban.hip
# (variants/libragen_amd_oldsk.so), alternating on one box, then the phase stamps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06_steps}; mkdir -p $OUT
step() { echo "[$1] rc=$2" | tee -a $OUT/status.txt; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
for rep in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export RAGEN_AMD_LIB=$PWD/variants/libragen_amd_oldsk.so; else unset RAGEN_AMD_LIB; fi
    timeout -k 10 240 python bench.py --no-extras --no-cpu-baseline > $OUT/bench_${v}_$rep.json 2> $OUT/bench_${v}_$rep.err; step bench_${v}_$rep $?
    python -c "import json;d=json.load(open('$OUT/bench_${v}_$rep.json'));print('$v', d['ms_per_step'], d['roofline']['avg_launch_us'])" | tee -a $OUT/ab.txt
  done
done
unset RAGEN_AMD_LIB
PROBE_SO=$PWD/variants/libragen_amd_skst.so timeout -k 10 120 python tools/prof_sokoban_stamps.py > $OUT/stamps.txt 2>&1; step stamps $?
cat $OUT/stamps.txt
echo session-done
