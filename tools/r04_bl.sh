#!/bin/bash
# Bi-level GAE in and out of the Infinity Cache: timing (segment / tiled kernels at 1107 columns,
# the tiled kernel at 4096) and the FETCH_SIZE / WRITE_SIZE passes of the 4096-column launch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04bl}; mkdir -p $OUT
step() { echo "[$1] rc=$2" | tee -a $OUT/status.txt; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 200 python tools/prof_bilevel.py --reps 20 > $OUT/bl_1107.txt 2>&1; step bl_1107 $?
timeout -k 10 300 python tools/prof_bilevel.py --reps 5 --max-len 4096 > $OUT/bl_4096.txt 2>&1; step bl_4096 $?
cat $OUT/bl_1107.txt $OUT/bl_4096.txt | grep -v amdgpu.ids
if [ "${PMC:-1}" = "1" ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $c --kernel-trace -d $OUT/bl4096_$c -o pmc --output-format csv \
      -- python3 tools/prof_bilevel.py --reps 3 --max-len 4096 > $OUT/bl4096_$c.log 2>&1; step "bl4096 $c" $?
  done
fi
echo session-done
