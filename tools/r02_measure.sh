#!/bin/bash
# Round-2 measurement session: store-variant timing at 8192..4M envs, PMC traffic of the turn
# kernel at 8192 and 4M envs, and the PMC calibration kernels.  Each GPU step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r02_measure}; mkdir -p $OUT
timeout -k 10 600 python3 tools/prof_sokoban_scale.py > $OUT/scale.log 2>&1 || { echo scale failed; tail $OUT/scale.log; exit 1; }
cat $OUT/scale.log
for tile in 1 512; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $c --kernel-trace -d $OUT/t${tile}_$c -o pmc --output-format csv \
      -- python3 tools/prof_scale_pmc.py $tile > $OUT/t${tile}_$c.log 2>&1 || { echo "t$tile $c failed"; exit 1; }
  done
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d $OUT/calib_$c -o pmc --output-format csv \
    -- python3 tools/pmc_calib.py > $OUT/calib_$c.log 2>&1 || { echo "calib $c failed"; exit 1; }
done
echo measured
