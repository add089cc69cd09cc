#!/bin/bash
# Round-2 measurement session: the bench line, the rocprof kernel trace of the headline step,
# PMC FETCH/WRITE passes (headline 8192 envs, 4M envs, GAE 8192 x 4096), summaries.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r02s}
OUT=gpurun_out/$TAG; mkdir -p $OUT
step() { echo "[$1] rc=$2" | tee -a $OUT/status.txt; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1; step bench $?
tail -c 600 $OUT/bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench --output-format csv \
  -- python3 bench.py --steps 1000 --warmup 40 --no-cpu-baseline --no-extras > $OUT/prof.log 2>&1; step prof $?
for tile in 1 512; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $c --kernel-trace -d $OUT/t${tile}_$c -o pmc --output-format csv \
      -- python3 tools/prof_scale_pmc.py $tile > $OUT/t${tile}_$c.log 2>&1; step "t$tile $c" $?
  done
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c --kernel-trace -d $OUT/gae_$c -o pmc --output-format csv \
    -- python3 tools/prof_gae.py --reps 5 --cols 4096 > $OUT/gae_$c.log 2>&1; step "gae $c" $?
done
echo session-done
