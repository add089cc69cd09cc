#!/bin/bash
# Round-2 closing measurement session: GPU tests, the bench line, rocprof kernel stats of the
# headline path and of all legs, PMC FETCH/WRITE passes over the bi-level kernels.  Each GPU step
# has its own limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r02final}; mkdir -p $OUT
step() { echo "[$1] rc=$2" | tee -a $OUT/status.txt; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; step pytest $?
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1; step bench $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench --output-format csv \
  -- python3 bench.py --steps 1000 --warmup 40 --no-cpu-baseline --no-extras > $OUT/prof.log 2>&1; step prof $?
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof_all -o all --output-format csv \
  -- python3 bench.py --no-cpu-baseline > $OUT/prof_all.log 2>&1; step prof_all $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d $OUT/bl_$c -o pmc --output-format csv \
    -- python3 tools/prof_bilevel.py --reps 5 > $OUT/bl_$c.log 2>&1; step "bilevel $c" $?
done
echo session-done
