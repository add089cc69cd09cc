#!/bin/bash
# Round-4 measurement session: the -m gpu suite, the bench line, the rocprof kernel trace of the
# headline path (the exact graph-replayed bench step; reconciled with the same run's ms_per_step),
# the kernel stats of all legs, and the PMC FETCH_SIZE / WRITE_SIZE passes of the headline
# kernel (bench shape and 4 M envs).  Each GPU step has its own limit; the script stops at the
# first failure.  Raw CSVs the summaries cite are kept under $OUT (copied into profiles/).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04p}; mkdir -p $OUT
step() { echo "[$1] rc=$2" | tee -a $OUT/status.txt; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; step pytest $?
  tail -2 $OUT/pytest_gpu.log
fi
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1; step bench $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench --output-format csv \
  -- python3 bench.py --steps 200 --warmup 40 --no-cpu-baseline --no-extras > $OUT/prof.log 2>&1; step prof $?
python3 tools/trace_reconcile.py $OUT/prof $OUT/prof.log $OUT/trace_reconcile.json > /dev/null; step reconcile $?
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof_all -o all --output-format csv \
  -- python3 bench.py --no-cpu-baseline > $OUT/prof_all.log 2>&1; step prof_all $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d $OUT/sk_$c -o pmc --output-format csv \
    -- python3 tools/prof_sokoban.py --reps 20 > $OUT/sk_$c.log 2>&1; step "sokoban $c" $?
  timeout -s KILL 180 rocprofv3 --pmc $c --kernel-trace -d $OUT/t512_$c -o pmc --output-format csv \
    -- python3 tools/prof_scale_pmc.py 512 > $OUT/t512_$c.log 2>&1; step "scale $c" $?
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_api -o api --output-format csv \
  -- python3 tools/api_leg.py > $OUT/api.log 2>&1; step prof_api $?
python3 tools/api_timeline.py $OUT/prof_api/api_kernel_trace.csv > $OUT/api_timeline.txt; step api_timeline $?
echo session-done
