#!/bin/bash
# Round-4 (second session) GPU check: the -m gpu suite (first failure stops), smoke, the bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04s2}; mkdir -p $OUT
step() { echo "[$1] rc=$2" | tee -a $OUT/status.txt; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_gpu.log 2>&1; step pytest $?
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; step smoke $?
if [ "${SKIP_BENCH:-0}" = "0" ]; then
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > $OUT/bench.log 2>&1; step bench $?
  tail -1 $OUT/bench.log | cut -c1-400
fi
echo session-done
