#!/bin/bash
# Round-3 GPU check: the -m gpu suite, smoke, and the default bench line.  Each GPU step has
# its own limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03check}; mkdir -p $OUT
step() { echo "[$1] rc=$2" | tee -a $OUT/status.txt; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; step pytest $?
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; step smoke $?
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1; step bench $?
tail -1 $OUT/bench.log
echo session-done
