#!/bin/bash
# Round-6 GPU check: chosen -m gpu tests, then optional extra commands given in EXTRA (each run
# under its own time limit by the caller).  Stops at the first failure.
#   tools/r06_check.sh OUT "tests/test_a.py tests/test_b.py"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06check}; mkdir -p $OUT
TESTS=${2:-tests}
step() { echo "[$1] rc=$2" | tee -a $OUT/status.txt; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; step pytest $?
  tail -3 $OUT/pytest_gpu.log
fi
if [ "${BENCH:-0}" = "1" ]; then
  timeout -k 10 300 python bench.py --no-extras --no-cpu-baseline > $OUT/bench_noextras.json 2> $OUT/bench_noextras.err; step bench $?
  python -c "import json;d=json.load(open('$OUT/bench_noextras.json'));print({k:d[k] for k in ('value','ms_per_step')}, d['roofline']['avg_launch_us'])"
fi
if [ "${DB:-0}" = "1" ]; then
  timeout -k 10 300 python bench.py --no-extras --no-cpu-baseline --double-buffer > $OUT/bench_db.json 2> $OUT/bench_db.err; step bench_db $?
  python -c "import json;d=json.load(open('$OUT/bench_db.json'));print({k:d[k] for k in ('value','ms_per_step','exchange_variants_ms_per_rollout','gathered')}, d['config']['exchange_transport'])"
fi
echo session-done
