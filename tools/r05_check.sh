#!/bin/bash
# Round-5 GPU check: a chosen set of -m gpu tests (or all), then the API leg alone and its kernel
# timeline.  Each GPU step has its own limit; the script stops at the first failure.
#   tools/r05_check.sh OUT "tests/test_a.py tests/test_b.py"   (TESTS empty: the whole -m gpu suite)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05check}; mkdir -p $OUT
TESTS=${2:-tests}
step() { echo "[$1] rc=$2" | tee -a $OUT/status.txt; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
if [ "${SKIP_PYTEST:-0}" = "0" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; step pytest $?
  tail -3 $OUT/pytest_gpu.log
fi
if [ "${SKIP_API:-0}" = "0" ]; then
  timeout -k 10 300 python tools/api_leg.py > $OUT/api.json 2> $OUT/api.err; step api $?
  python -c "import json;d=json.load(open('$OUT/api.json'))['device_path'];print({k:d[k] for k in ('env_steps_per_s','turn_loop_s','formulate_rollouts_s','reset_s','readbacks')})"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o api --output-format csv \
    -- python3 tools/api_leg.py > $OUT/api_prof.log 2>&1; step prof_api $?
  python3 tools/api_timeline.py $OUT/prof/api_kernel_trace.csv > $OUT/api_timeline.txt; step api_timeline $?
  tail -1 $OUT/api_timeline.txt
fi
echo session-done
