#!/bin/bash
# Short GPU check: the gpu tests, then the headline bench without extras.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-quick}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -8 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-extras > "$OUT/bench.log" 2>&1
rc2=$?
tail -c 1500 "$OUT/bench.log"
exit $rc2
