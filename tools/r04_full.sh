#!/bin/bash
# Round-4 GPU session: the whole -m gpu suite, the toytext leg timing, the copy probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04full}; mkdir -p $OUT
step() { echo "[$1] rc=$2" | tee -a $OUT/status.txt; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_gpu.log 2>&1; step pytest $?
tail -3 $OUT/pytest_gpu.log
timeout -k 10 200 python tools/toy_leg.py > $OUT/toy_leg.log 2>&1; step toy_leg $?
tail -2 $OUT/toy_leg.log
if [ "${COPY_PROBE:-1}" = "1" ]; then
  hipcc --offload-arch=gfx950 -O3 -o /tmp/copy_probe tools/copy_probe.hip 2>/dev/null && timeout -k 10 120 /tmp/copy_probe > $OUT/copy_probe.json; step copy_probe $?
fi
echo session-done
