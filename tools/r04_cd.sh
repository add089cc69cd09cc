#!/bin/bash
# Round-4 Countdown big-int check: the Countdown GPU tests, the toytext leg timing, the copy probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04cd}; mkdir -p $OUT
step() { echo "[$1] rc=$2" | tee -a $OUT/status.txt; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_countdown_bigint.py tests/test_gpu_parity.py tests/test_gpu_facade.py tests/test_gpu_configs.py -k "countdown or Countdown" -v -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_cd.log 2>&1; step pytest_cd $?
tail -3 $OUT/pytest_cd.log
timeout -k 10 200 python tools/toy_leg.py > $OUT/toy_leg.log 2>&1; step toy_leg $?
tail -5 $OUT/toy_leg.log
if [ "${COPY_PROBE:-1}" = "1" ]; then
  hipcc --offload-arch=gfx950 -O3 -o /tmp/copy_probe tools/copy_probe.hip 2>/dev/null && timeout -k 10 120 /tmp/copy_probe > $OUT/copy_probe.json; step copy_probe $?
fi
echo session-done
