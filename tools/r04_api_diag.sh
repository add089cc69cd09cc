#!/bin/bash
# API-leg diagnosis: host cProfile of one device-path rollout and the per-phase wall times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04apidiag}; mkdir -p $OUT
step() { echo "[$1] rc=$2" | tee -a $OUT/status.txt; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 300 python tools/prof_api_cprofile.py > $OUT/cprofile.txt 2>&1; step cprofile $?
timeout -k 10 300 python tools/prof_api_phases.py > $OUT/phases.txt 2>&1; step phases $?
echo session-done
