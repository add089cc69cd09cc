#!/bin/bash
# Kernel stats of the API leg alone (LLMAgentProxy.rollout device path, 4 rollouts + the dict facade).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04api}; mkdir -p $OUT
step() { echo "[$1] rc=$2" | tee -a $OUT/status.txt; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o api --output-format csv \
  -- python3 tools/api_leg.py > $OUT/api.log 2>&1; step prof_api $?
tail -1 $OUT/api.log | cut -c1-300
python3 tools/api_timeline.py $OUT/prof/api_kernel_trace.csv > $OUT/api_timeline.txt; step api_timeline $?
echo session-done
