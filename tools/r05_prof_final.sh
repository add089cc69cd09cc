#!/bin/bash
# Round-5 profiles: the headline bench under rocprofv3 (kernel trace + stats, --no-extras), the
# API rollout's kernel timeline and host stamps, and the BPE kernel's PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05prof}; mkdir -p $OUT
step() { echo "[$1] rc=$2" | tee -a $OUT/status.txt; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/bench -o bench --output-format csv \
  -- python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > $OUT/bench_prof.log 2>&1; step bench_prof $?
tail -1 $OUT/bench_prof.log
SKIP_PYTEST=1 bash tools/r05_check.sh ${1:-r05prof}/api "tests/test_gpu_turnglue.py"; step api_check $?
bash tools/r05_prof_host.sh ${1:-r05prof}/host; step host $?
bash tools/pmc_bpe.sh ${1:-r05prof}/pmc_bpe; step pmc_bpe $?
echo prof-done
