#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the turn kernel at 1M envs (each counter its own pass)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-scale_pmc}; mkdir -p $OUT
timeout -k 10 120 python3 tools/prof_scale_pmc.py > $OUT/plain.log 2>&1 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d $OUT/$c -o pmc --output-format csv \
    -- python3 tools/prof_scale_pmc.py > $OUT/$c.log 2>&1 || { echo "$c failed"; exit 1; }
done
echo ok
