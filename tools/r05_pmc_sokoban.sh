#!/bin/bash
# PMC counter passes over the Sokoban rollout (each pass its own rocprofv3 run, --kernel-trace only).
# usage: bash tools/gpu_pmc.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-pmc}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace -d "$OUT/pass$i" -o pmc --output-format csv \
    -- python3 tools/prof_sokoban.py --reps 20 > "$OUT/pass$i.log" 2>&1
  rc=$?
  echo "pass$i [$set] rc=$rc" | tee -a "$OUT/status.txt"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/pass$i.log"; [ $rc -ge 124 ] && exit $rc; fi
done
python3 tools/pmc_summary.py "$OUT" "$OUT/pmc_sokoban_step_turn.json"
echo done
