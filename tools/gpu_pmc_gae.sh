#!/bin/bash
# PMC passes over the GAE advantage leg (tools/prof_gae.py), one rocprofv3 run per counter set.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmcgae}
mkdir -p "$OUT"
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace -d "$OUT/pass$i" -o pmc --output-format csv \
    -- python3 tools/prof_gae.py --reps 5 > "$OUT/pass$i.log" 2>&1
  rc=$?
  echo "pass$i [$set] rc=$rc" | tee -a "$OUT/status.txt"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/pass$i.log"; exit $rc; fi
done
echo done
