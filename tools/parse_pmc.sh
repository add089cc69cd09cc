#!/bin/bash
# SQ instruction / wait counters of the response-boundary kernels (diagnostic): two rocprofv3
# --pmc passes (8 SQ counters each, --kernel-trace only) over tools/prof_parse_run.py, then the
# per-wave means per kernel.   bash tools/parse_pmc.sh [tag]  -> gpurun_out/<tag>/pass{1,2}
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-parsepmc}; mkdir -p $OUT
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" "SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace -d $OUT/pass$i -o pmc --output-format csv -- python3 tools/prof_parse_run.py > $OUT/pass$i.log 2>&1
  rc=$?; echo "pass$i rc=$rc" | tee -a $OUT/status.txt; [ $rc -ne 0 ] && exit $rc
done
python3 tools/pmc_per_wave.py $OUT parse_kernel detok_kernel detok_parse_kernel parse4_kernel detok_parse4_kernel
