#!/bin/bash
# SQ instruction / wait counters of the bi-level kernels (diagnostic): two rocprofv3 --pmc
# passes (8 SQ counters each, --kernel-trace only) over tools/prof_bilevel.py.
#   bash tools/bl_pmc.sh   -> gpurun_out/blpmc/pass{1,2}
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/blpmc; mkdir -p $OUT
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" "SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace -d $OUT/pass$i -o pmc --output-format csv -- python3 tools/prof_bilevel.py --reps 5 > $OUT/pass$i.log 2>&1
  rc=$?; echo "pass$i rc=$rc" | tee -a $OUT/status.txt; [ $rc -ne 0 ] && exit $rc
done
echo done
