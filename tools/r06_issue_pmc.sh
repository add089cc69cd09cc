#!/bin/bash
# One rocprofv3 --pmc pass (instruction counts; its own run) over the text leg and the API leg,
# then tools/issue_frac.py per text kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06_issue}; mkdir -p $OUT
CNT="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
timeout -s KILL 240 rocprofv3 --pmc $CNT --kernel-trace -d $OUT/text -o pmc --output-format csv \
  -- python3 tools/text_leg.py > $OUT/text.log 2>&1
rc=$?; echo "text rc=$rc" | tee -a $OUT/status.txt; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 240 rocprofv3 --pmc $CNT --kernel-trace -d $OUT/api -o pmc --output-format csv \
  -- python3 tools/api_leg.py > $OUT/api.log 2>&1
rc=$?; echo "api rc=$rc" | tee -a $OUT/status.txt; [ $rc -ne 0 ] && exit $rc
python3 tools/issue_frac.py $OUT/text "::parse_kernel(" "::detok_parse_kernel(" sokoban_token_turn_kernel > $OUT/text_issue.json
python3 tools/issue_frac.py $OUT/api bpe_encode_kernel prompt_text_kernel sokoban_token_turn_kernel > $OUT/api_issue.json
cat $OUT/text_issue.json $OUT/api_issue.json | grep -E '"(avg_us|issue_frac|valu_frac|salu_frac|launches)"|_kernel|parse' 
