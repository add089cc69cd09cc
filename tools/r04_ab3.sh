#!/bin/bash
# Round-4 session 3: host primitive costs, device rollout / prompt / tokenizer suites, the API leg
# (plain and under a kernel trace), BPE stamps (coarse + fine).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04ab3}; mkdir -p $OUT
V=ragen_amd/_build/variants
step() { echo "[$1] rc=$2" | tee -a $OUT/status.txt; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 120 python tools/prof_prims.py > $OUT/prims.txt 2>&1; step prims $?
grep -v amdgpu.ids $OUT/prims.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_device_prompts.py tests/test_gpu_tokenizer.py tests/test_gpu_device_rollout.py > $OUT/pytest_dev.log 2>&1; step pytest_dev $?
tail -1 $OUT/pytest_dev.log
timeout -k 10 300 python tools/api_leg.py > $OUT/api.log 2>&1; step api $?
tail -1 $OUT/api.log | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o api --output-format csv -- python3 tools/api_leg.py > $OUT/api_prof.log 2>&1; step prof_api $?
for s in bpst bpfine; do
  RAGEN_AMD_STAMP_SO=$V/libragen_amd_$s.so timeout -k 10 200 python tools/prof_prompt_stamps.py bpe > $OUT/stamps_$s.txt 2>&1; step stamps_$s $?
  grep call $OUT/stamps_$s.txt | cut -c1-330
done
echo session-done
