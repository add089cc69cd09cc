#!/bin/bash
# Round-4 session 4: device suites, API leg, host gaps, BPE stamps (coarse + fine).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04ab4}; mkdir -p $OUT
V=ragen_amd/_build/variants
step() { echo "[$1] rc=$2" | tee -a $OUT/status.txt; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_device_prompts.py tests/test_gpu_tokenizer.py tests/test_gpu_device_rollout.py > $OUT/pytest_dev.log 2>&1; step pytest_dev $?
tail -1 $OUT/pytest_dev.log
timeout -k 10 300 python tools/api_leg.py > $OUT/api.log 2>&1; step api $?
tail -1 $OUT/api.log | cut -c1-300
timeout -k 10 300 python tools/prof_host_gaps.py > $OUT/gaps.txt 2>&1; step gaps $?
grep -v amdgpu.ids $OUT/gaps.txt
for s in bpst bpfine; do
  RAGEN_AMD_STAMP_SO=$V/libragen_amd_$s.so timeout -k 10 200 python tools/prof_prompt_stamps.py bpe > $OUT/stamps_$s.txt 2>&1; step stamps_$s $?
  grep call $OUT/stamps_$s.txt | cut -c1-330
done

RAGEN_AMD_STAMP_SO=$V/libragen_amd_prst.so timeout -k 10 200 python tools/prof_prompt_stamps.py prompt > $OUT/stamps_prompt.txt 2>&1; step stamps_prompt $?
grep call $OUT/stamps_prompt.txt | cut -c1-330
echo session-done
