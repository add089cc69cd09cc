#!/bin/bash
# Round-4 A/B session: bi-level tile depth sweep, BPE LDS diet (stamps old vs new, prompt suite),
# API phase profile + cProfile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04ab}; mkdir -p $OUT
V=ragen_amd/_build/variants
step() { echo "[$1] rc=$2" | tee -a $OUT/status.txt; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
for D in 2 4 6 8; do
  RAGEN_AMD_LIB=$V/libragen_amd_bld$D.so timeout -k 10 120 python tools/prof_bilevel.py --reps 5 --max-len 4096 > $OUT/bld$D.txt 2>&1; step bld$D $?
done
grep -h tiled $OUT/bld*.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_device_prompts.py tests/test_gpu_tokenizer.py > $OUT/pytest_bpe.log 2>&1; step pytest_bpe $?
tail -2 $OUT/pytest_bpe.log
for s in bpstold bpst; do
  export RAGEN_AMD_STAMP_SO=$V/libragen_amd_$s.so
  RAGEN_AMD_VARIANT_DIR=$V timeout -k 10 200 python tools/prof_prompt_stamps.py bpe > $OUT/stamps_$s.txt 2>&1; step stamps_$s $?
  grep call $OUT/stamps_$s.txt
done
for s in bpeold main; do
  L=$V/libragen_amd_$s.so; [ $s = main ] && L=ragen_amd/_build/libragen_amd.so
  RAGEN_AMD_LIB=$L timeout -k 10 300 python tools/api_leg.py > $OUT/api_$s.log 2>&1; step api_$s $?
  tail -1 $OUT/api_$s.log | cut -c1-200
done
timeout -k 10 200 python tools/prof_api_phases.py > $OUT/phases.txt 2>&1; step phases $?
timeout -k 10 200 python tools/prof_api_cprofile.py > $OUT/cprof.txt 2>&1; step cprof $?
echo session-done
