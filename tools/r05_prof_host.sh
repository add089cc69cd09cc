#!/bin/bash
# Host-side stamps of the chained API rollout (tools/prof_chain_stamps.py), optionally the BPE
# kernel's phase stamps (BPE=1: the variant libraries under variants/).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r05prof}; mkdir -p $OUT
timeout -k 10 300 python tools/prof_chain_stamps.py > $OUT/stamps.txt 2>&1 || exit $?
if [ "${BPE:-0}" = "1" ]; then
  RAGEN_AMD_VARIANT_DIR=variants timeout -k 10 300 python tools/prof_prompt_stamps.py bpe > $OUT/bpe_stamps.txt 2>&1 || exit $?
  RAGEN_AMD_STAMP_SO=variants/libragen_amd_bpstf.so timeout -k 10 300 python tools/prof_prompt_stamps.py bpe > $OUT/bpe_stamps_fine.txt 2>&1 || exit $?
fi
if [ "${PROMPT:-0}" = "1" ]; then
  RAGEN_AMD_VARIANT_DIR=variants timeout -k 10 300 python tools/prof_prompt_stamps.py prompt > $OUT/prompt_stamps.txt 2>&1 || exit $?
fi
echo done
