set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r05y
RAGEN_AMD_VARIANT_DIR=variants timeout -k 10 300 python tools/prof_prompt_stamps.py bpe > gpurun_out/r05y/bpe_stamps.txt 2>&1 || exit 1
RAGEN_AMD_STAMP_SO=variants/libragen_amd_bpstf.so timeout -k 10 300 python tools/prof_prompt_stamps.py bpe > gpurun_out/r05y/bpe_stamps_fine.txt 2>&1 || exit 1
tail -3 gpurun_out/r05y/bpe_stamps.txt; tail -3 gpurun_out/r05y/bpe_stamps_fine.txt
