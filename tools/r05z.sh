set -u
cd "${GRAFT_REPO_ROOT}"
SKIP_API=1 bash tools/r05_check.sh r05z "tests/test_gpu_bpe_two_pass.py tests/test_gpu_tokenizer.py tests/test_gpu_turn_chain.py tests/test_gpu_device_prompts.py" || exit $?
timeout -k 10 300 python tools/bench_bpe.py > gpurun_out/r05z/bench_bpe.txt 2>&1 || exit $?; tail -1 gpurun_out/r05z/bench_bpe.txt
RAGEN_AMD_VARIANT_DIR=variants timeout -k 10 300 python tools/prof_prompt_stamps.py bpe > gpurun_out/r05z/bpe_stamps.txt 2>&1 || exit 1
tail -3 gpurun_out/r05z/bpe_stamps.txt
