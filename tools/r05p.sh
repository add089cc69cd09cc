set -u
cd "${GRAFT_REPO_ROOT}"
SKIP_API=1 bash tools/r05_check.sh r05p "tests/test_gpu_tokenizer.py tests/test_gpu_device_prompts.py tests/test_gpu_turn_chain.py" || exit $?
timeout -k 10 300 python tools/bench_bpe.py > gpurun_out/r05p/bench_bpe.txt 2>&1 || exit $?
cat gpurun_out/r05p/bench_bpe.txt
bash tools/pmc_bpe.sh r05p/pmc || exit $?
BPE=1 bash tools/r05_prof_host.sh r05p || exit $?
