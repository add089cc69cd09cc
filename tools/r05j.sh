set -u
cd "${GRAFT_REPO_ROOT}"
bash tools/r05_check.sh r05j "tests/test_gpu_turnglue.py tests/test_gpu_turn_chain.py tests/test_gpu_device_rollout.py tests/test_gpu_device_prompts.py tests/test_gpu_val_rollout.py tests/test_gpu_tokenizer.py" || exit $?
timeout -k 10 300 python tools/bench_bpe.py > gpurun_out/r05j/bench_bpe.txt 2>&1 || exit $?
BPE=1 bash tools/r05_prof_host.sh r05j || exit $?
