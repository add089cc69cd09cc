set -u
cd "${GRAFT_REPO_ROOT}"
bash tools/r05_check.sh r05v "tests/test_gpu_bpe_two_pass.py tests/test_gpu_turn_chain.py tests/test_gpu_tokenizer.py tests/test_gpu_device_prompts.py tests/test_gpu_device_rollout.py tests/test_gpu_val_rollout.py" || exit $?
grep -n "bpe\|prompt_text\|pad_rows" gpurun_out/r05v/api_timeline.txt | head -12
timeout -k 10 300 python tools/bench_bpe.py > gpurun_out/r05v/bench_bpe.txt 2>&1 || exit $?; tail -1 gpurun_out/r05v/bench_bpe.txt
bash tools/r05_prof_host.sh r05v || exit $?
