set -u
cd "${GRAFT_REPO_ROOT}"
bash tools/r05_check.sh r05x "tests/test_gpu_turn_chain.py tests/test_gpu_device_prompts.py tests/test_gpu_prompt_staging.py tests/test_gpu_device_rollout.py" || exit $?
timeout -k 10 200 python tools/bench_prompt.py > gpurun_out/r05x/prompt.txt 2>&1 || exit 1; tail -1 gpurun_out/r05x/prompt.txt
grep -n "prompt_text" gpurun_out/r05x/api_timeline.txt | head -6
