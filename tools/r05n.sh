set -u
cd "${GRAFT_REPO_ROOT}"
bash tools/r05_check.sh r05n "tests/test_gpu_turn_chain.py tests/test_gpu_device_rollout.py tests/test_gpu_device_prompts.py tests/test_gpu_val_rollout.py tests/test_gpu_facade.py" || exit $?
PROMPT=1 bash tools/r05_prof_host.sh r05n || exit $?
cat gpurun_out/r05n/prompt_stamps.txt | tail -8
