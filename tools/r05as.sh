set -u
cd "${GRAFT_REPO_ROOT}"
bash tools/r05_check.sh r05as "tests/test_gpu_turn_chain.py tests/test_gpu_device_rollout.py tests/test_gpu_device_prompts.py tests/test_gpu_val_rollout.py tests/test_gpu_facade.py tests/test_gpu_token_turn.py tests/test_gpu_pad_rows.py" || exit $?
