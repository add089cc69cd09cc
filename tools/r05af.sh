set -u
cd "${GRAFT_REPO_ROOT}"
bash tools/r05_check.sh r05af "tests/test_gpu_turn_chain.py tests/test_gpu_device_rollout.py tests/test_gpu_device_prompts.py tests/test_gpu_val_rollout.py tests/test_gpu_facade.py" || exit $?
bash tools/r05_prof_host.sh r05af/host || exit $?
grep -A10 "per label" gpurun_out/r05af/host/stamps.txt | head -12
