set -u
cd "${GRAFT_REPO_ROOT}"
bash tools/r05_check.sh r05aa "tests/test_gpu_turn_chain.py tests/test_gpu_device_rollout.py tests/test_gpu_device_prompts.py tests/test_gpu_val_rollout.py tests/test_gpu_bpe_two_pass.py" || exit $?
grep -n "copyBuffer\|readback_kernel\|next_rows_list" gpurun_out/r05aa/api_timeline.txt | head -8
