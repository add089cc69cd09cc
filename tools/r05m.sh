set -u
cd "${GRAFT_REPO_ROOT}"
bash tools/r05_check.sh r05m "tests/test_gpu_turn_chain.py tests/test_gpu_device_prompts.py tests/test_gpu_device_rollout.py tests/test_gpu_val_rollout.py" || exit $?
python -c "import json;d=json.load(open('gpurun_out/r05m/api.json'))['device_path'];print(d.get('chain_padded_batches'))"
bash tools/r05_prof_host.sh r05m || exit $?
