set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r05ap
SKIP_API=1 bash tools/r05_check.sh r05ap "tests/test_gpu_parse.py tests/test_gpu_token_turn.py tests/test_gpu_device_rollout.py tests/test_gpu_device_prompts.py tests/test_gpu_turn_chain.py tests/test_gpu_configs.py" || exit $?
timeout -k 10 120 python -u tools/bench_token_turn.py > gpurun_out/r05ap/ab.txt 2> gpurun_out/r05ap/ab.err
rc=$?; echo "[ab] rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r05ap/ab.err; exit $rc; }
cat gpurun_out/r05ap/ab.txt
