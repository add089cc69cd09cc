set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r05aq
SKIP_API=1 bash tools/r05_check.sh r05aq "tests/test_gpu_pad_rows.py tests/test_gpu_device_prompts.py tests/test_gpu_turn_chain.py" || exit $?
for v in "" variants/libragen_amd_oldpad.so "" variants/libragen_amd_oldpad.so; do
  RAGEN_AMD_LIB=$v timeout -k 10 120 python -u tools/bench_pad_rows.py >> gpurun_out/r05aq/ab.txt 2>> gpurun_out/r05aq/ab.err
  rc=$?; echo "[$v] rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r05aq/ab.err; exit $rc; }
done
cat gpurun_out/r05aq/ab.txt
