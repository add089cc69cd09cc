set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r05ai
for v in "" variants/libragen_amd_tok_noturn.so variants/libragen_amd_tok_norender.so variants/libragen_amd_tok_neither.so ""; do
  RAGEN_AMD_LIB=$v timeout -k 10 120 python -u tools/bench_token_turn.py >> gpurun_out/r05ai/ab.txt 2>> gpurun_out/r05ai/ab.err
  rc=$?; echo "[$v] rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r05ai/ab.err; exit $rc; }
done
cat gpurun_out/r05ai/ab.txt
