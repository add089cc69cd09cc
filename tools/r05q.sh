set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r05q
for v in default bpe_noexp bpe_oneprobe bpe_both; do
  if [ $v = default ]; then L=ragen_amd/_build/libragen_amd.so; else L=variants/libragen_amd_$v.so; fi
  RAGEN_AMD_LIB=$L timeout -k 10 300 python tools/bench_bpe.py > gpurun_out/r05q/$v.txt 2>&1 || { tail -5 gpurun_out/r05q/$v.txt; exit 1; }
  echo $v; tail -1 gpurun_out/r05q/$v.txt
done
