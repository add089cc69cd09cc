set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r05w
timeout -k 10 200 python tools/bench_prompt.py > gpurun_out/r05w/base.txt 2>&1 || exit 1; tail -1 gpurun_out/r05w/base.txt
RAGEN_AMD_LIB=variants/libragen_amd_prnorepr.so timeout -k 10 200 python tools/bench_prompt.py > gpurun_out/r05w/norepr.txt 2>&1 || exit 1; tail -1 gpurun_out/r05w/norepr.txt
