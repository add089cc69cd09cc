set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r05u
timeout -k 10 300 python tools/bench_bpe.py > gpurun_out/r05u/bench_bpe.txt 2>&1 || exit $?; tail -1 gpurun_out/r05u/bench_bpe.txt
