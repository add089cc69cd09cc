set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r05ad
timeout -k 10 300 python tools/prof_chain_cprofile.py > gpurun_out/r05ad/cprofile.txt 2>&1 || exit 1
echo done
