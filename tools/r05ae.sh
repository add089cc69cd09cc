set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r05ae
timeout -k 10 300 python tools/prof_chain_stamps.py > gpurun_out/r05ae/stamps.txt 2>&1 || exit 1
echo done
