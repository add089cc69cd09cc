set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r05au
RAGEN_AMD_LIB=variants/libragen_amd_tokstamps.so timeout -k 10 120 python -u tools/prof_token_turn.py > gpurun_out/r05au/stamps.txt 2>&1
rc=$?; echo "[stamps] rc=$rc"; tail -6 gpurun_out/r05au/stamps.txt; exit $rc
