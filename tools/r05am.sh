set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r05am
RAGEN_AMD_PARSE1=1 timeout -k 10 300 python -u tools/prof_token_timeline.py > gpurun_out/r05am/token_timeline.txt 2>&1
rc=$?; echo "[timeline] rc=$rc"; tail -14 gpurun_out/r05am/token_timeline.txt; exit $rc
