set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r05ag
timeout -k 10 300 python -u tools/prof_token_timeline.py > gpurun_out/r05ag/token_timeline.txt 2>&1
rc=$?; echo "[timeline] rc=$rc"; tail -20 gpurun_out/r05ag/token_timeline.txt; [ $rc -ne 0 ] && exit $rc
bash tools/parse_pmc.sh r05ag/pmc > gpurun_out/r05ag/pmc.txt 2>&1
rc=$?; echo "[pmc] rc=$rc"; tail -20 gpurun_out/r05ag/pmc.txt; exit $rc
