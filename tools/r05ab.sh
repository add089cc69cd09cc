set -u
cd "${GRAFT_REPO_ROOT}"
bash tools/r05_check.sh r05ab "tests" || exit $?
grep -n "readback_kernel\|copyBuffer" gpurun_out/r05ab/api_timeline.txt | head -12
tail -1 gpurun_out/r05ab/api_timeline.txt
