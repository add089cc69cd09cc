#!/bin/bash
# GPU tests of the device prompt path and the facades it changes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r03p}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest ${2:-tests/test_gpu_device_prompts.py tests/test_gpu_device_rollout.py tests/test_gpu_facade.py tests/test_gpu_tokenizer.py tests/test_gpu_fit.py} -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "[tests] rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" $OUT/pytest.log | tail -40; exit $rc
