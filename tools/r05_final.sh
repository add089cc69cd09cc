#!/bin/bash
# Round-5 GPU check: the -m gpu suite, smoke, the launcher's --gpus 2 refusal on a 1-GPU box,
# the torchrun path at N=1, the 1-rank RCCL exchange path, and the default bench line.  Each
# GPU step has its own limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05final}; mkdir -p $OUT
step() { echo "[$1] rc=$2" | tee -a $OUT/status.txt; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; step pytest $?
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; step smoke $?
# --gpus 2 on one GPU: must exit 2 with the reason, before any GPU work
timeout -k 10 120 python bench.py --gpus 2 --no-extras > $OUT/gpus2.log 2>&1; rc=$?
echo "[gpus2] rc=$rc (2 expected)" | tee -a $OUT/status.txt; [ $rc -eq 2 ] || exit 1
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --steps 20 --warmup 5 --no-extras --no-cpu-baseline > $OUT/torchrun1.log 2>&1; step torchrun1 $?
tail -1 $OUT/torchrun1.log
timeout -k 10 200 python bench.py --double-buffer --steps 40 --warmup 8 --no-extras --no-cpu-baseline > $OUT/dbuf.log 2>&1; step dbuf $?
tail -1 $OUT/dbuf.log
if [ "${SKIP_BENCH:-0}" = "0" ]; then
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1; step bench $?
  tail -1 $OUT/bench.log
fi
echo session-done
