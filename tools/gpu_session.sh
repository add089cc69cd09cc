#!/bin/bash
# One GPU-box session: gpu tests -> smoke -> bench -> rocprofv3 kernel-trace stats.
# Every GPU step has its own time limit; a fault / abort / timeout ends the session.
# usage: bash tools/gpu_session.sh <tag> [steps...]   (steps: tests smoke bench prof prof_all pmc)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r01}
shift || true
STEPS=${*:-"tests smoke bench prof"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"

ok_or_stop() {  # $1 = rc, $2 = step; stop on anything but success / ordinary test failure
  local rc=$1
  echo "[$2] rc=$rc" | tee -a "$OUT/status.txt"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then
    echo "stopping after $2 (rc=$rc)" | tee -a "$OUT/status.txt"
    exit "$rc"
  fi
}

python -c "import __graft_entry__ as g; g.build()" > "$OUT/build.log" 2>&1 || { echo build failed; cat "$OUT/build.log"; exit 3; }

for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
      ok_or_stop $? tests; tail -5 "$OUT/pytest_gpu.log";;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      ok_or_stop $? smoke; tail -3 "$OUT/smoke.log";;
    bench)
      timeout -k 10 600 python bench.py > "$OUT/bench.log" 2>&1
      ok_or_stop $? bench; tail -2 "$OUT/bench.log";;
    prof)  # the headline path only: its kernel averages are the bench line's
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench --output-format csv \
        -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-extras > "$OUT/prof.log" 2>&1
      ok_or_stop $? prof; tail -2 "$OUT/prof.log";;
    prof_all)  # every leg (advantage, toy-text, text API, at-scale) for the extras' kernels
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_all" -o bench --output-format csv \
        -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline > "$OUT/prof_all.log" 2>&1
      ok_or_stop $? prof_all; tail -2 "$OUT/prof_all.log";;
    pmc)
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace -d "$OUT/pmc_$c" -o pmc --output-format csv \
          -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-graph > "$OUT/pmc_$c.log" 2>&1
        ok_or_stop $? "pmc_$c"
      done;;
    *)
      echo "unknown step $s";;
  esac
done
echo done | tee -a "$OUT/status.txt"
