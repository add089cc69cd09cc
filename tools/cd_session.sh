set -o pipefail
export TMPDIR=/tmp
for a in "1" "44 + 19 + 3 + 7" "(44 - 19) * (3 + 7)" "((44 / 19) - 3) * 7"; do timeout -k 5 30 ./tools/cd_stamp "$a" 1 || exit 1; done > gpurun_out/cds.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace -d gpurun_out/cdstamp_pmc -o pmc --output-format csv -- ./tools/cd_stamp "44 + 19 + 3 + 7" 1 > gpurun_out/cdstamp_pmc.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -k "countdown or Countdown" > gpurun_out/cdt.log 2>&1 || exit 1
timeout -k 10 120 python3 tools/prof_countdown.py > gpurun_out/cdp.log 2>&1
