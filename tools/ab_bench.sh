#!/bin/bash
# A/B (diagnostic): the headline bench (--no-extras) with the default library and variant builds
# (variants/libragen_amd_NAME.so), alternating three times; prints ms_per_step and the
# event-timed plain launch.
#   tools/ab_bench.sh OUT NAME [NAME ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-abbench}; shift; mkdir -p $OUT
for i in 1 2 3; do
  for v in default "$@"; do
    if [ $v = default ]; then L=""; else L=$PWD/variants/libragen_amd_$v.so; fi
    RAGEN_AMD_LIB=$L timeout -k 10 240 python bench.py --no-extras --no-cpu-baseline > $OUT/$v.$i.json 2>> $OUT/err.log || exit 1
    python -c "import json;d=json.load(open('$OUT/$v.$i.json'));print('$v', round(d['ms_per_step']*1e3, 2), round(d['roofline']['avg_launch_us'], 3))" | tee -a $OUT/ab.txt
  done
done
