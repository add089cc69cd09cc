#!/bin/bash
# A/B (diagnostic): the headline bench (--no-extras) under HIP runtime settings, alternating
# three times; prints ms_per_step and the event-timed plain launch per setting.
#   tools/ab_env.sh OUT "NAME=VALUE" ["NAME=VALUE" ...]     ("-" = the image's defaults)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-abenv}; shift; mkdir -p $OUT
for i in 1 2 3; do
  for e in - "$@"; do
    tag=$(echo "$e" | tr '=' '_')
    if [ "$e" = - ]; then
      timeout -k 10 240 python bench.py --no-extras --no-cpu-baseline > $OUT/$tag.$i.json 2>> $OUT/err.log || exit 1
    else
      export "$e"
      timeout -k 10 240 python bench.py --no-extras --no-cpu-baseline > $OUT/$tag.$i.json 2>> $OUT/err.log || exit 1
      unset "${e%%=*}"
    fi
    python -c "import json;d=json.load(open('$OUT/$tag.$i.json'));print('$e', round(d['ms_per_step']*1e3, 2), round(d['roofline']['avg_launch_us'], 3))" | tee -a $OUT/ab.txt
  done
done
