#!/bin/bash
# PMC passes over rmi_bpe_encode alone (tools/bench_bpe.py pmc: the API rollout's turn-2 text,
# 8192 rows, 10 launches at the chain's row bound), one rocprofv3 run per counter group: the
# per-wave SQ means (tools/pmc_per_wave.py) and the per-launch HBM bytes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmc_bpe}; mkdir -p $OUT
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace -d $OUT/pass$i -o pmc --output-format csv \
    -- python3 tools/bench_bpe.py 2 pmc > $OUT/pass$i.log 2>&1
  rc=$?; echo "pass$i rc=$rc" | tee -a $OUT/status.txt; [ $rc -ne 0 ] && exit $rc
done
python3 tools/pmc_per_wave.py $OUT bpe_encode_kernel | tee $OUT/per_wave.txt
python3 - "$OUT" <<'PY' | tee $OUT/traffic.txt
import csv, glob, os, sys
d = sys.argv[1]
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    v = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if "bpe_encode_kernel" in row["Kernel_Name"] and row["Counter_Name"] == c:
                v.append(float(row["Counter_Value"]))
    print(c, "KiB per launch (raw, uncorrected):", sum(v) / max(len(v), 1), "launches:", len(v))
PY
