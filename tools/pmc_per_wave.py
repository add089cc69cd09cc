"""Per-wave means of SQ counters per kernel from rocprofv3 --pmc pass directories (diagnostic).
    python tools/pmc_per_wave.py <dir with pass*/> <kernel substring> ..."""
import csv
import glob
import gzip
import os
import sys
from collections import defaultdict


def main():
    d, kernels = sys.argv[1], sys.argv[2:]
    tot = {k: defaultdict(float) for k in kernels}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv*"), recursive=True):
        with (gzip.open(f, "rt") if f.endswith(".gz") else open(f)) as fh:
            for row in csv.DictReader(fh):
                name = row["Kernel_Name"]
                for k in kernels:
                    if "::" + k + "(" in name or "::" + k + "<" in name:
                        tot[k][(f, row["Counter_Name"])] += float(row["Counter_Value"])
    for k in kernels:
        per = defaultdict(float)
        waves = defaultdict(float)
        for (f, c), v in tot[k].items():
            per[(os.path.dirname(f), c)] += v
        for (p, c), v in per.items():
            if c == "SQ_WAVES":
                waves[p] = v
        out = {}
        for (p, c), v in per.items():
            if c != "SQ_WAVES" and waves.get(p):
                out[c] = v / waves[p]
        print(k, {c: round(v, 1) for c, v in sorted(out.items())})


if __name__ == "__main__":
    main()
