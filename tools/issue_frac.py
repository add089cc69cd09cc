"""Issue-rate efficiency of the text kernels from one rocprofv3 --pmc pass (with --kernel-trace):
per kernel (name substring), per launch: waves, VALU / SALU / LDS / VMEM instructions, the
launch's duration (kernel trace), and

    issue_frac = (VALU + SALU + LDS instructions) / (cycles x 1024 SIMDs)

with cycles = duration x 2.4 GHz (MI355X peak engine clock, MI355X_MICROARCH.md) and a peak of one
instruction issued per SIMD per cycle; valu_frac = VALU x 2 / (cycles x 1024) (a wave64 VALU
instruction holds its SIMD-32 two cycles, MI355X_MICROARCH.md); salu_frac = SALU / (cycles x 256)
(one scalar unit per CU).  These kernels are bound by dependent instruction chains inside a wave,
not by HBM: the fractions say how much of the chip's issue capacity the launch used.
    python tools/issue_frac.py <pass dir> <kernel substring> ... > summary.json"""
import csv
import glob
import gzip
import json
import os
import sys
from collections import defaultdict

CLK_GHZ, SIMDS, CUS = 2.4, 1024, 256


def _open(f):
    return gzip.open(f, "rt") if f.endswith(".gz") else open(f)


def main():
    d, kernels = sys.argv[1], sys.argv[2:]
    counts = {k: defaultdict(float) for k in kernels}
    launches = {k: set() for k in kernels}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv*"), recursive=True):
        with _open(f) as fh:
            for row in csv.DictReader(fh):
                for k in kernels:
                    if k in row["Kernel_Name"]:
                        counts[k][row["Counter_Name"]] += float(row["Counter_Value"])
                        launches[k].add(row.get("Dispatch_Id") or row.get("Correlation_Id"))
    durs = {k: [] for k in kernels}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv*"), recursive=True):
        with _open(f) as fh:
            for row in csv.DictReader(fh):
                for k in kernels:
                    if k in row["Kernel_Name"]:
                        durs[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    out = {}
    for k in kernels:
        n = max(len(launches[k]), 1)
        c = {name: v / n for name, v in counts[k].items()}
        if not durs[k] or not c:
            out[k] = None
            continue
        dur = sum(durs[k]) / len(durs[k])
        cyc = dur * CLK_GHZ * 1e9
        valu, salu, lds = c.get("SQ_INSTS_VALU", 0.0), c.get("SQ_INSTS_SALU", 0.0), c.get("SQ_INSTS_LDS", 0.0)
        waves = c.get("SQ_WAVES", 0.0)
        out[k] = {"launches": len(launches[k]), "avg_us": dur * 1e6, "waves": waves,
                  "per_wave": {x: round(c.get("SQ_INSTS_" + x, 0.0) / waves, 1) if waves else None
                               for x in ("VALU", "SALU", "LDS", "VMEM_RD", "VMEM_WR")},
                  "wave_cycles_per_wave": c.get("SQ_WAVE_CYCLES", 0.0) / waves if waves else None,
                  "issue_frac": (valu + salu + lds) / (cyc * SIMDS),
                  "valu_frac": valu * 2 / (cyc * SIMDS), "salu_frac": salu / (cyc * CUS),
                  "formula": "(VALU+SALU+LDS)/(dur*2.4GHz*1024 SIMDs); valu x2/(..*1024); salu/(..*256 CUs)"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
