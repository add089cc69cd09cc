"""Per-launch HBM traffic of one kernel from separate rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

    python tools/pmc_traffic.py <fetch_dir> <write_dir> <kernel substring> <min grid size> \\
        <algorithmic bytes per launch> <out.json> [workload text]

Correction, calibrated on this kernel's own access patterns (tools/pmc_calib.py, 604 MB
buffers past the Infinity Cache, profiles/r02_pmc_calibration.json): FETCH_SIZE reports
exactly 1/2 of the bytes read (16-B row pieces, dword and byte loads alike) and WRITE_SIZE the
bytes of every 64-B line a store touches.  So hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
Only launches with Grid_Size >= the given minimum are averaged (separates a tiled batch's
launches from the small ones of the same process)."""
import csv
import gzip
import glob
import json
import os
import sys


def per_launch(d, kernel, counter, min_grid):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True) + glob.glob(os.path.join(d, "**", "*counter_collection.csv.gz"), recursive=True):
        with (gzip.open(f, "rt") if f.endswith(".gz") else open(f)) as fh:
            for row in csv.DictReader(fh):
                if kernel in row["Kernel_Name"] and row["Counter_Name"] == counter and \
                        int(row["Grid_Size"]) >= min_grid:
                    k = (f, row["Dispatch_Id"])
                    vals[k] = vals.get(k, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    fdir, wdir, kernel, min_grid, algo, dst = sys.argv[1:7]
    workload = sys.argv[7] if len(sys.argv) > 7 else ""
    min_grid, algo = int(min_grid), float(algo)
    fetch = per_launch(fdir, kernel, "FETCH_SIZE", min_grid)
    write = per_launch(wdir, kernel, "WRITE_SIZE", min_grid)
    if not fetch or not write:
        sys.exit(f"no {kernel} rows (grid >= {min_grid}) under {fdir} / {wdir}")
    f_kb, w_kb = sum(fetch) / len(fetch), sum(write) / len(write)
    out = {"kernel": kernel, "workload": workload, "launches": [len(fetch), len(write)],
           "fetch_size_kib_raw": f_kb, "write_size_kib_raw": w_kb,
           "read_bytes_per_launch": 2 * f_kb * 1024, "write_bytes_per_launch": w_kb * 1024,
           "hbm_bytes_per_launch": (2 * f_kb + w_kb) * 1024, "algorithmic_bytes_per_launch": algo,
           "traffic_over_algorithmic": (2 * f_kb + w_kb) * 1024 / algo,
           "correction": "(2*FETCH_SIZE + WRITE_SIZE) * 1024, calibrated: profiles/r02_pmc_calibration.json",
           "source": [os.path.relpath(fdir), os.path.relpath(wdir)]}
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
