"""Summarise rocprofv3 --pmc passes over tools/prof_sokoban.py into the per-launch HBM
traffic of rmi_sokoban_step_turn (profiles/pmc_sokoban_step_turn.json, read by bench.py).

    python tools/pmc_summary.py gpurun_out/<tag> profiles/pmc_sokoban_step_turn.json

Correction (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7): FETCH_SIZE / WRITE_SIZE are
KiB; on gfx950 FETCH_SIZE reports half the bytes of a streaming read, so
hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.  Raw values are kept beside it.
"""
import csv
import glob
import json
import os
import sys

KERNEL = "sokoban_step_turn_kernel"
BYTES_PER_ENV_TURN = 141


def per_launch(d, counter):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if KERNEL in row["Kernel_Name"] and row["Counter_Name"] == counter:
                    k = (f, row["Dispatch_Id"])
                    vals[k] = vals.get(k, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def all_counters(d):
    names = set()
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            names |= {row["Counter_Name"] for row in csv.DictReader(fh) if KERNEL in row["Kernel_Name"]}
    return sorted(names)


def main():
    src, dst = sys.argv[1], sys.argv[2]
    fetch = per_launch(src, "FETCH_SIZE")
    write = per_launch(src, "WRITE_SIZE")
    if not fetch or not write:
        sys.exit(f"no {KERNEL} FETCH_SIZE/WRITE_SIZE rows under {src}")
    f_kb = sum(fetch) / len(fetch)
    w_kb = sum(write) / len(write)
    active = [8192, 7824, 7399, 6052, 4066]  # active envs per turn of the bench rollout
    algo = sum(active) / len(active) * BYTES_PER_ENV_TURN
    out = {
        "kernel": "rmi_sokoban_step_turn",
        "workload": "tools/prof_sokoban.py: bench rollout (8192 envs x 5 turns), eager",
        "launches_fetch": len(fetch), "launches_write": len(write),
        "fetch_size_kib_raw": f_kb, "write_size_kib_raw": w_kb,
        "hbm_bytes_per_launch": (2 * f_kb + w_kb) * 1024,
        "algorithmic_bytes_per_launch": algo,
        "correction": "(2*FETCH_SIZE + WRITE_SIZE) * 1024; gfx950 FETCH_SIZE = 1/2 of streamed read bytes",
        "source": os.path.relpath(src),
    }
    out["traffic_over_algorithmic"] = out["hbm_bytes_per_launch"] / algo
    out["per_launch_means"] = {c: sum(v) / len(v) for c in all_counters(src) for v in [per_launch(src, c)]}
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
