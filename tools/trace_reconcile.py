"""Reconcile a rocprofv3 kernel trace of `bench.py --no-extras` with the bench line.

    python tools/trace_reconcile.py <trace dir> <bench log> <out.json>

In the graph-replayed rollouts every launch of a rollout is one of the Sokoban turn kernels
(first / plain / finalize template instances, 8192 envs = 128 workgroups).  Per launch the trace
gives its duration (End - Start) and the period to the next launch of the same replay (Start of
the next - Start).  The sum of the periods over a rollout is the rollout's time on the GPU; the
kernels' summed durations can exceed it when a launch's end timestamp overlaps the next
launch's start (AQL completion-signal latency).  Compares both with the line's ms_per_step."""
import csv
import gzip
import glob
import json
import os
import re
import sys

import numpy as np


def main():
    tdir, log, dst = sys.argv[1:4]
    rows = []
    for f in glob.glob(os.path.join(tdir, "**", "*kernel_trace.csv"), recursive=True) + glob.glob(os.path.join(tdir, "**", "*kernel_trace.csv.gz"), recursive=True):
        with (gzip.open(f, "rt") if f.endswith(".gz") else open(f)) as fh:
            rows += [r for r in csv.DictReader(fh)]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    sk = [r for r in rows if "sokoban_step_turn_kernel" in r["Kernel_Name"] and int(r["Grid_Size_X"]) == 8192]
    line = [json.loads(x) for x in open(log) if x.startswith("{")][-1]
    # runs of back-to-back turn launches: consecutive sokoban launches less than 50 us apart
    start = np.array([int(r["Start_Timestamp"]) for r in sk], np.int64)
    end = np.array([int(r["End_Timestamp"]) for r in sk], np.int64)
    def kind_of(name):  # sokoban_step_turn_kernel<HW, M, LPE, kFin, kFirst, kLate[, kObs]>
        m = re.search(r"sokoban_step_turn_kernel<[^,>]*, [^,>]*, [^,>]*, (true|false), (true|false)", name)
        fin, first = (m.group(1) == "true", m.group(2) == "true") if m else (False, False)
        return "first" if first else "finalize" if fin else "plain"
    kind = [kind_of(r["Kernel_Name"]) for r in sk]
    dur = (end - start) / 1e3
    gap = np.diff(start) / 1e3
    # the graph-replayed rollouts: launches whose next launch follows within 20 us
    period = np.append(gap, np.nan)
    in_graph = period < 20
    # a rollout = first .. finalize; collect complete rollouts whose launches are all in-graph
    rollouts = []
    i = 0
    while i + 4 < len(sk):
        if kind[i] == "first" and kind[i + 4] == "finalize" and all(in_graph[i:i + 4]):
            p = start[i + 5] - start[i] if i + 5 < len(sk) and period[i + 4] < 20 else None
            rollouts.append({"durations_us": dur[i:i + 5].tolist(), "sum_dur_us": float(dur[i:i + 5].sum()),
                             "start_to_next_first_us": None if p is None else p / 1e3})
            i += 5
        else:
            i += 1
    sums = np.array([r["sum_dur_us"] for r in rollouts])
    spans = np.array([r["start_to_next_first_us"] for r in rollouts if r["start_to_next_first_us"] is not None])
    by_kind = {k: float(np.mean([d for d, kk in zip(dur, kind) if kk == k])) for k in ("first", "plain", "finalize")}
    out = {"bench_ms_per_step_us": line["ms_per_step"] * 1e3, "bench_value": line["value"],
           "rollouts_in_trace": len(rollouts), "mean_kernel_duration_us_by_kind": by_kind,
           "mean_sum_of_5_durations_us": float(sums.mean()) if len(sums) else None,
           "median_rollout_period_us": float(np.median(spans)) if len(spans) else None,
           "note": "period = Start(first launch of the next rollout) - Start(this rollout's first launch), inside "
                   "a graph replay; the sum of durations double-counts the overlap of each launch's end "
                   "timestamp with the next launch's start", "source": os.path.relpath(tdir)}
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
