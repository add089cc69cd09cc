"""GPU timeline of one device-path API rollout from a rocprofv3 kernel trace (diagnostic): every
kernel of the LAST device-path rollout of tools/api_leg.py (from its reset kernel to the next
one), its duration and the idle gap before it, and the rollout's span against its busy time.
    python tools/api_timeline.py gpurun_out/<run>/prof/api_kernel_trace.csv"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
resets = [i for i, r in enumerate(rows) if "sokoban_reset_kernel" in r["Kernel_Name"] or "sokoban_load_rooms_kernel" in r["Kernel_Name"]]
# api_leg: 4 device-path rollouts (one reset each), then the dict-path rollouts
a, b = resets[3], resets[4] if len(resets) > 4 else len(rows)
seg = rows[a:b]
for i in range(1, len(seg)):  # the rollout ends at the first idle stretch over 5 ms
    if int(seg[i]["Start_Timestamp"]) - int(seg[i - 1]["End_Timestamp"]) > 5_000_000:
        seg = seg[:i]
        break
# ... and at the formulated batch: formulate_tail_kernel and the readbacks right behind it (what
# follows is the bench's own step count after rollout() returned)
tails = [i for i, r in enumerate(seg) if "formulate_tail_kernel" in r["Kernel_Name"]]
if tails:
    j = tails[-1] + 1
    while (j < len(seg) and ("readback_kernel" in seg[j]["Kernel_Name"] or "copyBuffer" in seg[j]["Kernel_Name"])
           and int(seg[j]["Start_Timestamp"]) - int(seg[j - 1]["End_Timestamp"]) < 50_000):
        j += 1
    seg = seg[:j]
t0 = int(seg[0]["Start_Timestamp"])
busy, prev = 0, t0
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].replace("rmi::(anonymous namespace)::", "").replace("void ", "")[:56]
    print(f"{(s - t0) / 1e3:9.1f} us  {(e - s) / 1e3:7.1f} us  gap {(s - prev) / 1e3:7.1f}  {name}")
    busy += e - s
    prev = max(prev, e)
print(f"rollout span {(prev - t0) / 1e3:.1f} us, kernels busy {busy / 1e3:.1f} us, {len(seg)} launches")
