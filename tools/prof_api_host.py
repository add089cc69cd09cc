"""Host-time anatomy of the device-path rollout (diagnostic): tools/prof_api_cprofile.py's setup,
warmed up, then 5 rollouts under cProfile; prints, per rollout and in microseconds, every
function's own and cumulative time (top 45 by own time, top 45 by cumulative), so the C-level
calls (torch.empty, stream synchronisation, ctypes launches) show with their counts."""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import prof_api_cprofile as base  # noqa: E402  (builds the proxy and runs 3 warm-up rollouts)

N = 5
pr = cProfile.Profile()
pr.enable()
for _ in range(N):
    tm = base.run()
pr.disable()
print("profiled (last):", {k: (round(v * 1e3, 2) if isinstance(v, float) else v) for k, v in tm.items()}, "ms")
st = pstats.Stats(pr).stats


def name(k):
    f, ln, fn = k
    return f"{os.path.basename(f)}:{ln}({fn})" if f != "~" else fn


rows = [(name(k), v[1] / N, v[2] * 1e6 / N, v[3] * 1e6 / N) for k, v in st.items()]
tot = sum(r[2] for r in rows)
print(f"own time per rollout (all functions): {tot:.0f} us")
for title, idx in (("own", 2), ("cumulative", 3)):
    print(f"--- top by {title} time (per rollout: calls, own us, cum us)")
    for r in sorted(rows, key=lambda r: -r[idx])[:45]:
        print(f"{r[1]:8.1f} {r[2]:9.1f} {r[3]:9.1f}  {r[0]}")
