"""Diagnostic: cProfile of the chained device turn loop (bench.api_leg's setup, warmed up): the
callees of gen_batch, _step_device, get_env_inputs and formulate, with own and cumulative times
(cProfile inflates every call by its own cost: compare the split, not the absolute)."""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import prof_api_cprofile as base  # noqa: E402  (the proxy, warmed up)

for _ in range(2):
    base.run()
pr = cProfile.Profile()
pr.enable()
for _ in range(4):
    base.run()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(45)
for fn in ("gen_batch", "_step_device", "_device_env_inputs", "run", "get_lm_inputs", "generate_sequences"):
    st.print_callees(fn)
