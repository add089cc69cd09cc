"""Speed of the CPU port (oracle/port.py, bench.py's cpu_baseline) against the REFERENCE's own
EnvStateManager.step on the same Sokoban workload, in this container ("the ratio
restatement-speed / reference-speed is recorded").

TEST INFRASTRUCTURE, build container only (the reference is absent on the GPU box):

    PYTHONHASHSEED=0 python tests/golden/time_reference.py

The reference runs with tests/golden/refshim's gym_sokoban restatement (gym_sokoban is not
installed), which omits upstream's per-step 96x96 RGB render: the true reference is slower
still, so the ratio below understates how much faster than the reference the port is.
Workload: 2048 envs (128 groups x 16, the bench's seeds), 5 turns of the bench's synthetic
actions (K=5, cap 10), reset excluded; both sides step the same rooms with the same action
texts, and their env.step counts and final room states are checked equal.
Writes tests/golden/port_vs_reference.json (data only)."""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
import make_golden as mg  # noqa: E402  (installs refshim, imports the reference)

from oracle import port  # noqa: E402
from ragen_amd import synthetic  # noqa: E402


def main(n_groups=128, group_size=16, T=5, K=5, reps=3):
    B = n_groups * group_size
    ids, n = synthetic.rollout_actions(B, T, K, 1, 4)
    best = {}
    for rep in range(reps):
        es = mg.EnvStateManager(mg.make_cfg("SimpleSokoban", n_groups, group_size), mode="train")
        es.reset(seed=synthetic.ENV_SEED)  # env i -> ENV_SEED + i // 16, as the bench
        fixed = np.stack([e["env"].room_fixed.astype(np.uint8).ravel() for e in es.envs])
        state0 = np.stack([e["env"].room_state.astype(np.uint8).ravel() for e in es.envs])
        player0 = np.stack([np.asarray(e["env"].player_position, np.int64) for e in es.envs])
        steps0 = sum(e["env"].num_env_steps for e in es.envs)
        active = list(range(B))
        t0 = time.perf_counter()
        for t in range(T):
            inputs = [{"env_id": i, "llm_response": "", "llm_raw_response": "",
                       "actions": [port.NAMES[int(a)] for a in ids[t, i, :int(n[t, i])]]} for i in active]
            outs = es.step(inputs)
            active = [o["env_id"] for o in outs]
            if not active:
                break
        ref_dt = time.perf_counter() - t0
        ref_steps = sum(e["env"].num_env_steps for e in es.envs) - steps0
        ref_final = np.stack([e["env"].room_state.astype(np.uint8).ravel() for e in es.envs])
        envs = port.make_sokoban_envs(fixed, state0, player0)
        t0 = time.perf_counter()
        port_steps = port.sokoban_rollout(envs, ids, n)
        port_dt = time.perf_counter() - t0
        port_final = np.stack([e["env"].room_state.astype(np.uint8).ravel() for e in envs])
        assert port_steps == ref_steps, (port_steps, ref_steps)
        assert np.array_equal(port_final, ref_final)
        if not best or ref_dt + port_dt < best["ref_s"] + best["port_s"]:
            best = {"ref_s": ref_dt, "port_s": port_dt, "env_steps": ref_steps}
    out = {
        "workload": f"Sokoban 6x6, {B} envs ({n_groups} groups x {group_size}), {T} turns, K={K}, cap 10, reset excluded",
        "env_steps": best["env_steps"],
        "reference_env_steps_per_s": best["env_steps"] / best["ref_s"],
        "port_env_steps_per_s": best["env_steps"] / best["port_s"],
        "port_over_reference": best["ref_s"] / best["port_s"],
        "reference": "ragen/llm_agent/es_manager.py EnvStateManager.step over ragen/env/sokoban/env.py, "
                     "gym_sokoban restated by tests/golden/refshim.py (no per-step RGB render)",
        "port": "oracle/port.py (bench.py cpu_baseline, kind 'port')",
        "host": "build container, 1 thread, best of %d" % reps,
    }
    with open(os.path.join(HERE, "port_vs_reference.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
