"""ContextManager.device_metrics (the formulate path's mean / non-zero metrics from the device
metric rows) against the reference's own aggregation, restated over per-env metric dicts
(ctx_manager.py:308-327: np.sum(list) / env_num per key, np.mean over the non-zero values;
es_manager.py:183-197: success a float 0 / 1, num_actions an int, the custom metrics f64
means of the turns' info values, present only for envs whose turns reported them): the same
keys in the same order, the same values and types, bit for bit."""
import types

import numpy as np

from ragen_amd.llm_agent.ctx_manager import ContextManager


def _reference(tags, rows, env_nums):
    """ctx_manager.py:308-327 over the per-env dicts es_manager.get_rollout_states builds."""
    metrics = {}
    for tag in tags:
        m, cust = rows[tag]
        for i in range(m.shape[0]):
            env = {f"{tag}/success": float(m[i, 0]), f"{tag}/num_actions": int(m[i, 1])}
            if cust[i]:
                env[f"{tag}/action_is_effective"] = float(m[i, 2])
                env[f"{tag}/action_is_valid"] = float(m[i, 3])
            for k, v in env.items():
                metrics.setdefault(k, []).append(v)
    mean = {k: np.sum(v) / env_nums[k.split("/")[0]] for k, v in metrics.items()}
    for k, vals in metrics.items():
        prefix, suffix = k.split("/", 1)
        nz = [v for v in vals if v != 0]
        if nz:
            mean[f"{prefix}/non-zero/{suffix}"] = np.mean(nz)
    return mean


def test_device_metrics_equal_reference_aggregation():
    rng = np.random.default_rng(7)
    for trial in range(60):
        tags = ["SimpleSokoban", "FrozenLake"] if trial % 3 == 0 else ["SimpleSokoban"]
        fake = types.SimpleNamespace(process_group=None, world_size=1, env_nums={},
                                     es_cfg=types.SimpleNamespace(env_configs=types.SimpleNamespace(tags=tags)))
        rows, parts = {}, []
        for t in tags:
            n = int(rng.integers(1, 600))
            m = np.zeros((n, 4))
            m[:, 0] = rng.random(n) < rng.random()
            m[:, 1] = rng.integers(0, 20, n) * (rng.random(n) < 0.7)
            m[:, 2] = np.where(rng.random(n) < 0.5, rng.integers(0, 6, n) / 5.0, 0.0)
            m[:, 3] = np.where(rng.random(n) < 0.5, rng.integers(0, 7, n) / 3.0, 0.0)
            cust = rng.random(n) < (0.0, 1.0, 0.6)[trial % 3]
            if trial % 2:  # the formulate chain hands its rows over column-major
                m = np.ascontiguousarray(m.T).T
            rows[t] = (m, cust)
            fake.env_nums[t] = n
            parts.append((t, m, cust, None))
        want = _reference(tags, rows, fake.env_nums)
        got = ContextManager.device_metrics(fake, None, parts)
        # (the reference lists keys in first-seen order over the envs; compare as sets and values)
        assert set(got) == set(want), (sorted(got), sorted(want))
        for k in want:
            assert got[k] == want[k], (trial, k, got[k], want[k])
            assert isinstance(got[k], np.floating), (k, type(got[k]))
