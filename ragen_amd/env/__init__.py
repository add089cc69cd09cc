"""Env registries keyed by ``env_type`` exactly like ragen/env/__init__.py:15-31, but
holding batched (one object per tag) GPU envs."""
from .bandit import BanditBatch
from .base import BatchEnv
from .configs import BanditEnvConfig, CountdownEnvConfig, FrozenLakeEnvConfig, SokobanEnvConfig
from .countdown import CountdownBatch
from .frozen_lake import FrozenLakeBatch
from .sokoban import SokobanBatch

REGISTERED_ENVS = {
    "bandit": BanditBatch,
    "countdown": CountdownBatch,
    "sokoban": SokobanBatch,
    "frozen_lake": FrozenLakeBatch,
}

REGISTERED_ENV_CONFIGS = {
    "bandit": BanditEnvConfig,
    "countdown": CountdownEnvConfig,
    "sokoban": SokobanEnvConfig,
    "frozen_lake": FrozenLakeEnvConfig,
}

__all__ = ["REGISTERED_ENVS", "REGISTERED_ENV_CONFIGS", "BatchEnv", "SokobanBatch", "FrozenLakeBatch", "BanditBatch",
           "CountdownBatch"]
