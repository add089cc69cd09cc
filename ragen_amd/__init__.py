"""ragen_amd — MI355X (gfx950) engine for RAGEN's StarPO rollout-and-advantage hot path.

Native core: ragen_amd/_build/libragen_amd.so (C ABI: include/ragen_amd.h).
Drop-in Python surface: ragen_amd.env (registries), ragen_amd.llm_agent (EnvStateManager,
ContextManager, LLMAgentProxy), ragen_amd.trainer (compute_advantage, core_algos).
"""
__version__ = "0.1.0"
