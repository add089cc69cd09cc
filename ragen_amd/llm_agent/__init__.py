from .agent_proxy import LLMAgentProxy, ScriptedActor
from .ctx_manager import ContextManager, get_masks_and_scores
from .es_manager import EnvStateManager, EnvStatus

__all__ = ["LLMAgentProxy", "ScriptedActor", "ContextManager", "get_masks_and_scores", "EnvStateManager", "EnvStatus"]
