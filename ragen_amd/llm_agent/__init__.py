from .agent_proxy import LLMAgentProxy, ScriptedActor, TokenActor
from .ctx_manager import ContextManager, get_masks_and_scores
from .es_manager import EnvStateManager, EnvStatus

__all__ = ["LLMAgentProxy", "ScriptedActor", "TokenActor", "ContextManager", "get_masks_and_scores", "EnvStateManager", "EnvStatus"]
