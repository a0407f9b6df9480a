"""eco_hip: MI355X-native ECO-DQN MaxCut environment + rollout engine.

Host-side mirror of the reference's src/envs, src/networks and src/agents/dqn APIs
over libecohip.so (include/eco_hip.h).  Importing the package loads the HIP
library and fails loudly (ImportError) if it has not been built.
"""
from . import _lib  # noqa: F401  (loads libecohip.so or raises)

__all__ = ["envs", "networks", "agents", "graphs"]
