"""mgx -- MI355X-native vectorised MiniGrid (PlaygroundEnv) engine.

Host-side mirror of the reference's env/rollout interface (Idokorro/MiniGrid-RL
src/custom_env.py, src/environment.py, src/ppo.py) over libmgx.so (HIP/gfx950).
"""
from ._lib import MgxError, mission_text  # noqa: F401
from .describe import LLMDescriptionWrapper  # noqa: F401
from .engine import MgxEngine, gae, gae_dones, random_actions  # noqa: F401
from .evaluation import EvalCallback, StopTrainingOnRewardThreshold, evaluate_policy, evaluate_test_protocol  # noqa: F401
from .vec_env import MgxVecEnv  # noqa: F401

__all__ = ["EvalCallback", "LLMDescriptionWrapper", "MgxEngine", "MgxError", "MgxVecEnv", "StopTrainingOnRewardThreshold", "evaluate_policy", "evaluate_test_protocol", "gae", "gae_dones", "mission_text", "random_actions"]
