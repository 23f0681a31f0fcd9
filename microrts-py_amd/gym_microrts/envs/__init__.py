from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv  # noqa: F401
from gym_microrts.envs.vec_env import MicroRTSBotVecEnv  # noqa: F401
from gym_microrts.envs.vec_env import MicroRTSGridModeSharedMemVecEnv  # noqa: F401
