from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv  # noqa: F401
