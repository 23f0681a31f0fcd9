"""Stand-in for the parts of stable_baselines3 the reference drivers import
(`stable_baselines3.common.vec_env`: ppo_gridnet.py:18).  Not installed in this image."""
__microrts_compat__ = True
__version__ = "0.0-microrts-compat"
