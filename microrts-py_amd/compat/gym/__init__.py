"""Stand-in for the parts of `gym` the reference drivers import (gym is not in
this image).  Only `gym.spaces` is provided: experiments/ppo_gridnet.py:17 and
ppo_gridnet_eval.py import `MultiDiscrete` from it and check
`isinstance(envs.action_space, MultiDiscrete)` (ppo_gridnet.py:390), so the
classes are the ones gym_microrts builds its spaces from.

Put on sys.path by gym_microrts.run_driver only when the real package is absent.
"""
__microrts_compat__ = True
__version__ = "0.0-microrts-compat"

from . import spaces  # noqa: E402,F401
