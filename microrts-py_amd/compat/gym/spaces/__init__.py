"""gym.spaces stand-in: the Box / MultiDiscrete / Discrete classes of gym_microrts._spaces."""
from gym_microrts._spaces import Box, Discrete, MultiDiscrete  # noqa: F401

Space = object
