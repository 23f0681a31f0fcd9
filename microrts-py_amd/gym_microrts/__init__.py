"""MI355X-native vectorised MicroRTS, drop-in for gym_microrts (adFrej/MicroRTS-Py).

The game engine runs as HIP kernels on gfx950 (libmicrorts_amd.so); this package
keeps the reference's Python surface (envs.vec_env.MicroRTSGridModeVecEnv,
microrts_ai, microrts_maps).
"""
__version__ = "0.1.0"
