"""Opponent factories, same names as /root/reference/gym_microrts/microrts_ai.py.

In the reference each factory returns a Java AI object (`f(utt) -> AI`).  Here
bots run on the device (mrts_bots.hip, one wavefront per bot game, launched
before the step kernel), so a factory returns a descriptor naming the device
bot.  Bots whose device implementation does not exist (naiveMCTSAI and the
competition bots other than coacAI) carry `ai_id = None` and make
MicroRTSGridModeVecEnv raise NotImplementedError instead of silently
substituting another policy.
"""


class DeviceAI:
    def __init__(self, name, ai_id):
        self.name = name
        self.ai_id = ai_id

    def __repr__(self):
        return f"DeviceAI({self.name})"

    def __str__(self):
        return self.name


# ids match MRTS_AI_* in include/microrts_amd.h
_IDS = {"passiveAI": 0, "workerRushAI": 1, "lightRushAI": 2, "randomBiasedAI": 3, "coacAI": 4,
        "POWorkerRush": 5, "POLightRush": 6, "POHeavyRush": 7, "PORangedRush": 8, "randomAI": 9}


def _factory(name):
    def f(utt=None):
        return DeviceAI(name, _IDS.get(name))

    f.__name__ = name
    f.__qualname__ = name
    return f


randomBiasedAI = _factory("randomBiasedAI")   # microrts_ai.py:1-4
randomAI = _factory("randomAI")               # :7-10
passiveAI = _factory("passiveAI")             # :13-16
workerRushAI = _factory("workerRushAI")       # :19-22
lightRushAI = _factory("lightRushAI")         # :25-28
POLightRush = _factory("POLightRush")         # :31-34
POWorkerRush = _factory("POWorkerRush")       # :37-40
POHeavyRush = _factory("POHeavyRush")         # :43-46
PORangedRush = _factory("PORangedRush")       # :49-52
coacAI = _factory("coacAI")                   # :58-61
naiveMCTSAI = _factory("naiveMCTSAI")         # :64-67
mixedBot = _factory("mixedBot")
rojo = _factory("rojo")
izanagi = _factory("izanagi")
tiamat = _factory("tiamat")
droplet = _factory("droplet")
mayari = _factory("mayari")
guidedRojoA3N = _factory("guidedRojoA3N")

ALL_AIS = [
    randomBiasedAI,
    randomAI,
    passiveAI,
    workerRushAI,
    lightRushAI,
    coacAI,
    naiveMCTSAI,
]
