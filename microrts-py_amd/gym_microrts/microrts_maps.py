"""Training-map catalogue: the same entries, in the same order, as
/root/reference/gym_microrts/microrts_maps.py:1-20 (ALL16x16_MAPS).  Paths are
relative to gym_microrts/microrts; the maps themselves are authored in this repo
(scripts/author_maps.py: the Java submodule holding the originals is absent, so
every layout except basesWorkers16x16A's is an authored one, parity unpinned)."""

_VARIANTS = ["A", "E", "I", "noResources", "melee:Mixed12", "B", "F", "J", "R20", "melee:Mixed8", "C", "G", "K",
             "TwoBasesBarracks", "D", "H", "L", "EightBasesWorkers"]


def _path(v):
    if v.startswith("melee:"):
        return f"maps/16x16/melee16x16{v.split(':')[1]}.xml"
    if v in ("TwoBasesBarracks", "EightBasesWorkers"):
        return f"maps/16x16/{v}16x16.xml"
    return f"maps/16x16/basesWorkers16x16{v}.xml"


ALL16x16_MAPS = [_path(v) for v in _VARIANTS]
