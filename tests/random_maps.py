"""Seeded random maps (test infrastructure): walls, resources and both players' bases,
barracks and units of every type placed on free cells, written in the reference's map XML
format (PCG/maps/wall-1; PhysicalGameState.load).  Dense maps put more than 64 units in
a game -- the bots' unit-list / abstract-action paths past one wavefront (rush_serial,
coac_serial, the serial translateActions) and wide unit lists everywhere else."""
import numpy as np

TYPES = ["Resource", "Base", "Barracks", "Worker", "Light", "Heavy", "Ranged"]
HP = {"Resource": 1, "Base": 10, "Barracks": 4, "Worker": 1, "Light": 4, "Heavy": 4, "Ranged": 1}


def write_random_map(path, w, h, seed, n_units=40, wall_frac=0.08, res=(5, 5)):
    rng = np.random.default_rng(seed)
    wall = (rng.random(h * w) < wall_frac).astype(np.uint8)
    free = np.flatnonzero(wall == 0)
    rng.shuffle(free)
    units, uid = [], 0
    # at least one base and one worker per player, then random units
    kinds = [("Base", 0), ("Base", 1), ("Worker", 0), ("Worker", 1)]
    while len(kinds) < n_units:
        t = TYPES[rng.integers(0, len(TYPES))]
        kinds.append((t, -1 if t == "Resource" else int(rng.integers(0, 2))))
    for (t, p), c in zip(kinds, free):
        x, y = int(c % w), int(c // w)
        r = int(rng.integers(5, 30)) if t == "Resource" else int(rng.integers(0, 2)) if t == "Worker" else 0
        hp = HP[t] if t in ("Resource", "Worker", "Ranged") else int(rng.integers(1, HP[t] + 1))
        units.append(f'<rts.units.Unit type="{t}" ID="{uid}" player="{p}" x="{x}" y="{y}" resources="{r}" hitpoints="{hp}" >'
                     "</rts.units.Unit>")
        uid += 1
    xml = (f'<rts.PhysicalGameState width="{w}" height="{h}"><terrain>{"".join(map(str, wall))}</terrain><players>'
           f'<rts.Player ID="0" resources="{res[0]}"></rts.Player><rts.Player ID="1" resources="{res[1]}"></rts.Player>'
           f'</players><units>{"".join(units)}</units></rts.PhysicalGameState>')
    with open(path, "w") as f:
        f.write(xml)
    return path
