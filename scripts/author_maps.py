"""Author the PhysicalGameState map XMLs the build needs.

The reference's maps live in the absent submodule gym_microrts/microrts
(/root/reference/.gitmodules:1-3), so they are authored here in the same XML
format (/root/reference/PCG/maps/wall-1:1-16, /root/reference/PCG/pcg.py:38-153:
players with 5 resources, resource piles of 25, bases hp 10, workers hp 1).

Layouts are pinned where the reference tests pin them:
  * 16x16/basesWorkers16x16A: tests/test_observation.py:61-78
  * 4x4/baseTwoWorkers4x4:    tests/test_mask.py:28-84, tests/test_reward.py
  * barricades24x24 wall (6,6): tests/test_observation.py:98-108
Everything else is an authored layout (parity unpinned for its geometry).

Run: python scripts/author_maps.py   (writes under microrts-py_amd/gym_microrts/microrts/maps)
"""
import os

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "microrts-py_amd", "gym_microrts", "microrts", "maps")


def write_map(rel, w, h, units, walls=(), res=(5, 5)):
    terrain = ["0"] * (w * h)
    for (x, y) in walls:
        terrain[y * w + x] = "1"
    lines = [f'<rts.PhysicalGameState width="{w}" height="{h}">', f"  <terrain>{''.join(terrain)}</terrain>", "  <players>"]
    for pid, r in enumerate(res):
        lines += [f'    <rts.Player ID="{pid}" resources="{r}">', "    </rts.Player>"]
    lines += ["  </players>", "  <units>"]
    for uid, (t, p, x, y, r, hp) in enumerate(units):
        assert terrain[y * w + x] == "0", (rel, x, y)
        lines += [
            f'    <rts.units.Unit type="{t}" ID="{uid}" player="{p}" x="{x}" y="{y}" resources="{r}" hitpoints="{hp}" >',
            "    </rts.units.Unit>",
        ]
    lines += ["  </units>", "</rts.PhysicalGameState>", ""]
    path = os.path.join(ROOT, rel)
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        f.write("\n".join(lines))


def R(x, y, r=25):
    return ("Resource", -1, x, y, r, 1)


def B(p, x, y):
    return ("Base", p, x, y, 0, 10)


def W(p, x, y):
    return ("Worker", p, x, y, 0, 1)


def bases_workers(n, extra_res=()):
    """Point-symmetric bases+worker layout scaled to an n x n map."""
    m = n - 1
    return [R(0, 0), R(0, 1), R(m, m - 1), R(m, m), *extra_res, B(0, 2, 2), B(1, m - 2, m - 2), W(0, 1, 1), W(1, m - 1, m - 1)]


def main():
    # 16x16 (bench map + test map A share the pinned layout)
    write_map("16x16/basesWorkers16x16.xml", 16, 16, bases_workers(16))
    write_map("16x16/basesWorkers16x16A.xml", 16, 16, bases_workers(16))
    # 16x16 variants used by microrts_maps.ALL16x16_MAPS-style cycling (authored)
    write_map("16x16/basesWorkers16x16B.xml", 16, 16,
              [R(0, 0), R(1, 0), R(15, 15), R(14, 15), B(0, 3, 2), B(1, 12, 13), W(0, 2, 1), W(1, 13, 14)])
    write_map("16x16/basesWorkers16x16C.xml", 16, 16,
              [R(0, 15), R(0, 14), R(15, 0), R(15, 1), B(0, 2, 13), B(1, 13, 2), W(0, 1, 14), W(1, 14, 1)])
    write_map("16x16/basesWorkers16x16noResources.xml", 16, 16, [B(0, 2, 2), B(1, 13, 13), W(0, 1, 1), W(1, 14, 14)])
    write_map("16x16/TwoBasesBarracks16x16.xml", 16, 16,
              [R(0, 0), R(0, 1), R(15, 14), R(15, 15), B(0, 2, 2), ("Barracks", 0, 4, 2, 0, 4), B(1, 13, 13),
               ("Barracks", 1, 11, 13, 0, 4), W(0, 1, 1), W(1, 14, 14)])
    # the rest of microrts_maps.ALL16x16_MAPS (authored, point-symmetric; parity unpinned for geometry)
    def sym(units):   # add player 1's point-symmetric copy of player-0 / neutral units
        out = []
        for (t, p, x, y, r, hp) in units:
            out.append((t, p, x, y, r, hp))
            out.append((t, -1 if p < 0 else 1 - p, 15 - x, 15 - y, r, hp))
        return out
    variants = {   # base (x, y), worker (x, y), resource piles
        "D": ((2, 3), (1, 3), [(0, 2), (0, 3)]), "E": ((3, 3), (2, 2), [(0, 0), (1, 0)]),
        "F": ((2, 4), (1, 4), [(0, 5), (0, 6)]), "G": ((4, 2), (4, 1), [(5, 0), (6, 0)]),
        "H": ((3, 2), (3, 1), [(0, 0), (0, 1), (1, 0)]), "I": ((2, 2), (2, 1), [(0, 3), (0, 4)]),
        "J": ((5, 2), (5, 1), [(0, 0), (7, 0)]), "K": ((2, 5), (1, 5), [(0, 0), (0, 7)]),
        "L": ((4, 4), (3, 3), [(0, 0), (0, 1), (1, 0), (1, 1)]),
    }
    for v, (b, wk, piles) in variants.items():
        write_map(f"16x16/basesWorkers16x16{v}.xml", 16, 16,
                  sym([R(x, y) for (x, y) in piles] + [B(0, *b), W(0, *wk)]))
    write_map("16x16/basesWorkers16x16R20.xml", 16, 16, sym([R(0, 0, 20), R(0, 1, 20), B(0, 2, 2), W(0, 1, 1)]), res=(20, 20))
    write_map("16x16/EightBasesWorkers16x16.xml", 16, 16,
              sym([R(0, 0), R(0, 15), B(0, 2, 2), B(0, 2, 6), B(0, 6, 2), B(0, 2, 10), W(0, 1, 1), W(0, 3, 6), W(0, 6, 3),
                   W(0, 3, 10)]))

    def army(kinds):   # melee maps: two armies facing each other, no bases
        units = []
        for i, k in enumerate(kinds):
            hp = {"Light": 4, "Heavy": 4, "Ranged": 1, "Worker": 1}[k]
            units.append((k, 0, 4 + (i % 8), 3 + i // 8, 0, hp))
        return sym(units)
    write_map("16x16/melee16x16Mixed8.xml", 16, 16, army(["Light", "Heavy", "Ranged", "Worker"] * 2))
    write_map("16x16/melee16x16Mixed12.xml", 16, 16, army(["Light", "Heavy", "Ranged", "Worker"] * 3))
    # 4x4 mask / reward test map
    write_map("4x4/baseTwoWorkers4x4.xml", 4, 4,
              [R(0, 0), R(3, 3), B(0, 1, 1), B(1, 2, 2), W(0, 1, 0), W(0, 0, 1), W(1, 2, 3), W(1, 3, 2)])
    # 8x8 and 24x24 size buckets
    write_map("8x8/basesWorkers8x8.xml", 8, 8, bases_workers(8))
    write_map("24x24/basesWorkers24x24.xml", 24, 24, bases_workers(24))
    # reference default map (vec_env.py:95)
    write_map("10x10/basesTwoWorkers10x10.xml", 10, 10,
              [R(0, 0), R(9, 9), B(0, 2, 2), B(1, 7, 7), W(0, 1, 1), W(0, 2, 1), W(1, 8, 8), W(1, 7, 8)])
    # 32x32: the largest map the engine takes (fused bot LDS > 64 KB)
    write_map("32x32/basesWorkers32x32.xml", 32, 32, bases_workers(32))
    # 40 barracks for player 0 (issue()'s pending-produce candidates beyond 16)
    field = [("Barracks", 0, x, y, 0, 4) for y in (1, 4, 7, 10, 13) for x in range(0, 16, 2)]
    write_map("16x16/barracksField16x16.xml", 16, 16, field + [B(1, 15, 15), W(1, 15, 14)], res=(40, 5))
    # walled maps whose cell count is not a multiple of 4 (the fused k_step's early bot
    # reads the step's terrain in place there: VERDICT r2 item 1); any size is legal
    # (PCG/pcg.py:9-10 draws width and height freely), the terrain format is PCG/maps/wall-1
    write_map("15x15/basesWorkersWalls15x15.xml", 15, 15,
              [R(0, 0), R(0, 1), R(14, 14), R(14, 13), B(0, 2, 2), B(1, 12, 12), W(0, 1, 1), W(1, 13, 13)],
              walls=[(7, 5), (7, 6), (7, 8), (7, 9), (5, 7), (6, 7), (8, 7), (9, 7), (4, 2), (4, 3), (10, 12), (10, 11)])
    write_map("9x13/basesWorkersWalls9x13.xml", 9, 13,
              [R(0, 0), R(0, 1), R(8, 12), R(8, 11), B(0, 2, 2), B(1, 6, 10), W(0, 1, 1), W(1, 7, 11)],
              walls=[(1, 6), (2, 6), (3, 6), (5, 6), (6, 6), (7, 6), (4, 3), (4, 9)])
    # barricades: wall at (6,6) pinned, the rest authored (point symmetric)
    walls = []
    for k in range(6, 10):
        walls += [(6, k), (k, 6), (23 - 6, 23 - k), (23 - k, 23 - 6)]
    walls += [(11, 11), (12, 12), (11, 12), (12, 11)]
    write_map("barricades24x24.xml", 24, 24,
              [R(0, 0), R(0, 1), R(1, 0), R(23, 23), R(23, 22), R(22, 23), B(0, 3, 3), B(1, 20, 20), W(0, 2, 2), W(1, 21, 21)],
              walls=sorted(set(walls)))


if __name__ == "__main__":
    main()
