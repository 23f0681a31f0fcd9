"""Generate tests/golden/maps/pcg/*.xml with the REFERENCE's own map generator.

Runs only in the build container (where /root/reference exists): loads
/root/reference/PCG/pcg.py (stdlib only: argparse, random, xml.etree) and calls its
PCG(...).get_map() (pcg.py:17-153) with `random` seeded per map.  The files are the
generator's own output bytes (get_map writes ./maps/filename.xml; this script runs it
in a scratch directory and keeps what it wrote).  MANIFEST.json records, per map, the
seed, the parameters the generator drew (wallRings), the file's sha256, and the
sha256 of the pcg.py that made it.  No reference source is copied: the fixtures are
data (map XMLs), like tests/golden/maps/wall-1.

The generator's own variation, all kept as it writes it:
* wallRings in [0, min(w, h) // 2 - 3] concentric wall rings (pcg.py:23-26) -- the
  seed search below picks a seed per wanted value, so every value is covered at 12x12
  and 16x16 and a spread at 8x8 / 24x24;
* random interior obstacles (pcg.py:43-48), 4 resource piles of 25, one base and one
  worker per side in random quadrant sections (pcg.py:76-133);
* non-square maps, whose x-wall test reads `self.height` (pcg.py:57): for w > h the
  "right" rings land on interior columns [h - r, h), for w < h they are absent;
* two bases per side: the generator's own initiate_bases (pcg.py:96-116) called twice
  (a subclass's initiate_units; its section choices and occupancy records are the
  generator's).

    python tests/golden/make_pcg_maps.py

A campaign set, `--campaign N` (tests/golden/maps/pcg_campaign.json): N more maps from the
same generator, each with its own seed, its size drawn from 8..24 (a quarter of them
non-square) and one or two bases per side, the generator drawing wallRings and the
obstacles itself -- the XML text of each is stored in the JSON (data, as the generator
wrote it) for tests/test_pcg_maps.py's campaign lock-step.
"""
import contextlib
import hashlib
import importlib.util
import json
import os
import random
import signal
import sys
import tempfile

REF_PCG = "/root/reference/PCG/pcg.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "maps", "pcg")

# (name, width, height, wallRings wanted, bases per side)
SPECS = [("pcg8x8_r0", 8, 8, 0, 1), ("pcg8x8_r1", 8, 8, 1, 1)]
SPECS += [(f"pcg12x12_r{r}", 12, 12, r, 1) for r in range(4)]
SPECS += [(f"pcg16x16_r{r}", 16, 16, r, 1) for r in range(6)]
SPECS += [(f"pcg24x24_r{r}", 24, 24, r, 1) for r in (0, 3, 6, 9)]
SPECS += [("pcg16x12_r2", 16, 12, 2, 1), ("pcg12x16_r1", 12, 16, 1, 1), ("pcg24x16_r3", 24, 16, 3, 1)]
SPECS += [("pcg16x16_r1_2bases", 16, 16, 1, 2), ("pcg24x24_r2_2bases", 24, 24, 2, 2), ("pcg12x12_r0_2bases", 12, 12, 0, 2)]


def load_pcg():
    sys.dont_write_bytecode = True
    spec = importlib.util.spec_from_file_location("reference_pcg", REF_PCG)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


class _Hang(Exception):
    pass


@contextlib.contextmanager
def _deadline(sec):
    """get_xy (pcg.py:135-144) redraws until it finds a free cell: a full section never
    ends.  Such a seed is skipped."""
    def on_alarm(*_):
        raise _Hang()

    old = signal.signal(signal.SIGALRM, on_alarm)
    signal.alarm(sec)
    try:
        yield
    finally:
        signal.alarm(0)
        signal.signal(signal.SIGALRM, old)


def generate(pcg, w, h, rings, bases, seed0):
    class TwoBases(pcg.PCG):
        def initiate_units(self, root, tag):
            import xml.etree.cElementTree as ET

            units = ET.SubElement(root, tag)
            self.initiate_resources(units, "rts.units.Unit")
            self.initiate_bases(units, "rts.units.Unit")
            self.initiate_bases(units, "rts.units.Unit")
            self.initiate_workers(units, "rts.units.Unit")

    cls = pcg.PCG if bases == 1 else TwoBases
    for seed in range(seed0, seed0 + 10_000):
        random.seed(seed)
        # fresh lists: PCG's defaults are shared mutable lists (pcg.py:18-19)
        g = cls(width=w, height=h, unit_location_records=[], base_location_records=[])
        if g.wallRings != rings:
            continue
        with tempfile.TemporaryDirectory() as d:
            os.makedirs(os.path.join(d, "maps"))
            cwd = os.getcwd()
            os.chdir(d)
            try:
                with _deadline(2):
                    g.get_map()
            except _Hang:
                continue
            finally:
                os.chdir(cwd)
            data = open(os.path.join(d, "maps", "filename.xml"), "rb").read()
        return seed, data
    raise RuntimeError(f"no seed for {w}x{h} rings={rings}")


def campaign(pcg, n, out):
    import numpy as np

    rng = np.random.default_rng(20261018)
    maps = []
    for k in range(n):
        w = int(rng.integers(8, 25))
        h = w if rng.random() < 0.75 else int(rng.integers(8, 25))
        bases = 1 if rng.random() < 0.7 else 2
        seed0, got = 100_000 + 1000 * k, None
        for seed in range(seed0, seed0 + 1000):   # any wallRings: the generator's own draw
            random.seed(seed)
            rings = pcg.PCG(width=w, height=h, unit_location_records=[], base_location_records=[]).wallRings
            try:
                got, data = generate(pcg, w, h, rings, bases, seed)
            except RuntimeError:
                continue
            if got == seed:
                break
        if got is None:
            raise RuntimeError(f"campaign map {k}: no seed in [{seed0}, {seed0 + 1000}) generated a {w}x{h} map")
        maps.append({"seed": got, "width": w, "height": h, "wallRings": rings, "bases_per_side": bases,
                     "xml": data.decode()})
    with open(out, "w") as f:
        json.dump({"generator": REF_PCG, "generator_sha256": hashlib.sha256(open(REF_PCG, "rb").read()).hexdigest(),
                   "maps": maps}, f)
        f.write("\n")
    print("wrote", out, len(maps), "maps")


def main():
    pcg = load_pcg()
    if len(sys.argv) == 3 and sys.argv[1] == "--campaign":
        return campaign(pcg, int(sys.argv[2]), os.path.join(os.path.dirname(OUT), "pcg_campaign.json"))
    src_sha = hashlib.sha256(open(REF_PCG, "rb").read()).hexdigest()
    os.makedirs(OUT, exist_ok=True)
    manifest = {"generator": "/root/reference/PCG/pcg.py", "generator_sha256": src_sha, "maps": []}
    for k, (name, w, h, rings, bases) in enumerate(SPECS):
        seed, data = generate(pcg, w, h, rings, bases, 1000 * (k + 1))
        with open(os.path.join(OUT, name + ".xml"), "wb") as f:
            f.write(data)
        manifest["maps"].append({"name": name + ".xml", "seed": seed, "width": w, "height": h, "wallRings": rings,
                                 "bases_per_side": bases, "sha256": hashlib.sha256(data).hexdigest()})
        print(name, "seed", seed, len(data), "bytes")
    with open(os.path.join(OUT, "MANIFEST.json"), "w") as f:
        json.dump(manifest, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
