"""Extract the reference's only map file, /root/reference/PCG/maps/wall-1:1-16,
as a test fixture (data: a PhysicalGameState XML -- 8x8, walled border, two bases,
unit IDs 2 and 3, no workers, no resources, no `.xml` extension).  The bytes are
copied unchanged to tests/golden/maps/wall-1 and their sha256 is recorded beside
them, so the GPU box (which has no /root/reference) loads the same map.

  python tests/golden/make_wall1_fixture.py
"""
import hashlib
import os
import sys

SRC = "/root/reference/PCG/maps/wall-1"
HERE = os.path.dirname(os.path.abspath(__file__))
DST = os.path.join(HERE, "maps", "wall-1")


def main():
    data = open(SRC, "rb").read()
    os.makedirs(os.path.dirname(DST), exist_ok=True)
    with open(DST, "wb") as f:
        f.write(data)
    with open(DST + ".sha256", "w") as f:
        f.write(hashlib.sha256(data).hexdigest() + "  wall-1 (from " + SRC + ")\n")
    print(f"{DST}: {len(data)} bytes")


if __name__ == "__main__":
    sys.exit(main())
