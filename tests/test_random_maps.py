"""The seeded random-map generator (tests/random_maps.py) writes maps the reference's format
parser reads back (oracle_py.parse_map, PhysicalGameState.load restated): the requested
size and unit count, no unit on a wall or on another unit, both players present, and the
same map for the same seed."""
import numpy as np
import pytest

from random_maps import write_random_map


@pytest.mark.parametrize("w,h,n", [(16, 16, 90), (12, 20, 80), (24, 24, 150), (8, 8, 40)])
def test_random_map_is_valid(tmp_path, w, h, n):
    from oracle_py import parse_map

    a = parse_map(write_random_map(str(tmp_path / "a.xml"), w, h, 7, n_units=n))
    b = parse_map(write_random_map(str(tmp_path / "b.xml"), w, h, 7, n_units=n))
    assert (a["width"], a["height"]) == (w, h) and len(a["units"]) == n
    cells = a["units"][:, 3] * w + a["units"][:, 2]
    assert len(set(cells.tolist())) == n and not a["terrain"][cells].any()
    assert {0, 1} <= set(a["units"][:, 1].tolist())
    assert np.array_equal(a["units"], b["units"]) and np.array_equal(a["terrain"], b["terrain"])
