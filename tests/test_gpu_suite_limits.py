"""The -m gpu suite stays inside the driver's round-end time limit:
every GPU test carries its own @pytest.mark.timeout (module-level `pytestmark` or per
test), so one hung kernel ends its test, names it, and leaves the rest of the budget.
Collection only -- nothing here touches a GPU."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_COLLECT = r"""
import json, sys, pytest
class P:
    items = []
    def pytest_collection_finish(self, session):
        for it in session.items:
            m = it.get_closest_marker("timeout")
            P.items.append([it.nodeid, m.args[0] if m and m.args else (m.kwargs.get("timeout") if m else None)])
rc = pytest.main(["--collect-only", "-q", "-m", "gpu", "-p", "no:cacheprovider", "tests"], plugins=[P()])
print("@@" + json.dumps({"rc": int(rc), "items": P.items}))
"""


def _collect():
    out = subprocess.run([sys.executable, "-c", _COLLECT], cwd=REPO, capture_output=True, text=True, timeout=300)
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("@@")]
    assert line, out.stdout[-2000:] + out.stderr[-2000:]
    return json.loads(line[-1][2:])


def test_every_gpu_test_has_a_timeout():
    d = _collect()
    assert d["rc"] == 0, d
    items = d["items"]
    assert len(items) > 150, len(items)   # the suite was collected, not an import error
    missing = [n for n, t in items if t is None]
    assert not missing, f"GPU tests without @pytest.mark.timeout: {missing}"
    # no single test may take the driver's whole 900 s step on its own... except the
    # named full-size lock-steps, which the driver's suite budget accounts for.
    assert all(float(t) <= 1200 for _, t in items)
