"""_set_states_atomic (vec_env.py): several engines restored as one operation (multi-engine
checkpoints).  ADVICE r5: when an engine refuses its snapshot, the engines before it AND the
refusing engine itself (mrts_load_state may fail after its header checks) are put back.
Host logic only: fake engines, no GPU."""
import pytest


class FakeEngine:
    def __init__(self, name, fail_on=None):
        self.name, self.state, self.fail_on, self.calls = name, f"{name}:0", fail_on, []

    def _check_state(self, st):
        pass

    def get_state(self):
        return self.state

    def set_state(self, st):
        self.calls.append(st)
        if st == self.fail_on:
            self.state = f"{self.name}:half"   # a load that fails part-way
            raise RuntimeError("refused")
        self.state = st
        return st


def test_rollback_includes_the_refusing_engine():
    from gym_microrts.envs.vec_env import _set_states_atomic

    a, b, c = FakeEngine("a"), FakeEngine("b", fail_on="b:1"), FakeEngine("c")
    with pytest.raises(RuntimeError):
        _set_states_atomic([a, b, c], ["a:1", "b:1", "c:1"])
    assert (a.state, b.state, c.state) == ("a:0", "b:0", "c:0")
    assert c.calls == []   # never reached


def test_all_restored_when_none_refuses():
    from gym_microrts.envs.vec_env import _set_states_atomic

    es = [FakeEngine(n) for n in "xyz"]
    assert _set_states_atomic(es, ["x:1", "y:1", "z:1"]) == ["x:1", "y:1", "z:1"]
    assert [e.state for e in es] == ["x:1", "y:1", "z:1"]
