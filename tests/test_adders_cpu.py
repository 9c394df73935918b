"""Adders against the reference's own golden tables (tests/golden/adder_cases.json, data
transcribed from acme/adders/reverb/transition_test.py:29-170 and sequence_test.py:25-170),
with the writer life-cycle checks of acme/adders/reverb/test_utils.py:120-224."""

import json
import os

import numpy as np
import pytest

from acme_amd import dm_env
from acme_amd.adders import reverb as adders
from acme_amd.testing.fakes import FakeClient
from acme_amd.utils import tree

CASES = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "adder_cases.json")))


def _ts(d):
    if d["kind"] == "mid":
        return dm_env.transition(reward=d["reward"], observation=d["observation"],
                                 discount=d["discount"])
    return dm_env.termination(reward=d["reward"], observation=d["observation"])


def _run(adder, client, first, steps, expected):
    adder.add_first(dm_env.restart(first))
    for s in steps[:-1]:
        adder.add(s[0], _ts(s[1]), s[2] if len(s) == 3 else ())
    if len(steps) == 1:
        assert client.writers == []
    else:
        assert len(client.writers) == 1 and not client.writers[0].closed
    last = steps[-1]
    adder.add(last[0], _ts(last[1]), last[2] if len(last) == 3 else ())
    assert len(client.writers) == 1 and client.writers[0].closed
    observed = [p[1] for p in client.writers[0].priorities]
    # The reference compares with zip(expected, observed) (test_utils.py:385-392), so an
    # adder emitting fewer items than listed still passes there.  One golden case relies
    # on that: EarlyTerminationNoPadding lists a 3-step item, but SequenceAdder only emits
    # when `sequence_length` steps exist (sequence.py:111-116) and, unpadded, never gets
    # there.  We follow the reference CODE (no item) and pin the count exactly.
    n_expected = 0 if getattr(adder, "_pad", True) is False else len(expected)
    assert len(observed) == n_expected
    for exp, got in zip(expected, observed):
        fe, fg = tree.flatten(exp), tree.flatten(got)
        assert len(fe) == len(fg), (exp, got)
        np.testing.assert_array_almost_equal(np.array(fe, np.float64), np.array(fg, np.float64))
    assert all(p[2] == 1.0 and p[0] == adders.DEFAULT_PRIORITY_TABLE
               for p in client.writers[0].priorities)
    # A second trajectory opens a new writer (lazily).
    adder.add_first(dm_env.restart(first))
    s = steps[0]
    adder.add(s[0], _ts(s[1]), s[2] if len(s) == 3 else ())
    assert len(client.writers) == 2
    assert client.writers[1].closed == (s[1]["kind"] == "last")


@pytest.mark.parametrize("case", CASES["transition"], ids=lambda c: c["name"])
def test_nstep_transition_golden(case):
    client = FakeClient()
    adder = adders.NStepTransitionAdder(client, case["n_step"], case["discount"])
    _run(adder, client, case["first"], case["steps"], case["expected"])


@pytest.mark.parametrize("case", CASES["sequence"], ids=lambda c: c["name"])
def test_sequence_golden(case):
    client = FakeClient()
    adder = adders.SequenceAdder(client, sequence_length=case["sequence_length"],
                                 period=case["period"],
                                 pad_end_of_episode=case.get("pad_end_of_episode", True))
    _run(adder, client, case["first"], case["steps"], case["expected"])


def _trajectory(observations):
    first = observations[0]
    steps = [[0, {"kind": "mid", "reward": 0.0, "observation": o, "discount": 1.0}]
             for o in observations[1:-1]]
    steps.append([0, {"kind": "last", "reward": 0.0, "observation": observations[-1],
                      "discount": 0.0}])
    return first, steps


@pytest.mark.parametrize("length", [2, 10, 50])
def test_episode_adder(length):
    """acme/adders/reverb/episode_test.py:26-40: one item holding the whole episode."""
    obs = list(range(length))
    first, steps = _trajectory(obs)
    expected = [[[o, 0, 0.0, 1.0 if i < length - 2 else 0.0, i == 0, []]
                 for i, o in enumerate(obs[:-1])] + [[obs[-1], 0, 0.0, 0.0, False, []]]]
    client = FakeClient()
    _run(adders.EpisodeAdder(client, length), client, first, steps, expected)


@pytest.mark.parametrize("length", [2, 10, 50])
def test_episode_adder_max_length(length):
    client = FakeClient()
    adder = adders.EpisodeAdder(client, length)
    first, steps = _trajectory(list(range(length + 1)))
    adder.add_first(dm_env.restart(first))
    for s in steps[:-1]:
        adder.add(s[0], _ts(s[1]))
    assert len(client.writers[0].timesteps) == length - 1
    with pytest.raises(ValueError):
        adder.add(steps[-1][0], _ts(steps[-1][1]))
    assert len(client.writers[0].timesteps) == length - 1


def test_misuse_raises():
    adder = adders.NStepTransitionAdder(FakeClient(), 3, 0.99)
    with pytest.raises(ValueError):
        adder.add(0, dm_env.transition(0.0, 1))
    with pytest.raises(ValueError):
        adder.add_first(dm_env.transition(0.0, 1))
    adder.add_first(dm_env.restart(1))
    with pytest.raises(ValueError):
        adder.add_first(dm_env.restart(1))
    with pytest.raises(ValueError):
        adders.NStepTransitionAdder(FakeClient(), 0, 0.99)


def test_custom_priority_fn_and_tables():
    client = FakeClient()
    adder = adders.NStepTransitionAdder(
        client, 2, 1.0, priority_fns={"a": lambda x: float(np.sum(x.rewards)), "b": lambda x: 2.0})
    with pytest.raises(ValueError):
        adder.add_priority_table("a", lambda x: 0.0)
    adder.add_first(dm_env.restart(1))
    adder.add(0, dm_env.transition(3.0, 2))
    adder.add(0, dm_env.termination(5.0, 3))
    pr = client.writers[0].priorities
    # Priority input stacks the window plus the zero-filled closing step.
    assert [(t, p) for t, _, p in pr] == [("a", 3.0), ("b", 2.0), ("a", 8.0), ("b", 2.0),
                                          ("a", 5.0), ("b", 2.0)]
