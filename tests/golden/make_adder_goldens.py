"""Writes tests/golden/adder_cases.json: the reference's own adder golden vectors, as data.

Transcribed from the parameterized cases of
  acme/adders/reverb/transition_test.py:29-170  (NStepTransitionAdder, 7 cases)
  acme/adders/reverb/sequence_test.py:25-170    (SequenceAdder, 7 cases)
Each case: the first observation, the (action, timestep[, extras]) steps, and the items
the adder must create.  Timestep kinds: "mid" = dm_env.transition(reward, obs, discount),
"last" = dm_env.termination(reward, obs) (discount 0).
Sequence items are lists of steps (observation, action, reward, discount,
start_of_episode, extras).
"""

import json
import os


def mid(r, o, d=1.0):
    return {"kind": "mid", "reward": r, "observation": o, "discount": d}


def last(r, o):
    return {"kind": "last", "reward": r, "observation": o, "discount": 0.0}


TRANSITION = [
    dict(name="OneStepFinalReward", n_step=1, discount=1.0, first=1,
         steps=[[0, mid(0.0, 2)], [0, mid(0.0, 3)], [0, last(1.0, 4)]],
         expected=[[1, 0, 0.0, 1.0, 2], [2, 0, 0.0, 1.0, 3], [3, 0, 1.0, 0.0, 4]]),
    dict(name="OneStepDict", n_step=1, discount=1.0, first={"foo": 1},
         steps=[[0, mid(0.0, {"foo": 2})], [0, mid(0.0, {"foo": 3})], [0, last(1.0, {"foo": 4})]],
         expected=[[{"foo": 1}, 0, 0.0, 1.0, {"foo": 2}], [{"foo": 2}, 0, 0.0, 1.0, {"foo": 3}],
                   [{"foo": 3}, 0, 1.0, 0.0, {"foo": 4}]]),
    dict(name="OneStepExtras", n_step=1, discount=1.0, first=1,
         steps=[[0, mid(0.0, 2), {"state": 0}], [0, mid(0.0, 3), {"state": 1}],
                [0, last(1.0, 4), {"state": 2}]],
         expected=[[1, 0, 0.0, 1.0, 2, {"state": 0}], [2, 0, 0.0, 1.0, 3, {"state": 1}],
                   [3, 0, 1.0, 0.0, 4, {"state": 2}]]),
    dict(name="TwoStep", n_step=2, discount=1.0, first=1,
         steps=[[0, mid(1.0, 2, 0.5)], [0, mid(1.0, 3, 0.5)], [0, last(1.0, 4)]],
         expected=[[1, 0, 1.0, 0.50, 2], [1, 0, 1.5, 0.25, 3], [2, 0, 1.5, 0.00, 4],
                   [3, 0, 1.0, 0.00, 4]]),
    dict(name="TwoStepWithExtras", n_step=2, discount=1.0, first=1,
         steps=[[0, mid(1.0, 2, 0.5), {"state": 0}], [0, mid(1.0, 3, 0.5), {"state": 1}],
                [0, last(1.0, 4), {"state": 2}]],
         expected=[[1, 0, 1.0, 0.50, 2, {"state": 0}], [1, 0, 1.5, 0.25, 3, {"state": 0}],
                   [2, 0, 1.5, 0.00, 4, {"state": 1}], [3, 0, 1.0, 0.00, 4, {"state": 2}]]),
    dict(name="ThreeStepDiscounted", n_step=3, discount=0.4, first=1,
         steps=[[0, mid(1.0, 2, 0.5)], [0, mid(1.0, 3, 0.5)], [0, last(1.0, 4)]],
         expected=[[1, 0, 1.00, 0.5, 2], [1, 0, 1.20, 0.1, 3], [1, 0, 1.24, 0.0, 4],
                   [2, 0, 1.20, 0.0, 4], [3, 0, 1.00, 0.0, 4]]),
    dict(name="ThreeStepVaryingReward", n_step=3, discount=0.5, first=1,
         steps=[[0, mid(2.0, 2)], [0, mid(3.0, 3)], [0, mid(5.0, 4)], [0, last(7.0, 5)]],
         expected=[[1, 0, 2.0, 1.00, 2], [1, 0, 2 + 0.5 * 3, 0.50, 3],
                   [1, 0, 2 + 0.5 * 3 + 0.25 * 5, 0.25, 4], [2, 0, 3 + 0.5 * 5 + 0.25 * 7, 0.00, 5],
                   [3, 0, 5 + 0.5 * 7, 0.00, 5], [4, 0, 7.0, 0.00, 5]]),
]

_S4 = [[0, mid(2.0, 2)], [0, mid(3.0, 3)], [0, mid(5.0, 4)], [0, last(7.0, 5)]]
_S2 = [[0, mid(2.0, 2)], [0, last(3.0, 3)]]
SEQUENCE = [
    dict(name="PeriodOne", sequence_length=3, period=1, first=1, steps=_S4,
         expected=[[[1, 0, 2.0, 1.0, True, []], [2, 0, 3.0, 1.0, False, []], [3, 0, 5.0, 1.0, False, []]],
                   [[2, 0, 3.0, 1.0, False, []], [3, 0, 5.0, 1.0, False, []], [4, 0, 7.0, 0.0, False, []]],
                   [[3, 0, 5.0, 1.0, False, []], [4, 0, 7.0, 0.0, False, []], [5, 0, 0.0, 0.0, False, []]]]),
    dict(name="PeriodTwo", sequence_length=3, period=2, first=1, steps=_S4,
         expected=[[[1, 0, 2.0, 1.0, True, []], [2, 0, 3.0, 1.0, False, []], [3, 0, 5.0, 1.0, False, []]],
                   [[3, 0, 5.0, 1.0, False, []], [4, 0, 7.0, 0.0, False, []], [5, 0, 0.0, 0.0, False, []]]]),
    dict(name="EarlyTerminationPeriodOne", sequence_length=3, period=1, first=1, steps=_S2,
         expected=[[[1, 0, 2.0, 1.0, True, []], [2, 0, 3.0, 0.0, False, []], [3, 0, 0.0, 0.0, False, []]]]),
    dict(name="EarlyTerminationPeriodTwo", sequence_length=3, period=2, first=1, steps=_S2,
         expected=[[[1, 0, 2.0, 1.0, True, []], [2, 0, 3.0, 0.0, False, []], [3, 0, 0.0, 0.0, False, []]]]),
    dict(name="EarlyTerminationPaddingPeriodOne", sequence_length=4, period=1, first=1, steps=_S2,
         expected=[[[1, 0, 2.0, 1.0, True, []], [2, 0, 3.0, 0.0, False, []], [3, 0, 0.0, 0.0, False, []],
                    [0, 0, 0.0, 0.0, False, []]]]),
    dict(name="EarlyTerminationPaddingPeriodTwo", sequence_length=4, period=2, first=1, steps=_S2,
         expected=[[[1, 0, 2.0, 1.0, True, []], [2, 0, 3.0, 0.0, False, []], [3, 0, 0.0, 0.0, False, []],
                    [0, 0, 0.0, 0.0, False, []]]]),
    dict(name="EarlyTerminationNoPadding", sequence_length=4, period=1, first=1, steps=_S2,
         pad_end_of_episode=False,
         expected=[[[1, 0, 2.0, 1.0, True, []], [2, 0, 3.0, 0.0, False, []], [3, 0, 0.0, 0.0, False, []]]]),
]

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "adder_cases.json")
    with open(out, "w") as f:
        json.dump({"source": {"transition": "acme/adders/reverb/transition_test.py:29-170",
                              "sequence": "acme/adders/reverb/sequence_test.py:25-170"},
                   "transition": TRANSITION, "sequence": SEQUENCE}, f, indent=1)
    print(out)
