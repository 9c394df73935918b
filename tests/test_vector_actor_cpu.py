"""VectorActor (agents/impala/actors.py) behaves, per environment, exactly as IMPALAActor
(acme/agents/tf/impala/acting.py:30-95): the same actions, the same adder calls with the
same extras (logits of the step, the LSTM state before it) and the state reset at episode
starts, for K environments stepped with one batched policy call (chunked or not)."""

import numpy as np
import pytest

from acme_amd.agents.impala.acting import IMPALAActor
from acme_amd.agents.impala.actors import VectorActor
from acme_amd.environments.atari_like import AtariLike
from acme_amd.networks import LSTMState
from acme_amd.wrappers import ObservationActionRewardWrapper

A, H = 6, 8


def policy(obs, prev_a, prev_r, h, c):
    """Row-wise and deterministic: one action has all the mass (chosen from the frame and
    the previous action), so any correct categorical sampler picks it."""
    n = obs.shape[0]
    pick = (obs.reshape(n, -1)[:, ::97].astype(np.int64).sum(axis=1) + prev_a) % A
    logits = np.full((n, A), -60.0, np.float32)
    logits[np.arange(n), pick] = 60.0
    return (logits, np.zeros(n, np.float32), (h + 1.0).astype(np.float32),
            (0.5 * c + prev_r[:, None]).astype(np.float32))


def initial_state(b):
    z = np.zeros((b, H), np.float32)
    return LSTMState(z, z.copy())


class Recorder:
    def __init__(self):
        self.log = []

    def add_first(self, ts):
        self.log.append(("first", ts.observation.observation.copy()))

    def add(self, action, ts, extras):
        cs = extras["core_state"]
        self.log.append(("add", int(action), ts.observation.observation.copy(), float(ts.reward),
                         np.array(extras["logits"]), np.array(cs.hidden), np.array(cs.cell)))


def env(seed):
    return ObservationActionRewardWrapper(AtariLike(seed=seed, num_actions=A, min_length=5,
                                                    max_length=12))


def reference(seed, steps):
    e, rec = env(seed), Recorder()
    actor = IMPALAActor(policy, initial_state, rec, seed=0)
    ts = e.reset()
    actor.observe_first(ts)
    for _ in range(steps):
        a = actor.select_action(ts.observation)
        ts = e.step(a)
        actor.observe(a, ts)
        if ts.last():
            ts = e.reset()
            actor.observe_first(ts)
    return rec.log


@pytest.mark.parametrize("max_rows", [None, 2])
def test_vector_actor_matches_impala_actor(max_rows):
    seeds, steps = [3, 4, 5], 40
    recs = [Recorder() for _ in seeds]
    va = VectorActor([env(s) for s in seeds], recs, policy, initial_state, seed=1,
                     max_rows=max_rows)
    va.start()
    for _ in range(steps):
        va.step()
    assert va.steps == steps * len(seeds)
    for s, rec in zip(seeds, recs):
        ref = reference(s, steps)
        assert len(rec.log) == len(ref)
        for got, want in zip(rec.log, ref):
            assert got[0] == want[0]
            for x, y in zip(got[1:], want[1:]):
                np.testing.assert_array_equal(x, y)
