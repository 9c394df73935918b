"""ProcessActorPool (agents/impala/process_actors.py): environments and SequenceAdders in
worker processes, the policy batched in the parent, items through shared-memory rings.
Per environment it must behave exactly as IMPALAActor with a SequenceAdder
(acme/agents/tf/impala/acting.py:30-95, acme/adders/reverb/sequence.py): the same actions,
the same items (observations, actions, rewards, discounts, episode starts, extras with the
step's logits and the LSTM state before it), the state reset at episode starts.  The items
of the pool's rings are compared, as packed rows, with the items the reference actor's
adder hands to its client, over several episodes of every environment."""

import functools
import hashlib

import numpy as np
import pytest

from acme_amd import specs
from acme_amd.adders import reverb as adders
from acme_amd.adders.reverb._common import stack_steps
from acme_amd.agents.impala.acting import IMPALAActor
from acme_amd.agents.impala.process_actors import (ProcessActorPool, atari_like_oar,
                                                   sequence_fields)
from acme_amd.networks import LSTMState
from acme_amd.testing import fakes
from acme_amd.utils import tree

A, H, T = 6, 8, 5


def policy(obs, prev_a, prev_r, h, c):
    """Row-wise and deterministic: one action has all the mass (from the frame and the
    previous action), so any correct categorical sampler picks it; the state evolves."""
    n = obs.shape[0]
    pick = (obs.reshape(n, -1)[:, ::97].astype(np.int64).sum(axis=1) + prev_a) % A
    logits = np.full((n, A), -60.0, np.float32)
    logits[np.arange(n), pick] = 60.0
    logits += np.arange(A, dtype=np.float32)[None] * 0.01
    return (logits, np.zeros(n, np.float32), (h + 1.0).astype(np.float32),
            (0.5 * c + prev_r[:, None]).astype(np.float32))


def initial_state(b):
    return LSTMState(np.full((b, H), 0.25, np.float32), np.zeros((b, H), np.float32))


def _env(i):
    return atari_like_oar(i, seed=11, num_actions=A, min_length=4, max_length=9)


def _signature():
    env = _env(0)
    spec = specs.make_environment_spec(env)
    extra = {"core_state": LSTMState(specs.Array((H,), np.float32), specs.Array((H,), np.float32)),
             "logits": specs.Array((A,), np.float32)}
    return adders.SequenceAdder.signature(spec, extras_spec=extra)


def _pack(item, fields):
    if isinstance(item, list):  # FakeWriter keeps a T-step item as its list of steps
        item = stack_steps(item)
    rows = []
    for leaf, (shape, dt, nb, rb) in zip(tree.flatten(item), fields):
        a = np.ascontiguousarray(np.asarray(leaf, dt))
        assert a.shape == shape, (a.shape, shape)
        r = np.zeros(rb, np.uint8)
        r[:nb] = a.reshape(-1).view(np.uint8)
        rows.append(r.tobytes())
    return hashlib.sha256(b"".join(rows)).hexdigest()


def _reference_items(i, steps, fields):
    env, client = _env(i), fakes.FakeClient()
    actor = IMPALAActor(policy, initial_state,
                        adders.SequenceAdder(client, sequence_length=T, period=T), seed=0)
    ts = env.reset()
    actor.observe_first(ts)
    for _ in range(steps):
        a = actor.select_action(ts.observation)
        ts = env.step(a)
        actor.observe(a, ts)
        if ts.last():
            ts = env.reset()
            actor.observe_first(ts)
    return [_pack(item, fields) for w in client.writers for (_, item, _) in w.priorities]


class Pipelined:
    """The issue/result form of `policy` (as IMPALALearner.pipelined_policy)."""

    def issue(self, *args):
        self._out = policy(*[np.array(a) for a in args])

    def result(self):
        return self._out


@pytest.mark.parametrize("pipelined", [False, True])
def test_process_pool_items_equal_impala_actor_items(pipelined):
    N, steps = 6, 23
    fields = sequence_fields(_signature(), T)
    got = []

    def sink(rows, n):
        for k in range(n):
            got.append(hashlib.sha256(b"".join(r[k].tobytes() for r in rows)).hexdigest())

    pool = ProcessActorPool(functools.partial(_env), fields, (84, 84, 4), A, H, initial_state,
                            num_actors=N, processes=3, groups=2, sequence_length=T, period=T,
                            ring_items=2)
    try:
        pool.start()
        pool.run([Pipelined(), Pipelined()] if pipelined else policy, sink, ticks=steps)
        assert pool.env_steps == N * steps
    finally:
        pool.close()
    want = [h for i in range(N) for h in _reference_items(i, steps, fields)]
    assert len(want) > 2 * N  # several items per environment, episode ends included
    assert sorted(got) == sorted(want)
