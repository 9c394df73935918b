"""Host-side plumbing without a GPU: EnvironmentLoop counts (acme/environment_loop_test.py
:36-51), Agent learner-step cadence (acme/agents/agent.py:45-89), Counter, checkpoint
round trip, CartPole restatement, nest utilities."""

import numpy as np
import pytest

from acme_amd import core, dm_env, specs
from acme_amd.agents.agent import Agent
from acme_amd.environment_loop import EnvironmentLoop
from acme_amd.environments.cartpole import CartPole
from acme_amd.testing import fakes
from acme_amd.utils import counting, loggers, savers, tree


class _CountingActor(core.Actor):
    def __init__(self):
        self.calls = dict(select=0, first=0, observe=0, update=0)

    def select_action(self, observation):
        self.calls["select"] += 1
        return np.int32(0)

    def observe_first(self, timestep):
        self.calls["first"] += 1

    def observe(self, action, next_timestep):
        self.calls["observe"] += 1

    def update(self):
        self.calls["update"] += 1


@pytest.mark.parametrize("episode_length", [1, 10])
def test_environment_loop_counts(episode_length):
    env = fakes.DiscreteEnvironment(episode_length=episode_length)
    actor = _CountingActor()
    log = loggers.InMemoryLogger()
    loop = EnvironmentLoop(env, actor, logger=log)
    loop.run(num_episodes=10)
    assert actor.calls == dict(select=10 * episode_length, first=10,
                               observe=10 * episode_length, update=10 * episode_length)
    assert len(log.data) == 10
    assert log.data[-1]["episodes"] == 10 and log.data[-1]["steps"] == 10 * episode_length
    with pytest.raises(ValueError):
        loop.run(num_episodes=1, num_steps=1)
    loop2 = EnvironmentLoop(env, actor, logger=loggers.NoOpLogger())
    before = actor.calls["select"]
    loop2.run(num_steps=2 * episode_length + 1)  # always finishes the episode
    assert actor.calls["select"] - before == 3 * episode_length


class _StepCounter(core.Learner):
    def __init__(self):
        self.steps = 0

    def step(self):
        self.steps += 1

    def get_variables(self, names):
        return [names]


@pytest.mark.parametrize("min_obs,ops,expect", [(5, 2.0, 3), (0, 1.0, 10), (4, 0.25, 28)])
def test_agent_update_cadence(min_obs, ops, expect):
    learner = _StepCounter()
    agent = Agent(_CountingActor(), learner, min_observations=min_obs, observations_per_step=ops)
    ts = dm_env.transition(0.0, np.zeros(1))
    for _ in range(10):
        agent.observe(0, ts)
        agent.update()
    assert learner.steps == expect
    assert agent.get_variables(["a"]) == [["a"]]


def test_counter_parent_and_prefix():
    parent = counting.Counter()
    child = counting.Counter(parent, prefix="learner", time_delta=0.0)
    child.increment(steps=2)
    c = child.increment(steps=1)
    assert parent.get_counts() == {"learner_steps": 3}
    assert c["learner_steps"] == 3
    st = child.save()
    child2 = counting.Counter()
    child2.restore(st)


class _Saveable(core.Saveable):
    def __init__(self, x):
        self.x = x

    def save(self):
        return {"network": {"a/w": self.x, "a/b": self.x[:1]}, "num_steps": 7}

    def restore(self, state):
        self.x = state["network"]["a/w"]
        self.steps = state["num_steps"]


def test_checkpointer_roundtrip(tmp_path):
    s = _Saveable(np.arange(4.0))
    ck = savers.Checkpointer({"obj": s}, str(tmp_path), time_delta_minutes=60)
    assert not ck.save()  # time-gated
    assert ck.save(force=True)
    s2 = _Saveable(np.zeros(4))
    savers.Checkpointer({"obj": s2}, str(tmp_path))  # restores on construction
    np.testing.assert_array_equal(s2.x, np.arange(4.0))
    assert s2.steps == 7


def test_cartpole_dynamics():
    env = CartPole(seed=0)
    spec = specs.make_environment_spec(env)
    assert spec.actions.num_values == 2
    ts = env.reset()
    n = 0
    while not ts.last():
        ts = env.step(1)  # always push right: falls over quickly
        n += 1
    assert 5 < n < 60 and ts.discount == 0.0
    # One Euler step from rest with action 1 matches the closed form.
    env._state = np.zeros(4)
    env.step(1)
    total = 1.1
    temp = 10.0 / total
    th_acc = -temp / (0.5 * (4 / 3 - 0.1 / total))
    x_acc = temp - 0.05 * th_acc / total
    np.testing.assert_allclose(env._state, [0.0, 0.02 * x_acc, 0.0, 0.02 * th_acc], rtol=1e-12)


def test_tree_roundtrip():
    nest = {"b": (1, [2, 3]), "a": np.zeros(2)}
    flat = tree.flatten(nest)
    assert len(flat) == 4 and flat[1] == 1
    back = tree.unflatten_as(nest, flat)
    assert back["b"] == (1, [2, 3])
    assert tree.map_structure(lambda x, y: x, nest, nest)["b"][1] == [2, 3]
