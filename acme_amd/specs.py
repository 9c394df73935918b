"""Environment specs (acme/specs.py:34-49): the observation / action / reward / discount
specs an agent is built from."""

from typing import Any, NamedTuple

from acme_amd import dm_env

Array = dm_env.specs.Array
BoundedArray = dm_env.specs.BoundedArray
DiscreteArray = dm_env.specs.DiscreteArray


class EnvironmentSpec(NamedTuple):
    observations: Any
    actions: Any
    rewards: Any
    discounts: Any


def make_environment_spec(environment) -> EnvironmentSpec:
    return EnvironmentSpec(observations=environment.observation_spec(),
                           actions=environment.action_spec(),
                           rewards=environment.reward_spec(),
                           discounts=environment.discount_spec())
