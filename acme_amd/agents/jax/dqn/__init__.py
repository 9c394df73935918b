"""JAX DQN learner (drop-in for acme.agents.jax.dqn.DQNLearner)."""
from acme_amd.agents.jax.dqn.learning import DQNLearner  # noqa: F401
