"""DQN agent + learner (drop-in for acme.agents.tf.dqn)."""
from acme_amd.agents.dqn.agent import DQN  # noqa: F401
from acme_amd.agents.dqn.learning import DQNLearner  # noqa: F401
