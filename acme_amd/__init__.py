"""acme_amd — MI355X-native Acme learner core.

Drop-in surface (same names as the reference package `acme`):
  acme_amd.core           Actor, Learner, VariableSource, Worker, Saveable
  acme_amd.specs          EnvironmentSpec, make_environment_spec
  acme_amd.EnvironmentLoop
  acme_amd.adders.reverb  NStepTransitionAdder, SequenceAdder, EpisodeAdder
  acme_amd.replay         Table / Server / Client (GPU-resident Reverb replacement)
  acme_amd.datasets       make_reverb_dataset (device-side sample + gather)
  acme_amd.agents.dqn     DQN, DQNLearner (HIP learner step)
The compute path is libacme_hip.so (include/acme_hip.h); there is no CPU fallback.
"""

from acme_amd import core, specs  # noqa: F401
from acme_amd.environment_loop import EnvironmentLoop  # noqa: F401
from acme_amd.specs import make_environment_spec  # noqa: F401

__version__ = "0.1.0"
