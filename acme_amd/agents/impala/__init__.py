"""IMPALA agent + learner + actor (drop-in for acme.agents.tf.impala)."""
from acme_amd.agents.impala.acting import IMPALAActor  # noqa: F401
from acme_amd.agents.impala.agent import IMPALA  # noqa: F401
from acme_amd.agents.impala.learning import IMPALALearner  # noqa: F401
