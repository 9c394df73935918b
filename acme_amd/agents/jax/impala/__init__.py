"""JAX IMPALA learner (drop-in for acme.agents.jax.impala.IMPALALearner)."""
from acme_amd.agents.jax.impala.learning import IMPALALearner  # noqa: F401
