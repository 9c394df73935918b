"""D4PG agent + learner (drop-in for acme.agents.tf.d4pg)."""
from acme_amd.agents.d4pg.agent import D4PG  # noqa: F401
from acme_amd.agents.d4pg.learning import D4PGLearner  # noqa: F401
