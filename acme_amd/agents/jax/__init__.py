"""Drop-ins for the JAX learners (acme/agents/jax): same math on the same HIP kernels, with
the JAX learners' numerical semantics selected by ACME_SEMANTICS_JAX (include/acme_hip.h)."""
