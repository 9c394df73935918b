"""Optimizer descriptors (the learners run Adam inside the HIP step).

Stand-in for the `snt.optimizers.Adam(learning_rate)` objects the reference passes to its
learners (e.g. acme/agents/tf/d4pg/agent.py:149-152): only the hyper-parameters travel."""

from __future__ import annotations

import dataclasses


@dataclasses.dataclass(frozen=True)
class Adam:
    learning_rate: float = 1e-3
    beta1: float = 0.9
    beta2: float = 0.999
    epsilon: float = 1e-8
