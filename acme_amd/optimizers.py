"""Optimizer descriptors (the learners run Adam inside the HIP step).

Stand-in for the `snt.optimizers.Adam(learning_rate)` objects the reference passes to its
TF learners (e.g. acme/agents/tf/d4pg/agent.py:149-152) and for the `optix` chains its JAX
learners take (acme/agents/jax/dqn/agent.py:110 `optix.adam(learning_rate)`;
acme/agents/jax/impala/agent.py:98-101 `optix.chain(optix.clip_by_global_norm(c),
optix.adam(lr))`): only the hyper-parameters travel; the update itself is the fused HIP
kernel (kernels.hip: adam_kernel / clip_adam_kernel, optix rounding order for JAX learners)."""

from __future__ import annotations

import dataclasses
import math
from typing import Optional, Tuple


@dataclasses.dataclass(frozen=True)
class Adam:
    learning_rate: float = 1e-3
    beta1: float = 0.9
    beta2: float = 0.999
    epsilon: float = 1e-8


@dataclasses.dataclass(frozen=True)
class ClipByGlobalNorm:
    max_norm: float


@dataclasses.dataclass(frozen=True)
class Chain:
    transforms: Tuple


class optix:  # noqa: N801  (module-like namespace, as jax.experimental.optix)
    @staticmethod
    def adam(learning_rate: float, b1: float = 0.9, b2: float = 0.999,
             eps: float = 1e-8) -> Adam:
        return Adam(learning_rate, b1, b2, eps)

    @staticmethod
    def clip_by_global_norm(max_norm: float) -> ClipByGlobalNorm:
        return ClipByGlobalNorm(float(max_norm))

    @staticmethod
    def chain(*transforms) -> Chain:
        return Chain(tuple(transforms))


def unpack(optimizer) -> Tuple[Adam, Optional[float]]:
    """(Adam hyper-parameters, global-norm clip or None) of an optimizer descriptor; raises
    for transforms the fused kernels do not implement."""
    if isinstance(optimizer, Adam):
        return optimizer, None
    if isinstance(optimizer, Chain):
        adam, clip = None, None
        for t in optimizer.transforms:
            if isinstance(t, Adam) and adam is None:
                adam = t
            elif isinstance(t, ClipByGlobalNorm) and clip is None and adam is None:
                clip = t.max_norm
            else:
                raise ValueError(f"unsupported optimizer chain element {t!r}")
        if adam is None:
            raise ValueError("the optimizer chain has no adam")
        return adam, (None if clip is not None and math.isinf(clip) else clip)
    raise ValueError(f"unsupported optimizer {optimizer!r}")
