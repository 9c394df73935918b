"""CPU restatement of R2D2's replay-facing arithmetic (TEST INFRASTRUCTURE ONLY: imported
by tests/, never by the product path).

Follows acme/agents/tf/r2d2/learning.py:230-236 (compute_priority) and :178-183
(importance weights).  TF is absent; the float32 / float64 steps are
restated with numpy scalar semantics.  Parity unpinned at the TF boundary: no reference
test pins these values.
"""

import numpy as np


def compute_priority(errors: np.ndarray, alpha: float) -> np.ndarray:
    """errors [T, B] float32 -> float64 [B]; the mean sums over t in order."""
    a = np.abs(errors.astype(np.float32))
    T = a.shape[0]
    s = np.zeros(a.shape[1], np.float32)
    for t in range(T):
        s = (s + a[t]).astype(np.float32)
    mean = (s / np.float32(T)).astype(np.float32)
    mx = a.max(axis=0)
    p = np.float32(alpha) * mx + np.float32(1.0 - alpha) * mean
    return p.astype(np.float32).astype(np.float64)


def importance_weights(probabilities: np.ndarray, max_replay_size: int,
                       beta: float) -> np.ndarray:
    w = (1.0 / (max_replay_size * probabilities.astype(np.float64))) ** beta
    return (w / w.max()).astype(np.float32)
