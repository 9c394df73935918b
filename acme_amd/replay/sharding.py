"""Global-probability sampling over per-rank replay shards.

Data-parallel DQN (BASELINE configs[4]): one process per GPU, each holding a 1/N shard of
the replay (its own sum tree), one learner replica per GPU, gradients all-reduced.  A single
table of the whole replay would draw the global batch of N * B items with P(i) =
p_i^alpha / S (agents/tf/dqn/agent.py:95-101; Reverb Prioritized).  Here the global draw is
stratified by shard: the ranks exchange their shard masses S_r (one f64 each, an all-reduce of
an N-vector), every rank computes the same allocation n_r of the N * B draws in proportion to
S_r / S (largest remainder), and draws its n_r from its own shard.  An item of shard r is then
drawn with marginal probability (n_r / (N B)) * p_i^alpha / S_r, which is p_i^alpha / S when
the shares are proportional; that exact marginal is what the sampler reports
(acme_replay_sample_share), so the learners' importance weights are those of the draw that
happened.  No item data crosses GPUs.

The shares of draw k come from the masses snapshotted after draw k - LAG was issued (the
snapshot is copied to pinned host memory asynchronously), so the host learns n_r without a
device synchronisation; every rank uses the same snapshot, so all ranks agree on the shares.
Draws before the first snapshot split the batch equally (probability scaled by 1 / N).
"""

from __future__ import annotations

import math
from typing import List, Optional, Sequence

LAG = 2  # draws between a mass snapshot and the draw whose shares it sets


def allocate_shares(totals: Sequence[float], global_batch: int,
                    cap: Optional[int] = None) -> List[int]:
    """Largest-remainder allocation of `global_batch` draws in proportion to `totals`.

    Every shard with positive mass gets at least one draw and at most `cap`; ties in the
    remainders go to the lower rank.  Deterministic: identical inputs give identical shares
    on every rank."""
    n = len(totals)
    if n == 0 or global_batch < 0:
        raise ValueError("need at least one shard and a non-negative batch")
    tot = [float(t) for t in totals]
    if any(not (t >= 0.0) or math.isinf(t) for t in tot):
        raise ValueError(f"shard masses must be finite and >= 0, got {tot}")
    live = [i for i in range(n) if tot[i] > 0.0]
    if not live:
        raise RuntimeError("every replay shard is empty (rate limiter MinSize(1))")
    cap = global_batch if cap is None else int(cap)
    if cap * len(live) < global_batch:
        raise ValueError(f"{global_batch} draws do not fit {len(live)} shards of at most {cap}")
    S = math.fsum(tot[i] for i in live)
    quota = [global_batch * tot[i] / S if tot[i] > 0.0 else 0.0 for i in range(n)]
    share = [int(math.floor(q)) for q in quota]
    left = global_batch - sum(share)
    order = sorted(live, key=lambda i: (-(quota[i] - share[i]), i))
    for i in order[:left]:
        share[i] += 1
    # At least one draw per live shard (taken from the largest shares), at most `cap`.
    for i in live:
        while share[i] < 1:
            j = max(live, key=lambda k: (share[k], -k))
            share[j] -= 1
            share[i] += 1
    over = sum(max(0, share[i] - cap) for i in live)
    for i in live:
        share[i] = min(share[i], cap)
    while over > 0:
        for i in sorted(live, key=lambda k: (share[k], k)):
            if over == 0:
                break
            if share[i] < cap:
                share[i] += 1
                over -= 1
    assert sum(share) == global_batch
    return share
