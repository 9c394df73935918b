"""Prefetching dataset vs concurrent writers (datasets/reverb.py): priority
updates and inserts queued right after next() with no host synchronisation must not race
the draws issued ahead on the dataset's stream.  Every draw is checked bit-exactly against
the C sum-tree oracle replaying the same writes in stream order: draw j is issued at
iteration j - P, after the writes of iterations < j - P."""

import numpy as np
import pytest
import torch

from acme_amd import replay, specs
from acme_amd.adders import reverb as adders
from acme_amd.datasets import make_reverb_dataset

pytestmark = pytest.mark.gpu

CAP, B, P, ITERS, NEW = 4096, 64, 3, 10, 5


def test_prefetched_draws_ordered_after_writes():
    from tests._oracle import OracleTable
    spec = specs.EnvironmentSpec(observations=specs.Array((8,), np.float32),
                                 actions=specs.BoundedArray((2,), np.float32, -1.0, 1.0),
                                 rewards=specs.Array((), np.float32),
                                 discounts=specs.BoundedArray((), np.float32, 0.0, 1.0))
    table = replay.Table(adders.DEFAULT_PRIORITY_TABLE, replay.selectors.Prioritized(0.6),
                         replay.selectors.Fifo(), CAP, replay.rate_limiters.MinSize(1),
                         signature=adders.NStepTransitionAdder.signature(spec), seed=21)
    table.native.fill_synthetic(CAP, layout=1, num_actions=1, seed=0)
    mirror = OracleTable(CAP, True, 0.6, 21)
    mirror.insert(np.ones(CAP))
    it = iter(make_reverb_dataset(replay.Server([table]), batch_size=B, prefetch_size=P))
    rng = np.random.default_rng(0)
    writes = []          # (iteration, keys, priorities, new-item priorities)
    inserted = {}        # key -> observation of items this test inserted
    next_key = CAP
    for i in range(ITERS):
        s = next(it)
        # Writes queued immediately, no synchronisation with the dataset's stream.
        keys = s.info.key
        pr = torch.as_tensor(rng.uniform(0.0, 5.0, B), device="cuda")
        table.update_priorities(keys, pr)
        new_pr = rng.uniform(0.5, 2.0, NEW)
        for j in range(NEW):
            o = np.full(8, next_key, np.float32)
            table.insert((o, np.zeros(2, np.float32), np.float32(1), np.float32(1), o),
                         float(new_pr[j]))
            inserted[next_key] = o
            next_key += 1
        table.flush()
        # Host copies (synchronising) only after the writes were queued.
        info_keys = keys.view(torch.int64).cpu().numpy().view(np.uint64)
        probs = s.info.probability.cpu().numpy()
        sizes = s.info.table_size.cpu().numpy()
        obs = s.data[0].cpu().numpy()
        writes.append((i, info_keys, pr.cpu().numpy(), new_pr))
        # Mirror: the writes of iterations < i - P precede draw i.
        while writes and writes[0][0] < i - P:
            _, wk, wp, wn = writes.pop(0)
            mirror.update(wk, wp)
            mirror.insert(wn)
        ref = mirror.sample(B, i)
        np.testing.assert_array_equal(info_keys, ref["keys"], err_msg=f"iteration {i}")
        np.testing.assert_array_equal(probs, ref["probabilities"], err_msg=f"iteration {i}")
        np.testing.assert_array_equal(sizes, ref["table_size"], err_msg=f"iteration {i}")
        for r, k in enumerate(info_keys):
            if int(k) in inserted:
                np.testing.assert_array_equal(obs[r], inserted[int(k)])
