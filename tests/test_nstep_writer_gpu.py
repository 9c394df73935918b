"""NStepTransitionAdder's native path (csrc/replay.hip acme_nstep_writer): the adder hands
each environment step to the GPU table's n-step writer, which forms the items in C straight
into pinned staging rows (acme/adders/reverb/transition.py:119-172).

Checked bit-exactly:
  * the rows the native path leaves in the table equal the items the Python adder writes
    (the same adder class driven through a FakeClient, which the reference's golden adder
    cases pin: tests/test_adders_cpu.py), in the same key order, padding bytes zero;
  * a second table filled with those items through acme_replay_stage / commit holds the
    same bytes, keys, priorities and sum-tree leaves, and draws the same samples;
  * an episode whose step stops fitting the native path (a float64 reward) finishes on
    the Python path with the same items;
  * pending rows count towards Table.size() and a reader's flush commits them only when the
    device table could not serve the draw otherwise.
"""

import numpy as np
import pytest
import torch

from acme_amd import dm_env, replay, specs
from acme_amd.adders import reverb as adders
from acme_amd.testing import fakes

pytestmark = pytest.mark.gpu

LAYOUTS = {
    # Atari-like: u8 frames (90 B payload in a 92 B row) and a discrete action.
    "u8_discrete": (specs.Array((6, 5, 3), np.uint8), specs.DiscreteArray(18, np.int32)),
    # Control: f32 observation and a 2-vector action.
    "f32_vector": (specs.Array((7,), np.float32),
                   specs.BoundedArray((2,), np.float32, -1.0, 1.0)),
}


def _env_spec(layout):
    obs, act = LAYOUTS[layout]
    return specs.EnvironmentSpec(observations=obs, actions=act,
                                 rewards=specs.Array((), np.float32),
                                 discounts=specs.BoundedArray((), np.float32, 0.0, 1.0))


def _episodes(layout, lengths, seed, f64_reward_at=None):
    """[(first timestep, [(action, timestep), ...]), ...] with float32 rewards/discounts
    (discount 0 at a termination, some mid-episode discounts below 1)."""
    obs_spec, act_spec = LAYOUTS[layout]
    rng = np.random.default_rng(seed)

    def obs():
        if obs_spec.dtype == np.uint8:
            return rng.integers(0, 256, obs_spec.shape).astype(np.uint8)
        return rng.standard_normal(obs_spec.shape).astype(np.float32)

    def act():
        if isinstance(act_spec, specs.DiscreteArray):
            return np.int32(rng.integers(0, act_spec.num_values))
        return rng.uniform(-1, 1, act_spec.shape).astype(np.float32)

    eps = []
    for e, T in enumerate(lengths):
        steps = []
        for t in range(T):
            r = np.float32(rng.standard_normal())
            if rng.uniform() < 0.25:
                r = float(r) / 3.0  # a Python float reward (weak scalar: f32 arithmetic)
            if f64_reward_at is not None and (e, t) == f64_reward_at:
                r = np.float64(r) + 1e-9
            if t == T - 1:
                ts = (dm_env.termination(r, obs()) if e % 2 == 0
                      else dm_env.truncation(r, obs(), np.float32(0.9)))
            else:
                d = np.float32(1.0 if rng.uniform() < 0.7 else rng.uniform(0.5, 1.0))
                ts = dm_env.transition(r, obs(), d)
            steps.append((act(), ts))
        eps.append((dm_env.restart(obs()), steps))
    return eps


def _run(adder, episodes):
    for first, steps in episodes:
        adder.add_first(first)
        for a, ts in steps:
            adder.add(a, ts)


def _python_items(n_step, discount, episodes):
    client = fakes.FakeClient()
    _run(adders.NStepTransitionAdder(client, n_step=n_step, discount=discount), episodes)
    return [item for w in client.writers for (_, item, _) in w.priorities]


def _rows(items, fields):
    """Packed row bytes per field of each item, as the table stores them (zero padding)."""
    out = []
    for f in fields:
        rows = np.zeros((len(items), f.row_bytes), np.uint8)
        out.append(rows)
    for i, item in enumerate(items):
        for leaf, f, rows in zip(item, fields, out):
            a = np.ascontiguousarray(np.asarray(leaf, f.dtype))
            rows[i, :f.nbytes] = a.reshape(-1).view(np.uint8)
    return out


def _table(layout, cap=4096):
    return replay.Table(adders.DEFAULT_PRIORITY_TABLE, replay.selectors.Prioritized(0.6),
                        replay.selectors.Fifo(), cap, replay.rate_limiters.MinSize(1),
                        signature=adders.NStepTransitionAdder.signature(_env_spec(layout)),
                        seed=7, device=torch.device("cuda"))


@pytest.mark.parametrize("layout", sorted(LAYOUTS))
@pytest.mark.parametrize("n_step", [1, 3, 5])
def test_native_rows_equal_python_items_and_stage_commit_rows(layout, n_step):
    discount = 0.97
    episodes = _episodes(layout, [1, 2, n_step, 3 * n_step + 4, 40], seed=n_step)
    want = _python_items(n_step, discount, episodes)

    table = _table(layout)
    adder = adders.NStepTransitionAdder(replay.Client(replay.Server([table])), n_step=n_step,
                                        discount=discount, rows_per_chunk=5)
    _run(adder, episodes)
    assert adder._fast, "the GPU table's native writer was not used"  # noqa: SLF001
    assert table._fill == 0  # noqa: SLF001  (nothing went through the Python rows)
    table.flush()
    got = table.native.export_state()
    expect = _rows(want, table.fields)
    assert int(got["inserted"]) == len(want)
    np.testing.assert_array_equal(got["keys"], np.arange(len(want), dtype=np.uint64))
    for f in range(5):
        np.testing.assert_array_equal(got[f"field_{f}"], expect[f], err_msg=f"field {f}")
    np.testing.assert_array_equal(got["raw_priorities"], np.ones(len(want)))

    # The same items through acme_replay_stage / commit: identical table.
    ref = _table(layout)
    nat = ref.native
    chunk = nat.stage_capacity()
    for s in range(0, len(want), chunk):
        m = min(chunk, len(want) - s)
        bufs = nat.stage(m)
        for b, e in zip(bufs, expect):
            b[:] = e[s:s + m]
        nat.commit(m, np.ones(m))
    other = nat.export_state()
    for k in got:
        np.testing.assert_array_equal(got[k], other[k], err_msg=k)
    np.testing.assert_array_equal(table.native.debug_state()["leaves"],
                                  nat.debug_state()["leaves"])
    a = table.native.sample(64, 3)
    b = nat.sample(64, 3)
    for k in a:
        np.testing.assert_array_equal(a[k].cpu().numpy(), b[k].cpu().numpy(), err_msg=k)


def test_step_that_does_not_fit_falls_back_to_python():
    layout, n_step = "u8_discrete", 3
    episodes = _episodes(layout, [9, 12, 7], seed=11, f64_reward_at=(1, 5))
    want = _python_items(n_step, 0.99, episodes)
    table = _table(layout)
    adder = adders.NStepTransitionAdder(replay.Client(replay.Server([table])), n_step=n_step,
                                        discount=0.99, rows_per_chunk=4)
    _run(adder, episodes)
    table.flush()
    got = table.native.export_state()
    expect = _rows(want, table.fields)
    assert int(got["inserted"]) == len(want)
    for f in range(5):
        np.testing.assert_array_equal(got[f"field_{f}"], expect[f], err_msg=f"field {f}")


def test_pending_rows_count_and_reader_flush():
    layout = "f32_vector"
    table = _table(layout)
    adder = adders.NStepTransitionAdder(replay.Client(replay.Server([table])), n_step=2,
                                        discount=0.9, rows_per_chunk=64)
    (first, steps), = _episodes(layout, [30], seed=3)
    adder.add_first(first)
    for a, ts in steps[:10]:
        adder.add(a, ts)
    assert table.committed_size() == 0 and table.size() == 10
    table.flush_for_sampling(4)  # the device table cannot serve a draw: commit
    assert table.committed_size() == 10
    for a, ts in steps[10:20]:
        adder.add(a, ts)
    table.flush_for_sampling(4)  # it can: the writer keeps its rows
    assert table.committed_size() == 10 and table.size() == 20
    for a, ts in steps[20:]:
        adder.add(a, ts)  # the last step drains the window and the reset commits it
    assert table.committed_size() == table.size() == 30 + 1
