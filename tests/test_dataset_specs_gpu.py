"""make_reverb_dataset's element spec and yielded data, the reference's own spec cases
(acme/datasets/reverb_test.py:85-231): simple, nested observation specs, transition
adder, batch, sequence, batch + sequence, and variable-length (zero-size) dimensions.

The reference builds the datasets and checks `dataset.element_spec.data` against the
environment spec (its _check_specs maps over both structures, so the structure must match;
the leaves' shapes and dtypes are what tf.data would report).  Here the same expected specs
are checked leaf by leaf against `element_spec.data`, and additionally against the device
tensors of a batch actually drawn from a GPU table filled with items of that layout."""

import numpy as np
import pytest
import torch

from acme_amd import replay, specs
from acme_amd.adders import reverb as adders
from acme_amd.datasets import make_reverb_dataset
from acme_amd.datasets.reverb import TensorSpec
from acme_amd.testing import fakes
from acme_amd.utils import tree

pytestmark = pytest.mark.gpu


def _continuous_spec():
    return specs.make_environment_spec(fakes.ContinuousEnvironment())


def _nested_spec():
    return specs.EnvironmentSpec(
        observations={"obs_1": specs.Array((3, 64, 64), "uint8"),
                      "obs_2": specs.Array((10,), "int32")},
        actions=specs.BoundedArray((), "float32", minimum=-1., maximum=1.),
        rewards=specs.Array((), "float32"),
        discounts=specs.BoundedArray((), "float32", minimum=0., maximum=1.))


def _step_spec(env_spec):
    return adders.Step(observation=env_spec.observations, action=env_spec.actions,
                       reward=env_spec.rewards, discount=env_spec.discounts,
                       start_of_episode=specs.Array(shape=(), dtype=bool), extras=())


def _value(rng, spec, lead=()):
    shape = tuple(lead) + tuple(spec.shape)
    dt = np.dtype(spec.dtype)
    if dt == np.bool_:
        return rng.integers(0, 2, shape).astype(bool)
    if dt.kind in "iu":
        return rng.integers(0, 100, shape).astype(dt)
    return rng.standard_normal(shape).astype(dt)


def _table(signature, n_items, make_item, seed=0):
    t = replay.Table(adders.DEFAULT_PRIORITY_TABLE, replay.selectors.Uniform(), replay.selectors.Fifo(),
                     max_size=100, rate_limiter=replay.rate_limiters.MinSize(1),
                     signature=signature)
    rng = np.random.default_rng(seed)
    for _ in range(n_items):
        t.insert(make_item(rng), 1.0)
    return replay.Server([t])


def _expected(structure, lead=()):
    leaves = tree.flatten(structure)
    return tree.unflatten_as(structure, [TensorSpec(tuple(lead) + tuple(s.shape), s.dtype)
                                         for s in leaves])


def _check(dataset, expected):
    got = dataset.element_spec.data
    # Same structure (tree.unflatten_as raises on a mismatch) and the same leaves.
    assert tree.flatten(tree.unflatten_as(expected, tree.flatten(got))) == tree.flatten(got)
    for g, e in zip(tree.flatten(got), tree.flatten(expected)):
        assert g == e, (g, e)
    # A drawn element has exactly these shapes and dtypes.
    sample = next(iter(dataset))
    torch.cuda.synchronize()
    data = sample.data
    assert len(tree.flatten(data)) == len(tree.flatten(expected))
    for x, e in zip(tree.flatten(data), tree.flatten(expected)):
        assert tuple(x.shape) == e.shape, (tuple(x.shape), e)
        assert x.dtype == torch.from_numpy(np.zeros(0, e.dtype)).dtype, (x.dtype, e)
    info = sample.info
    lead = tuple(dataset.element_spec.info.key.shape)
    for x in info:
        assert tuple(x.shape) == lead


@pytest.mark.parametrize("env", ["simple", "nested"])
def test_make_dataset_step_specs(env):
    """reverb_test.py:85-123 (test_make_dataset_simple, test_make_dataset_nested_specs)."""
    es = _continuous_spec() if env == "simple" else _nested_spec()
    sig = _step_spec(es)
    server = _table(sig, 20, lambda rng: tree.unflatten_as(
        sig, [_value(rng, s) for s in tree.flatten(sig)]))
    ds = make_reverb_dataset(server_address=server, environment_spec=es)
    _check(ds, _expected(sig))


def test_make_dataset_transition_adder():
    """reverb_test.py:125-137: tuple(environment_spec) + (observations,)."""
    es = _continuous_spec()
    sig = tuple(es) + (es.observations,)
    server = _table(adders.NStepTransitionAdder.signature(es), 20, lambda rng: tuple(
        _value(rng, s) for s in sig))
    ds = make_reverb_dataset(server_address=server, environment_spec=es, transition_adder=True)
    _check(ds, _expected(sig))


def test_make_dataset_with_batch_size():
    """reverb_test.py:139-161: every leaf gains the batch dimension."""
    es = _continuous_spec()
    sig = _step_spec(es)
    server = _table(sig, 20, lambda rng: tree.unflatten_as(
        sig, [_value(rng, s) for s in tree.flatten(sig)]))
    ds = make_reverb_dataset(server_address=server, environment_spec=es, batch_size=4)
    _check(ds, _expected(sig, (4,)))


@pytest.mark.parametrize("batch_size", [None, 4])
def test_make_dataset_with_sequence_length(batch_size):
    """reverb_test.py:163-212 (sequence, sequence + batch): [T, ...] and [B, T, ...] from a
    table of SequenceAdder-shaped T-step items."""
    T = 6
    es = _continuous_spec()
    sig = _step_spec(es)
    server = _table(sig, 20, lambda rng: tree.unflatten_as(
        sig, [_value(rng, s, (T,)) for s in tree.flatten(sig)]))
    ds = make_reverb_dataset(server_address=server, environment_spec=es, batch_size=batch_size,
                             sequence_length=T)
    _check(ds, _expected(sig, ((batch_size,) if batch_size else ()) + (T,)))


def test_make_dataset_with_variable_length_instances():
    """reverb_test.py:214-227: convert_zero_size_to_none turns zero-size dimensions into
    None (the GPU table stores fixed-shape rows, so such items are refused at insert)."""
    es = specs.EnvironmentSpec(
        observations=specs.Array((0, 64, 64), "uint8"),
        actions=specs.BoundedArray((), "float32", minimum=-1., maximum=1.),
        rewards=specs.Array((), "float32"),
        discounts=specs.BoundedArray((), "float32", minimum=0., maximum=1.))
    t = replay.Table(adders.DEFAULT_PRIORITY_TABLE, replay.selectors.Uniform(), replay.selectors.Fifo(),
                     max_size=100, rate_limiter=replay.rate_limiters.MinSize(95))
    ds = make_reverb_dataset(server_address=replay.Server([t]), environment_spec=es,
                             convert_zero_size_to_none=True)
    assert list(ds.element_spec.data[0].shape) == [None, 64, 64]
    step = adders.Step(observation=np.zeros((3, 64, 64), np.uint8), action=np.float32(0),
                       reward=np.float32(0), discount=np.float32(1),
                       start_of_episode=np.bool_(True), extras=())
    t.insert(step, 1.0)  # the first item fixes the layout ...
    with pytest.raises(ValueError, match="shape"):  # ... a different length is refused
        t.insert(step._replace(observation=np.zeros((5, 64, 64), np.uint8)), 1.0)


def test_environment_spec_mismatch_is_refused():
    es = _continuous_spec()
    sig = _step_spec(specs.make_environment_spec(fakes.ContinuousEnvironment(obs_dim=7)))
    server = _table(sig, 5, lambda rng: tree.unflatten_as(
        sig, [_value(rng, s) for s in tree.flatten(sig)]))
    with pytest.raises(ValueError, match="does not match"):
        make_reverb_dataset(server_address=server, environment_spec=es, batch_size=4)
