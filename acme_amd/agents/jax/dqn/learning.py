"""DQNLearner — drop-in for acme/agents/jax/dqn/learning.py:54-191.

Same constructor (network, obs_spec, discount, importance_sampling_exponent,
target_update_period, iterator, optimizer, rng, max_abs_reward=1., huber_loss_parameter=1.,
replay_client=None, counter=None, logger=None) and `step()`: the whole SGD step is the same
HIP learner as the TF DQN (acme_dqn_step) run with ACME_SEMANTICS_JAX, which restates the
JAX learner's differences from the TF one:
  * importance weights `(1. / probs).astype(f32) ** beta / max`, all in f32 (:94-96);
  * params and target initialised from two different keys of `rng` (:148-151);
  * target <- params when (steps + 1) % target_update_period == 0, steps counted after the
    update (:114-119, jax/utils.py:148-154; the TF learner copies at steps % period == 0
    before counting, so at step 0);
  * optix.adam(learning_rate) (agents/jax/dqn/agent.py:110): update lr * (m_hat /
    (sqrt(v_hat) + eps)).
Priorities |td| (f64) go back as one batched update.  The reference issues one
`mutate_priorities({key: priority})` per key in order on a worker thread (:131-134, :175);
applying them in order makes the last update of a repeated key win, which is what the
batched update does (csrc/replay.hip), and the reference's asynchronous thread may land them
at any later point, of which "before the next sample" is one.  `network` is a network
descriptor of acme_amd.networks (the reference takes a Haiku function); `optimizer` an
optimizers.optix.adam descriptor; `rng` an int seed or an iterator of int seeds.
"""

from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np

from acme_amd import optimizers
from acme_amd.agents.dqn import learning as tf_learning
from acme_amd.agents.jax._rng import as_sequence
from acme_amd.utils import counting, loggers


class DQNLearner(tf_learning.DQNLearner):

    def __init__(self, network, obs_spec, discount: float, importance_sampling_exponent: float,
                 target_update_period: int, iterator, optimizer, rng,
                 max_abs_reward: float = 1., huber_loss_parameter: float = 1.,
                 replay_client=None, counter: Optional[counting.Counter] = None,
                 logger: Optional[loggers.Logger] = None, batch_size: Optional[int] = None,
                 device=None):
        adam, clip = optimizers.unpack(optimizer)
        if clip is not None:
            raise ValueError("the JAX DQN learner takes optix.adam (agents/jax/dqn/agent.py:110)")
        shape = tuple(getattr(obs_spec, "shape", network.obs_shape))
        if shape != tuple(network.obs_shape):
            raise ValueError(f"obs_spec shape {shape} does not match the network's "
                             f"{tuple(network.obs_shape)}")
        seeds = as_sequence(rng)
        params_seed, target_seed = next(seeds), next(seeds)
        B = batch_size or getattr(iterator, "batch_size", None)
        super().__init__(network, network, discount=discount,
                         importance_sampling_exponent=importance_sampling_exponent,
                         learning_rate=adam.learning_rate,
                         target_update_period=target_update_period, dataset=iterator,
                         huber_loss_parameter=huber_loss_parameter, replay_client=replay_client,
                         counter=counter, logger=logger, checkpoint=False,
                         max_abs_reward=max_abs_reward, batch_size=B, seed=params_seed,
                         target_seed=target_seed, device=device, semantics="jax", adam=adam)
        self._log_loss = False  # the JAX learner logs counts only (:178)

    def get_variables(self, names: List[str]) -> List[Dict[str, np.ndarray]]:
        # As the JAX learner: [params] (the Haiku params tree), names ignored (:180-181).
        return [self._native.get_params("params")]
