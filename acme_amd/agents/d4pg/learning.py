"""D4PGLearner — drop-in for acme/agents/tf/d4pg/learning.py:35-270.

Same constructor arguments and `step()` contract: one call draws a batch from the
dataset iterator and runs the whole D4PG step on the GPU (acme_d4pg_step: start-of-step
target copy, target/online policy and critic forwards, categorical L2-projection loss,
dpg loss with dqda norm clipping, per-network global-norm clipping, two Adams), then
counts and logs.  Losses are device scalars handed to the logger; nothing synchronises
the host with the device.

`policy_network` / `critic_network` are descriptors from acme_amd.networks
(LayerNormMLPPolicy, DistributionalCritic); the observation networks must be the
identity (the reference's control-suite setup, examples/control_suite/run_d4pg.py:66).
Optimizers are anything with a `learning_rate` (acme_amd.optimizers.Adam); the default is
Adam(1e-4) for both (learning.py:113-114).
"""

from __future__ import annotations

import time
from typing import Dict, List, Optional

import numpy as np
import torch

from acme_amd import core
from acme_amd.native import NativeD4PG
from acme_amd.utils import counting, loggers


def _is_identity(fn) -> bool:
    if fn is None or fn == "identity":
        return True
    try:
        x = np.arange(3.0)
        return fn(x) is x
    except Exception:
        return False


class D4PGLearner(core.Learner, core.Saveable):

    def __init__(self, policy_network, critic_network, target_policy_network,
                 target_critic_network, discount: float, target_update_period: int, dataset,
                 observation_network=lambda x: x, target_observation_network=lambda x: x,
                 policy_optimizer=None, critic_optimizer=None, clipping: bool = True,
                 counter: Optional[counting.Counter] = None,
                 logger: Optional[loggers.Logger] = None, checkpoint: bool = True,
                 batch_size: Optional[int] = None, seed: int = 0, device=None):
        if not (_is_identity(observation_network) and _is_identity(target_observation_network)):
            raise ValueError("acme_amd's D4PG learner supports identity observation networks "
                             "(flat observations) only")
        if critic_network.obs_dim != policy_network.obs_dim or \
                critic_network.act_dim != policy_network.act_dim:
            raise ValueError("policy and critic disagree on observation / action sizes")
        self._policy_network = policy_network
        self._critic_network = critic_network
        self._iterator = iter(dataset)
        B = batch_size or getattr(dataset, "batch_size", None) or 256
        lr = lambda opt: float(getattr(opt, "learning_rate", 1e-4)) if opt is not None else 1e-4  # noqa
        self._native = NativeD4PG(
            obs_dim=policy_network.obs_dim, act_dim=policy_network.act_dim, max_batch=B,
            policy_sizes=policy_network.layer_sizes, critic_sizes=critic_network.layer_sizes,
            num_atoms=critic_network.num_atoms, vmin=critic_network.vmin,
            vmax=critic_network.vmax, action_min=policy_network.action_min,
            action_max=policy_network.action_max, discount=discount,
            target_update_period=target_update_period,
            policy_learning_rate=lr(policy_optimizer), critic_learning_rate=lr(critic_optimizer),
            clipping=clipping, device=device)
        init = dict(policy_network.init(seed))
        init.update(critic_network.init(seed + 1))
        tinit = dict(target_policy_network.init(seed + 2))
        tinit.update(target_critic_network.init(seed + 3))
        self._native.set_params(init, tinit)
        self._counter = counter or counting.Counter()
        self._logger = logger or loggers.TerminalLogger("learner", time_delta=1.0)
        self._timestamp = None
        self._checkpoint = checkpoint

    def step(self):
        sample = next(self._iterator)
        o_tm1, a_tm1, r_t, d_t, o_t = sample.data[:5]
        B = int(r_t.shape[0])
        f = lambda x: x.reshape(B, -1).to(torch.float32).contiguous()  # noqa: E731
        self._native.step(f(o_tm1), f(a_tm1), f(r_t).reshape(B), f(d_t).reshape(B), f(o_t))
        now = time.time()
        elapsed = now - self._timestamp if self._timestamp else 0
        self._timestamp = now
        result = {"critic_loss": self._native.critic_loss, "policy_loss": self._native.policy_loss}
        result.update(self._counter.increment(steps=1, walltime=elapsed))
        self._logger.write(result)

    def policy(self, observations, use_target: bool = False) -> np.ndarray:
        x = torch.as_tensor(np.asarray(observations, np.float32))
        return self._native.policy(x, use_target).cpu().numpy()

    def get_variables(self, names: List[str]) -> List[Dict[str, np.ndarray]]:
        # As the TF learner (learning.py:117-122, 269-270): 'critic' -> target critic,
        # 'policy' -> target (observation + policy) network; host copies.
        target = self._native.get_params("target")
        out = []
        for name in names:
            if name not in ("critic", "policy"):
                raise KeyError(name)
            out.append({k: v for k, v in target.items() if k.startswith(name + "/")})
        return out

    @property
    def native(self) -> NativeD4PG:
        return self._native

    @property
    def num_steps(self) -> int:
        return self._native.num_steps

    @property
    def state(self) -> Dict:
        return self.save()

    def save(self) -> Dict:
        n = self._native
        return {"params": n.get_params("params"), "target": n.get_params("target"),
                "optimizer": {"m": n.get_params("m"), "v": n.get_params("v")},
                "num_steps": n.num_steps}

    def restore(self, state: Dict):
        n = self._native
        n.set_params(state["params"], state["target"])
        for buf, src in ((n.m, state["optimizer"]["m"]), (n.v, state["optimizer"]["v"])):
            for k, t in n.views(buf).items():
                t.copy_(torch.as_tensor(np.asarray(src[k], np.float32)).view(t.shape))
        n.num_steps = int(state["num_steps"])
