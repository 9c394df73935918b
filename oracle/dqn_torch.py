"""ORACLE — test infrastructure only (tests/ and bench.py's cpu_baseline leg).  Never
imported by the product package acme_amd.

float32 torch-CPU restatement of the TF DQN learner step, DQNLearner._step
(acme/agents/tf/dqn/learning.py:112-168), the CPU baseline SURVEY §8(d) names ("the
build's own float32 torch-CPU restatement of the TF _step, timed on the GPU box's host
cores").  Same math as oracle/dqn_oracle.py, written with torch.nn.functional and autograd:

  q_tm1 = net(o_tm1); q_t_value = target(o_t); q_t_selector = net(o_t)      :123-125
  r = clip(r, -1, 1); d = d * discount                                     :128-130
  trfl.double_qlearning (first-max argmax, target stop-gradient)           :133-134
  losses.huber(td, 1) with gradient clip(td) (acme/tf/losses/huber.py:45-57):135
  w = (1/p)^beta / max(w) in float64, cast to float32 at the multiply       :138-143
  loss = mean(w * huber); autograd; snt.Adam(1e-3)                         :144-148
  priorities = |td| (f64); target <- online after the update every 100     :151-161

DQNAtariNetwork (acme/tf/networks/atari.py:36-69, duelling.py:40-59) with Sonnet's SAME
padding done explicitly (pad_top = total // 2) on NCHW tensors; the parameters use the
product layout (HWIO convolutions, fused [7744, 1024] hidden layer, NHWC flatten order).
"""

from __future__ import annotations

from typing import Dict

import numpy as np
import torch
import torch.nn.functional as F

from oracle.dqn_oracle import nature_tensor_shapes, same_pads

CONVS = (("atari_torso/conv2_d", 8, 4), ("atari_torso/conv2_d_1", 4, 2),
         ("atari_torso/conv2_d_2", 3, 1))


def huber(x: torch.Tensor, delta: float = 1.0) -> torch.Tensor:
    """acme/tf/losses/huber.py:45-57: the 'lin' form, so d/dx = clip(x, -delta, delta)."""
    ax = x.abs()
    quad = torch.clamp(ax, max=delta)
    lin = ax - quad
    return 0.5 * quad * quad + delta * lin


class TorchDQN:
    """Nature-CNN DQN learner state (params, target, Adam m / v, num_steps) as float32
    torch tensors on the CPU (dtype / device: e.g. a float64 reference trajectory on the
    GPU for the plane engine's long-horizon test)."""

    def __init__(self, params: Dict[str, np.ndarray], num_actions: int, lr: float = 1e-3,
                 discount: float = 0.99, beta: float = 0.2, period: int = 100,
                 target: Dict[str, np.ndarray] = None, dtype=torch.float32, device="cpu"):
        self.A = num_actions
        self.dtype, self.device = dtype, torch.device(device)
        self.names = [n for n, _ in nature_tensor_shapes(num_actions)]
        self.p = {k: torch.tensor(np.asarray(params[k], np.float32), dtype=dtype,
                                  device=self.device, requires_grad=True)
                  for k in self.names}
        self.t = {k: v.detach().clone() for k, v in self.p.items()}
        if target is not None:
            for k in self.names:
                self.t[k].copy_(torch.as_tensor(np.asarray(target[k], np.float32)))
        self.m = {k: torch.zeros_like(v) for k, v in self.t.items()}
        self.v = {k: torch.zeros_like(v) for k, v in self.t.items()}
        self.lr, self.discount, self.beta, self.period = lr, discount, beta, period
        self.num_steps = 0

    def q(self, p, obs_u8: torch.Tensor) -> torch.Tensor:
        x = (obs_u8.to(self.device, self.dtype) / 255.0).permute(0, 3, 1, 2)  # NHWC -> NCHW
        for name, k, s in CONVS:
            H = x.shape[-1]
            out, pt, pb = same_pads(H, k, s)
            x = F.pad(x, (pt, pb, pt, pb))
            w = p[f"{name}/w"].permute(3, 2, 0, 1)  # HWIO -> OIHW
            x = F.relu(F.conv2d(x, w, p[f"{name}/b"], stride=s))
        x = x.permute(0, 2, 3, 1).reshape(x.shape[0], -1)  # NHWC flatten
        h = F.relu(x @ p["duelling_q_network/hidden/w"] + p["duelling_q_network/hidden/b"])
        v = h[:, :512] @ p["duelling_q_network/mlp/linear_1/w"] + \
            p["duelling_q_network/mlp/linear_1/b"]
        adv = h[:, 512:] @ p["duelling_q_network/mlp_1/linear_1/w"] + \
            p["duelling_q_network/mlp_1/linear_1/b"]
        return v + adv - adv.mean(dim=1, keepdim=True)

    def step(self, o_tm1, a_tm1, r_t, d_t, o_t, probs: np.ndarray):
        q_tm1 = self.q(self.p, o_tm1)
        with torch.no_grad():
            q_t_value = self.q(self.t, o_t)
            q_t_selector = self.q(self.p, o_t)
        r = torch.clamp(r_t, -1.0, 1.0)
        d = d_t * self.discount
        best = q_t_selector.argmax(dim=1)  # first max, as tf.argmax
        target = r + d * q_t_value.gather(1, best[:, None])[:, 0]
        td = target - q_tm1.gather(1, a_tm1.long()[:, None])[:, 0]
        iw = (1.0 / probs) ** self.beta
        w = torch.from_numpy((iw / iw.max()).astype(np.float32)).to(self.device, self.dtype)
        loss = (w * huber(td)).mean()
        grads = torch.autograd.grad(loss, [self.p[k] for k in self.names])
        t = self.num_steps + 1
        b1, b2, eps = 0.9, 0.999, 1e-8
        bc1, bc2 = 1.0 - b1 ** t, 1.0 - b2 ** t
        with torch.no_grad():
            for k, g in zip(self.names, grads):
                self.m[k].mul_(b1).add_(g, alpha=1.0 - b1)
                self.v[k].mul_(b2).addcmul_(g, g, value=1.0 - b2)
                self.p[k].sub_(self.lr * (self.m[k] / bc1) / ((self.v[k] / bc2).sqrt() + eps))
            if self.num_steps % self.period == 0:
                for k in self.names:
                    self.t[k].copy_(self.p[k])
        self.num_steps += 1
        return float(loss.detach()), td.detach().abs().double().cpu().numpy()
