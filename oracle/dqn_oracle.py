"""ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py's
cpu_baseline leg).  Never imported by the product package acme_amd.

numpy restatement of the TF DQN learner step, DQNLearner._step
(acme/agents/tf/dqn/learning.py:112-168), in float64 ("f64", the accuracy reference) or
float32 ("f32", the CPU baseline arithmetic):

  q_tm1 = net(o_tm1); q_t_value = target(o_t); q_t_selector = net(o_t)      :123-125
  r = clip(r, -1, 1); d = d * discount                                     :128-130
  trfl.double_qlearning: a* = argmax q_t_selector (first max),
      td = r + d * q_t_value[a*] - q_tm1[a]  (target stop-gradient)         :133-134
  losses.huber(td, delta)  (acme/tf/losses/huber.py:45-57, grad = clip(td))  :135
  w = (1/p)^beta / max(w) in float64, cast to f32 at the multiply            :138-143
  loss = mean(w * huber)                                                     :144
  grads, snt.Adam(lr)                                                        :147-148
  priorities = |td| (f64)                                                    :151-154
  if num_steps % period == 0: target <- online (AFTER the update)            :157-161

Networks: DQNAtariNetwork (acme/tf/networks/atari.py:36-69 — Conv2D(32,8,4), ReLU,
Conv2D(64,4,2), ReLU, Conv2D(64,3,1), ReLU, Flatten, DuellingMLP([512]) —
acme/tf/networks/duelling.py:40-59: q = v + (adv - mean(adv))), with Sonnet's default
SAME padding / NHWC layout; snt.nets.MLP([..., A]) (examples/bsuite/run_dqn.py:46-49).

Third-party semantics restated here (not in /root/reference; parity for them is
UNPINNED — no reference test holds a learner golden value):
  trfl.double_qlearning (tf.argmax first-max tie-break, batched_index), Sonnet Conv2D
  SAME padding (pad_top = total // 2), Sonnet Adam (Kingma & Ba Algorithm 1 with
  epsilon added to sqrt(v_hat), step incremented before the update).
Parameter layout: the same tensors as the product learner (fused duelling hidden layer
[7744, 1024] = [value | advantage]); see DESIGN.md §4.
"""

from __future__ import annotations

import dataclasses
from typing import Dict, List, Optional, Tuple

import numpy as np

# ------------------------------------------------------------------ network spec


def nature_tensor_shapes(num_actions: int) -> List[Tuple[str, Tuple[int, ...]]]:
    return [
        ("atari_torso/conv2_d/w", (8, 8, 4, 32)),
        ("atari_torso/conv2_d/b", (32,)),
        ("atari_torso/conv2_d_1/w", (4, 4, 32, 64)),
        ("atari_torso/conv2_d_1/b", (64,)),
        ("atari_torso/conv2_d_2/w", (3, 3, 64, 64)),
        ("atari_torso/conv2_d_2/b", (64,)),
        ("duelling_q_network/hidden/w", (7744, 1024)),
        ("duelling_q_network/hidden/b", (1024,)),
        ("duelling_q_network/mlp/linear_1/w", (512, 1)),
        ("duelling_q_network/mlp/linear_1/b", (1,)),
        ("duelling_q_network/mlp_1/linear_1/w", (512, num_actions)),
        ("duelling_q_network/mlp_1/linear_1/b", (num_actions,)),
    ]


def mlp_tensor_shapes(obs_dim: int, hidden: List[int], num_actions: int):
    out, d = [], obs_dim
    for i, h in enumerate(list(hidden) + [num_actions]):
        out.append((f"mlp/linear_{i}/w", (d, h)))
        out.append((f"mlp/linear_{i}/b", (h,)))
        d = h
    return out


CONVS = [  # (name, stride, (pad_top, pad_left, pad_bottom, pad_right)) — TF SAME
    ("atari_torso/conv2_d", 4, (2, 2, 2, 2)),
    ("atari_torso/conv2_d_1", 2, (1, 1, 2, 2)),
    ("atari_torso/conv2_d_2", 1, (1, 1, 1, 1)),
]


def same_pads(n: int, k: int, s: int) -> Tuple[int, int, int]:
    out = -(-n // s)
    total = max((out - 1) * s + k - n, 0)
    return out, total // 2, total - total // 2


# ------------------------------------------------------------------ conv via im2col


def _im2col(x: np.ndarray, kh: int, kw: int, s: int, pads) -> Tuple[np.ndarray, Tuple]:
    pt, pl, pb, pr = pads
    b, h, w, c = x.shape
    xp = np.pad(x, ((0, 0), (pt, pb), (pl, pr), (0, 0)))
    oh = (h + pt + pb - kh) // s + 1
    ow = (w + pl + pr - kw) // s + 1
    st = xp.strides
    cols = np.lib.stride_tricks.as_strided(
        xp, shape=(b, oh, ow, kh, kw, c),
        strides=(st[0], st[1] * s, st[2] * s, st[1], st[2], st[3]), writeable=False)
    return cols.reshape(b * oh * ow, kh * kw * c), (b, oh, ow, xp.shape)


def _col2im(dcols: np.ndarray, meta, kh, kw, s, pads, x_shape) -> np.ndarray:
    b, oh, ow, xp_shape = meta
    pt, pl, pb, pr = pads
    c = x_shape[3]
    dxp = np.zeros(xp_shape, dtype=dcols.dtype)
    d6 = dcols.reshape(b, oh, ow, kh, kw, c)
    for i in range(kh):
        for j in range(kw):
            dxp[:, i:i + s * oh:s, j:j + s * ow:s, :] += d6[:, :, :, i, j, :]
    return dxp[:, pt:pt + x_shape[1], pl:pl + x_shape[2], :]


def conv_forward(x, w, b, s, pads):
    kh, kw, ci, co = w.shape
    cols, meta = _im2col(x, kh, kw, s, pads)
    y = cols @ w.reshape(kh * kw * ci, co) + b
    return y.reshape(meta[0], meta[1], meta[2], co), (cols, meta)


# ------------------------------------------------------------------ forward/backward


def obs_to_float(o: np.ndarray, dtype) -> np.ndarray:
    """AtariWrapper(to_float=True) + SinglePrecisionWrapper: float32(uint8 / 255.0)."""
    if o.dtype == np.uint8:
        return (o / 255.0).astype(np.float32).astype(dtype)
    return o.astype(dtype)


def nature_forward(params: Dict[str, np.ndarray], o: np.ndarray, dtype):
    x = obs_to_float(o, dtype)
    cache = {"x0": x}
    for li, (name, s, pads) in enumerate(CONVS):
        z, (cols, meta) = conv_forward(x, params[name + "/w"].astype(dtype),
                                       params[name + "/b"].astype(dtype), s, pads)
        x = np.maximum(z, 0)
        cache[f"cols{li}"] = (cols, meta)
        cache[f"x{li + 1}"] = x
    flat = x.reshape(x.shape[0], -1)
    hz = flat @ params["duelling_q_network/hidden/w"].astype(dtype) + \
        params["duelling_q_network/hidden/b"].astype(dtype)
    h = np.maximum(hz, 0)
    hv, ha = h[:, :512], h[:, 512:]
    v = hv @ params["duelling_q_network/mlp/linear_1/w"].astype(dtype) + \
        params["duelling_q_network/mlp/linear_1/b"].astype(dtype)
    adv = ha @ params["duelling_q_network/mlp_1/linear_1/w"].astype(dtype) + \
        params["duelling_q_network/mlp_1/linear_1/b"].astype(dtype)
    adv = adv - adv.mean(axis=-1, keepdims=True)
    q = v + adv
    cache.update(flat=flat, h=h)
    return q, cache


def nature_backward(params, cache, dq, dtype, masks=None) -> Dict[str, np.ndarray]:
    """Backward pass.  `masks` (optional) overrides the ReLU branch decisions (x > 0) of
    the named activations ("hid", "x3", "x2", "x1") — used by the parity tests to check
    the backward pass conditional on the kernel's own ReLU pattern, since fp32 and fp64
    legitimately disagree for pre-activations within rounding of 0."""
    masks = masks or {}
    mask = lambda key, x: masks[key] if key in masks else (x > 0)  # noqa: E731
    g = {}
    h = cache["h"]
    hv, ha = h[:, :512], h[:, 512:]
    dv = dq.sum(axis=1, keepdims=True)
    dadv = dq - dq.mean(axis=1, keepdims=True)
    wv = params["duelling_q_network/mlp/linear_1/w"].astype(dtype)
    wa = params["duelling_q_network/mlp_1/linear_1/w"].astype(dtype)
    g["duelling_q_network/mlp/linear_1/w"] = hv.T @ dv
    g["duelling_q_network/mlp/linear_1/b"] = dv.sum(0)
    g["duelling_q_network/mlp_1/linear_1/w"] = ha.T @ dadv
    g["duelling_q_network/mlp_1/linear_1/b"] = dadv.sum(0)
    dh = np.concatenate([dv @ wv.T, dadv @ wa.T], axis=1) * mask("hid", h)
    cache["dzh"] = dh
    g["duelling_q_network/hidden/w"] = cache["flat"].T @ dh
    g["duelling_q_network/hidden/b"] = dh.sum(0)
    dflat = dh @ params["duelling_q_network/hidden/w"].astype(dtype).T
    dx = dflat.reshape(cache["x3"].shape) * mask("x3", cache["x3"])
    cache["dz3"] = dx
    for li in (2, 1, 0):
        name, s, pads = CONVS[li]
        w = params[name + "/w"].astype(dtype)
        kh, kw, ci, co = w.shape
        cols, meta = cache[f"cols{li}"]
        dz = dx.reshape(-1, co)
        g[name + "/w"] = (cols.T @ dz).reshape(w.shape)
        g[name + "/b"] = dz.sum(0)
        if li > 0:
            dcols = dz @ w.reshape(-1, co).T
            xin = cache[f"x{li}"]
            dx = _col2im(dcols, meta, kh, kw, s, pads, xin.shape) * mask(f"x{li}", xin)
            cache[f"dz{li}"] = dx
    return g


def mlp_forward(params, o, dtype, n_layers):
    x = obs_to_float(o, dtype).reshape(o.shape[0], -1)
    acts = [x]
    for i in range(n_layers):
        z = x @ params[f"mlp/linear_{i}/w"].astype(dtype) + params[f"mlp/linear_{i}/b"].astype(dtype)
        x = np.maximum(z, 0) if i < n_layers - 1 else z
        acts.append(x)
    return x, {"acts": acts}


def mlp_backward(params, cache, dq, dtype, n_layers, masks=None):
    masks = masks or {}
    g, acts, dz = {}, cache["acts"], dq
    for i in reversed(range(n_layers)):
        g[f"mlp/linear_{i}/w"] = acts[i].T @ dz
        g[f"mlp/linear_{i}/b"] = dz.sum(0)
        if i > 0:
            m = masks.get(f"act{i - 1}", acts[i] > 0)
            dz = (dz @ params[f"mlp/linear_{i}/w"].astype(dtype).T) * m
    return g


# ------------------------------------------------------------------ the learner step


@dataclasses.dataclass
class DQNConfig:
    num_actions: int
    network: str = "nature"          # "nature" | "mlp"
    obs_dim: int = 0
    hidden: Tuple[int, ...] = ()
    discount: float = 0.99
    importance_sampling_exponent: float = 0.2
    learning_rate: float = 1e-3
    huber_loss_parameter: float = 1.0
    target_update_period: int = 100
    max_abs_reward: float = 1.0
    adam_beta1: float = 0.9
    adam_beta2: float = 0.999
    adam_epsilon: float = 1e-8
    # "tf": acme/agents/tf/dqn/learning.py (the primary oracle); "jax":
    # acme/agents/jax/dqn/learning.py:74-178 — importance weights cast to f32 before ** beta
    # (:94-96), target copy when (steps + 1) % period == 0 (:114-119 with
    # jax/utils.py:148-154), optix.adam (agents/jax/dqn/agent.py:110).
    semantics: str = "tf"


def forward(cfg: DQNConfig, params, o, dtype):
    if cfg.network == "nature":
        return nature_forward(params, o, dtype)
    return mlp_forward(params, o, dtype, len(cfg.hidden) + 1)


def backward(cfg: DQNConfig, params, cache, dq, dtype, masks=None):
    if cfg.network == "nature":
        return nature_backward(params, cache, dq, dtype, masks)
    return mlp_backward(params, cache, dq, dtype, len(cfg.hidden) + 1, masks)


def dqn_loss_and_grads(cfg: DQNConfig, params, target, batch, dtype=np.float64,
                       global_min_probability: Optional[float] = None, masks=None):
    """Forward + backward of DQNLearner._step; returns (outputs, grads)."""
    o_tm1, a, r, d, o_t = (batch[k] for k in ("o_tm1", "a_tm1", "r_t", "d_t", "o_t"))
    probs = np.asarray(batch["probabilities"], np.float64)
    q_tm1, cache = forward(cfg, params, o_tm1, dtype)
    q_t_value, _ = forward(cfg, target, o_t, dtype)
    q_t_selector, _ = forward(cfg, params, o_t, dtype)
    r = np.clip(r.astype(np.float32), -cfg.max_abs_reward, cfg.max_abs_reward).astype(dtype)
    dd = (d.astype(np.float32) * np.float32(cfg.discount)).astype(dtype)
    best = np.argmax(q_t_selector, axis=1)  # first maximal index, as tf.argmax
    bidx = np.arange(len(a))
    target_v = r + dd * q_t_value[bidx, best]
    td = target_v - q_tm1[bidx, a]
    delta = dtype(cfg.huber_loss_parameter)
    ax = np.abs(td)
    quad = np.minimum(ax, delta)
    hub = 0.5 * quad ** 2 + delta * (ax - quad)
    if cfg.semantics == "jax":  # jax/dqn/learning.py:94-96, all in f32
        beta32 = np.float32(cfg.importance_sampling_exponent)
        iw32 = (1.0 / probs).astype(np.float32) ** beta32
        if global_min_probability is not None:
            wmax32 = np.float32(1.0 / global_min_probability) ** beta32
        else:
            wmax32 = iw32.max()
        iw = (iw32 / wmax32).astype(dtype)
    else:  # tf/dqn/learning.py:138-143: f64, cast to f32 at the multiply
        iw = (1.0 / probs) ** np.float64(cfg.importance_sampling_exponent)
        if global_min_probability is not None:
            wmax = (1.0 / global_min_probability) ** np.float64(cfg.importance_sampling_exponent)
        else:
            wmax = iw.max()
        iw = (iw / wmax).astype(np.float32).astype(dtype)
    loss = np.mean(hub * iw)
    B = len(a)
    dq = np.zeros_like(q_tm1)
    dq[bidx, a] = -(iw * np.clip(td, -delta, delta)) / B
    grads = backward(cfg, params, cache, dq, dtype, masks)
    out = dict(cache=cache, loss=loss, td_error=td, priorities=np.abs(td).astype(np.float64), q_tm1=q_tm1,
               q_t_value=q_t_value, q_t_selector=q_t_selector, importance_weights=iw)
    return out, grads


def adam_update(p, g, m, v, t, lr, b1=0.9, b2=0.999, eps=1e-8, optix=False):
    """snt.optimizers.Adam in float32, op order of the product kernel.  optix=True: the
    optix.adam form (scale_by_adam then scale(-lr)), update = lr * (m_hat / (sqrt(v_hat) + eps))."""
    f = np.float32
    p, g, m, v = (np.asarray(x, f) for x in (p, g, m, v))
    b1, b2, lr, eps = f(b1), f(b2), f(lr), f(eps)
    m = b1 * m + (f(1) - b1) * g
    v = b2 * v + (f(1) - b2) * (g * g)
    bc1 = f(1) - np.power(b1, f(t))
    bc2 = f(1) - np.power(b2, f(t))
    if optix:
        upd = lr * ((m / bc1) / (np.sqrt(v / bc2) + eps))
    else:
        upd = (lr * (m / bc1)) / (np.sqrt(v / bc2) + eps)
    return p - upd, m, v


def dqn_step(cfg: DQNConfig, state: dict, batch: dict, dtype=np.float64):
    """One full learner step.  state = {params, target, m, v, num_steps} (dicts of arrays)."""
    out, grads = dqn_loss_and_grads(cfg, state["params"], state["target"], batch, dtype)
    t = state["num_steps"] + 1
    new_p, new_m, new_v = {}, {}, {}
    for k in state["params"]:
        new_p[k], new_m[k], new_v[k] = adam_update(
            state["params"][k], grads[k], state["m"][k], state["v"][k], t, cfg.learning_rate,
            cfg.adam_beta1, cfg.adam_beta2, cfg.adam_epsilon, optix=cfg.semantics == "jax")
    target = state["target"]
    copy_at = state["num_steps"] + (1 if cfg.semantics == "jax" else 0)
    if copy_at % cfg.target_update_period == 0:
        target = {k: v.copy() for k, v in new_p.items()}
    new_state = dict(params=new_p, target=target, m=new_m, v=new_v,
                     num_steps=state["num_steps"] + 1)
    return out, grads, new_state
