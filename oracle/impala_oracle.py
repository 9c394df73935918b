"""ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py's
cpu_baseline leg).  Never imported by the product package acme_amd.

numpy restatement of the TF IMPALA learner step, IMPALALearner._step
(acme/agents/tf/impala/learning.py:97-169), in float64 (accuracy reference) or float32:

  data = batch_to_sequence(sample.data)  ([B, T] -> [T, B])                 :103
  core_state = extras['core_state'][0]                                     :109
  actions, rewards, discounts = [:-1]                                      :112-114
  (logits, values) = static_unroll(network, observations, core_state)      :118-119
  log_rhos = log pi(a) - log mu(a) (behaviour logits extras['logits'])     :122-125
  rewards clipped to +-max_abs_reward (default inf)                        :128-130
  trfl.vtrace_from_importance_weights(log_rhos, discount * discounts, rewards,
      values[:-1], bootstrap_value=values[-1])  (rho_bar = c_bar = 1)      :133-139
  critic = (vs - values[:-1])^2; pg = -log pi(a) * pg_advantages;
  entropy loss = -H(pi)                                                    :140-150
  loss = mean(pg + baseline_cost * critic + entropy_cost * entropy)        :153-155
  clip_by_global_norm(grads, max_gradient_norm (default 1e10)); Adam(lr)   :158-160

Network: IMPALAAtariNetwork (acme/tf/networks/atari.py:115-144): OAREmbedding
(acme/tf/networks/embedding.py:26-45: concat(torso(obs), one_hot(prev action),
tanh(prev reward))) -> snt.LSTM(256) -> Linear(256) -> ReLU -> PolicyValueHead
(acme/tf/networks/policy_value.py:24-37).  The "flat" torso (identity over a float
observation vector) serves the small parity cases.

Third-party semantics restated (not in /root/reference; parity UNPINNED):
trfl.vtrace_from_importance_weights (clipped rhos / cs = min(1, rho), backward scan
acc_t = delta_t + gamma_t c_t acc_{t+1}, vs = v + acc, pg_adv = min(1, rho) (r + gamma
vs_{t+1} - v), all stop-gradient), trfl.policy_gradient, trfl.policy_entropy_loss,
snt.LSTM (gates = x W_i + h W_h + b split as i, f, g, o; c' = sigmoid(f) c + sigmoid(i)
tanh(g); h' = sigmoid(o) tanh(c')), Sonnet Adam (dqn_oracle.adam_update).
Parameter layout: the product learner's flat buffer; the policy and value layers of the
PolicyValueHead are one fused [H2, A + 1] tensor (column A = value).
"""

from __future__ import annotations

import dataclasses
from typing import Dict, List, Tuple

import numpy as np

from oracle.dqn_oracle import CONVS, _col2im, adam_update, conv_forward, obs_to_float

PREFIX = "impala_atari_network"


@dataclasses.dataclass
class IMPALAConfig:
    num_actions: int = 18
    torso: str = "atari"       # "atari" (uint8 [84, 84, 4]) or "flat" (float [obs_dim])
    obs_dim: int = 0
    lstm_size: int = 256
    head_size: int = 256
    discount: float = 0.99
    entropy_cost: float = 0.01
    baseline_cost: float = 0.5
    max_abs_reward: float = float("inf")
    max_gradient_norm: float = 1e10
    learning_rate: float = 1e-3
    # "tf": agents/tf/impala/learning.py; "jax": agents/jax/impala/learning.py:66-136 with the
    # agent's optix.chain(clip_by_global_norm(max_gradient_norm), adam(lr))
    # (agents/jax/impala/agent.py:98-101).  The rlax losses (categorical IS ratios,
    # vtrace_td_error_and_advantage with lambda 1 and rho / pg-rho clips 1, policy_gradient_loss,
    # entropy_loss, per-sequence means averaged by vmap + mean) equal the TF ones here: every
    # sequence has T - 1 terms, so the mean of per-sequence means is the [T - 1, B] mean.
    semantics: str = "tf"

    @property
    def feat(self) -> int:
        return 7744 if self.torso == "atari" else self.obs_dim

    @property
    def embed(self) -> int:
        return self.feat + self.num_actions + 1


def tensor_shapes(cfg: IMPALAConfig) -> List[Tuple[str, Tuple[int, ...]]]:
    H, H2, A = cfg.lstm_size, cfg.head_size, cfg.num_actions
    out = []
    if cfg.torso == "atari":
        out += [(f"{PREFIX}/atari_torso/conv2_d/w", (8, 8, 4, 32)),
                (f"{PREFIX}/atari_torso/conv2_d/b", (32,)),
                (f"{PREFIX}/atari_torso/conv2_d_1/w", (4, 4, 32, 64)),
                (f"{PREFIX}/atari_torso/conv2_d_1/b", (64,)),
                (f"{PREFIX}/atari_torso/conv2_d_2/w", (3, 3, 64, 64)),
                (f"{PREFIX}/atari_torso/conv2_d_2/b", (64,))]
    out += [(f"{PREFIX}/lstm/w_i", (cfg.embed, 4 * H)), (f"{PREFIX}/lstm/w_h", (H, 4 * H)),
            (f"{PREFIX}/lstm/b", (4 * H,)),
            (f"{PREFIX}/linear/w", (H, H2)), (f"{PREFIX}/linear/b", (H2,)),
            (f"{PREFIX}/policy_value/w", (H2, A + 1)), (f"{PREFIX}/policy_value/b", (A + 1,))]
    return out


def _torso_names():
    return [f"{PREFIX}/atari_torso/{n.split('/')[-1]}" for n, _, _ in CONVS]


def sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def log_softmax(x):
    m = x.max(axis=-1, keepdims=True)
    z = x - m
    return z - np.log(np.exp(z).sum(axis=-1, keepdims=True))


# ------------------------------------------------------------------ forward


def forward(cfg: IMPALAConfig, p, batch, dtype):
    """Unroll over [B, T]; returns logits [B, T, A], values [B, T] and the cache."""
    f = dtype
    obs = batch["obs"]
    B, T = batch["action"].shape
    A, H = cfg.num_actions, cfg.lstm_size
    cache = {}
    frames = obs.reshape((B * T,) + obs.shape[2:])
    if cfg.torso == "atari":
        x = obs_to_float(frames, f)
        for li, (name, (_, s, pads)) in enumerate(zip(_torso_names(), CONVS)):
            z, (cols, meta) = conv_forward(x, p[name + "/w"].astype(f), p[name + "/b"].astype(f),
                                           s, pads)
            x = np.maximum(z, 0)
            cache[f"cols{li}"] = (cols, meta)
            cache[f"x{li + 1}"] = x
        feats = x.reshape(B * T, -1)
    else:
        feats = frames.reshape(B * T, -1).astype(f)
    onehot = np.eye(A, dtype=f)[batch["prev_action"].reshape(-1)]
    emb = np.concatenate([feats, onehot, np.tanh(batch["prev_reward"].astype(f)).reshape(-1, 1)],
                         axis=1)  # [B*T, D], row = b * T + t
    gx = emb @ p[f"{PREFIX}/lstm/w_i"].astype(f) + p[f"{PREFIX}/lstm/b"].astype(f)
    gx = gx.reshape(B, T, 4 * H)
    wh = p[f"{PREFIX}/lstm/w_h"].astype(f)
    h = batch["h0"].astype(f)
    c = batch["c0"].astype(f)
    hs, cs, gates = np.zeros((B, T, H), f), np.zeros((B, T, H), f), np.zeros((B, T, 4 * H), f)
    for t in range(T):
        z = gx[:, t] + h @ wh
        i, fg, g, o = (sigmoid(z[:, :H]), sigmoid(z[:, H:2 * H]), np.tanh(z[:, 2 * H:3 * H]),
                       sigmoid(z[:, 3 * H:]))
        c = fg * c + i * g
        h = o * np.tanh(c)
        hs[:, t], cs[:, t] = h, c
        gates[:, t] = np.concatenate([i, fg, g, o], axis=1)
    hflat = hs.reshape(B * T, H)
    hz = hflat @ p[f"{PREFIX}/linear/w"].astype(f) + p[f"{PREFIX}/linear/b"].astype(f)
    hh = np.maximum(hz, 0)
    pv = hh @ p[f"{PREFIX}/policy_value/w"].astype(f) + p[f"{PREFIX}/policy_value/b"].astype(f)
    logits = pv[:, :A].reshape(B, T, A)
    values = pv[:, A].reshape(B, T)
    cache.update(feats=feats, emb=emb, hs=hs, cs=cs, gates=gates, hh=hh)
    return logits, values, cache


def vtrace(log_rhos, discounts, rewards, values, bootstrap):
    """trfl.vtrace_from_importance_weights with clip thresholds 1 ([T, B] time-major)."""
    rhos = np.exp(log_rhos)
    clipped = np.minimum(1.0, rhos)
    cs = np.minimum(1.0, rhos)
    v_tp1 = np.concatenate([values[1:], bootstrap[None]], axis=0)
    deltas = clipped * (rewards + discounts * v_tp1 - values)
    acc = np.zeros_like(bootstrap)
    vs_minus_v = np.zeros_like(values)
    for t in reversed(range(values.shape[0])):
        acc = deltas[t] + discounts[t] * cs[t] * acc
        vs_minus_v[t] = acc
    vs = vs_minus_v + values
    vs_tp1 = np.concatenate([vs[1:], bootstrap[None]], axis=0)
    pg_adv = clipped * (rewards + discounts * vs_tp1 - values)
    return vs, pg_adv


def loss_and_grads(cfg: IMPALAConfig, p, batch, dtype=np.float64, masks=None):
    """masks: optional ReLU patterns {"x1", "x2", "x3", "hh"} that replace (x > 0) in the
    backward pass (a kernel's own branch decisions, for kink-conditioned comparisons)."""
    f = dtype
    B, T = batch["action"].shape
    A, H = cfg.num_actions, cfg.lstm_size
    logits, values, cache = forward(cfg, p, batch, f)
    # Time-major, drop the last action / reward / discount.
    lg = np.swapaxes(logits, 0, 1)[:-1]           # [T-1, B, A]
    v = np.swapaxes(values, 0, 1)                  # [T, B]
    act = np.swapaxes(batch["action"], 0, 1)[:-1]
    rew = np.swapaxes(batch["reward"], 0, 1)[:-1].astype(f)
    disc = np.swapaxes(batch["discount"], 0, 1)[:-1].astype(f)
    mu = np.swapaxes(batch["behaviour_logits"], 0, 1)[:-1].astype(f)
    logp = log_softmax(lg)
    logmu = log_softmax(mu)
    lp_a = np.take_along_axis(logp, act[..., None], -1)[..., 0]
    log_rhos = lp_a - np.take_along_axis(logmu, act[..., None], -1)[..., 0]
    rew = np.clip(rew, -cfg.max_abs_reward, cfg.max_abs_reward)
    gdisc = (f(np.float32(cfg.discount)) * disc).astype(f)
    vs, pg_adv = vtrace(log_rhos, gdisc, rew, v[:-1], v[-1])
    pi = np.exp(logp)
    ent = -(pi * logp).sum(-1)
    critic = np.square(vs - v[:-1])
    pg = -lp_a * pg_adv
    total = pg + cfg.baseline_cost * critic + cfg.entropy_cost * (-ent)
    N = total.size
    loss = total.mean()
    # d loss / d logits (t < T-1), d loss / d values (t < T-1).
    onehot = np.eye(A, dtype=f)[act]
    dlg = (-(onehot - pi) * pg_adv[..., None]
           + cfg.entropy_cost * pi * (logp + ent[..., None])) / N
    dv = cfg.baseline_cost * (-2.0) * (vs - v[:-1]) / N
    dlogits = np.zeros((T, B, A), f)
    dvalues = np.zeros((T, B), f)
    dlogits[:-1], dvalues[:-1] = dlg, dv
    dpv = np.concatenate([np.swapaxes(dlogits, 0, 1).reshape(B * T, A),
                          np.swapaxes(dvalues, 0, 1).reshape(B * T, 1)], axis=1)
    grads = backward(cfg, p, batch, cache, dpv, f, masks)
    out = dict(loss=loss, critic_loss=critic.mean(), entropy_loss=(-ent).mean(),
               policy_gradient_loss=pg.mean(), logits=logits, values=values, vs=vs,
               pg_advantages=pg_adv, log_rhos=log_rhos, dpv=dpv, hs=cache["hs"],
               cs=cache["cs"])
    return out, grads


def backward(cfg: IMPALAConfig, p, batch, cache, dpv, f, masks=None):
    B, T = batch["action"].shape
    H = cfg.lstm_size
    g = {}
    hh = cache["hh"]

    def relu_mask(name, x):
        if masks is not None and name in masks:
            return masks[name].reshape(x.shape)
        return x > 0

    g[f"{PREFIX}/policy_value/w"] = hh.T @ dpv
    g[f"{PREFIX}/policy_value/b"] = dpv.sum(0)
    dhh = (dpv @ p[f"{PREFIX}/policy_value/w"].astype(f).T) * relu_mask("hh", hh)
    hflat = cache["hs"].reshape(B * T, H)
    g[f"{PREFIX}/linear/w"] = hflat.T @ dhh
    g[f"{PREFIX}/linear/b"] = dhh.sum(0)
    dh_head = (dhh @ p[f"{PREFIX}/linear/w"].astype(f).T).reshape(B, T, H)
    # BPTT.
    wh = p[f"{PREFIX}/lstm/w_h"].astype(f)
    gates, cs, hs = cache["gates"], cache["cs"], cache["hs"]
    dgates = np.zeros((B, T, 4 * H), f)
    dh_next = np.zeros((B, H), f)
    dc_next = np.zeros((B, H), f)
    for t in reversed(range(T)):
        i, fg, gg, o = (gates[:, t, :H], gates[:, t, H:2 * H], gates[:, t, 2 * H:3 * H],
                        gates[:, t, 3 * H:])
        c = cs[:, t]
        c_prev = cs[:, t - 1] if t > 0 else batch["c0"].astype(f)
        tc = np.tanh(c)
        dh = dh_head[:, t] + dh_next
        dc = dc_next + dh * o * (1 - tc * tc)
        do = dh * tc * o * (1 - o)
        di = dc * gg * i * (1 - i)
        dg = dc * i * (1 - gg * gg)
        df = dc * c_prev * fg * (1 - fg)
        dz = np.concatenate([di, df, dg, do], axis=1)
        dgates[:, t] = dz
        dh_next = dz @ wh.T
        dc_next = dc * fg
    h_prev = np.concatenate([batch["h0"].astype(f)[:, None], hs[:, :-1]], axis=1)
    dgf = dgates.reshape(B * T, 4 * H)
    g[f"{PREFIX}/lstm/w_h"] = h_prev.reshape(B * T, H).T @ dgf
    g[f"{PREFIX}/lstm/w_i"] = cache["emb"].T @ dgf
    g[f"{PREFIX}/lstm/b"] = dgf.sum(0)
    if cfg.torso == "atari":
        dfeat = dgf @ p[f"{PREFIX}/lstm/w_i"].astype(f)[:cfg.feat].T
        dx = dfeat.reshape(cache["x3"].shape) * relu_mask("x3", cache["x3"])
        for li in (2, 1, 0):
            name = _torso_names()[li]
            _, s, pads = CONVS[li]
            w = p[name + "/w"].astype(f)
            kh, kw, ci, co = w.shape
            cols, meta = cache[f"cols{li}"]
            dz = dx.reshape(-1, co)
            g[name + "/w"] = (cols.T @ dz).reshape(w.shape)
            g[name + "/b"] = dz.sum(0)
            if li > 0:
                dcols = dz @ w.reshape(-1, co).T
                xin = cache[f"x{li}"]
                dx = _col2im(dcols, meta, kh, kw, s, pads, xin.shape) * relu_mask(f"x{li}", xin)
    return g


def clip_by_global_norm(grads, clip, f, optix=False):
    """tf.clip_by_global_norm: g * c * min(1 / G, 1 / c).  optix=True: optix's
    clip_by_global_norm, g unchanged when G < c, else (g / G) * c."""
    G = np.sqrt(sum(float(np.sum(np.square(x.astype(np.float64)))) for x in grads.values()))
    if optix:
        if G < clip:
            return {k: x.astype(f) for k, x in grads.items()}, G
        return {k: ((x / f(G)) * f(clip)).astype(f) for k, x in grads.items()}, G
    scale = f(clip) * min(f(1.0) / f(G), f(1.0) / f(clip)) if G > 0 else f(1.0)
    return {k: (x * f(scale)).astype(f) for k, x in grads.items()}, G


def impala_step(cfg: IMPALAConfig, state: dict, batch: dict, dtype=np.float64, masks=None):
    """One learner step. state = {params, m, v, num_steps}."""
    out, raw = loss_and_grads(cfg, state["params"], batch, dtype, masks)
    jax = cfg.semantics == "jax"
    grads, out["grad_norm"] = clip_by_global_norm(raw, cfg.max_gradient_norm, dtype, optix=jax)
    t = state["num_steps"] + 1
    new_p, new_m, new_v = {}, {}, {}
    for k in state["params"]:
        new_p[k], new_m[k], new_v[k] = adam_update(state["params"][k], grads[k], state["m"][k],
                                                   state["v"][k], t, cfg.learning_rate,
                                                   optix=jax)
    return out, raw, dict(params=new_p, m=new_m, v=new_v, num_steps=t)
