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


# ====================================================================== the learner step
# numpy restatement of R2D2Learner._step (acme/agents/tf/r2d2/learning.py:112-200) with
# R2D2AtariNetwork (acme/tf/networks/atari.py:72-112): OAREmbedding(AtariTorso) ->
# snt.LSTM(512) -> DuellingMLP(num_actions, [512]) (acme/tf/networks/duelling.py:26-59),
# in float64 (the accuracy reference) or float32.
#
#   core_state = extras['core_state'][0] (store_lstm_state) else zeros         :127-131
#   burn-in: both networks unrolled over the first burn_in steps, no gradient   :134-137
#   q = net.unroll(obs[burn:]), target_q = target.unroll(obs[burn:])            :146-150
#     (= one continuous unroll over all T steps, the burn-in's state carried)
#   greedy = argmax q (first max); target policy = one_hot(greedy)             :153-155
#   transformed_n_step_loss(q, target_q, actions, rewards[:-1],
#       discounts[:-1] * discount, one_hot, n)                                  :158-168
#     (acme/tf/losses/r2d2.py:29-119: bootstrap = sum(pi * h^-1(target_q[1:])),
#      n-step targets :122-169, non-finite targets masked to 0,
#      errors = q[:-1][a] - h(target), loss = 0.5 sum_t errors^2 per sequence)
#   w = (1 / (N p))^beta / max, f64, cast to f32; loss = mean(loss * w) over
#     the [T, B] broadcast (= the mean over sequences)                          :171-178
#   snt.Adam(lr, epsilon=1e-3), no gradient clipping                            :78, :181-182
#   if num_steps % period == 0: target <- online (after the update)            :185-189
#   priorities = eta max_t |errors| + (1 - eta) mean_t |errors|                 :192-199
#
# Third-party semantics restated (parity UNPINNED, SURVEY.md §8(c): no reference test
# holds an R2D2 learner value): trfl.batched_index, snt.LSTM, snt.static_unroll, Sonnet
# Adam (dqn_oracle.adam_update).  The DuellingMLP's two first layers are one fused
# [H, 2 H2] tensor [value | advantage] as in the DQN learner (dqn_oracle.py).

import dataclasses
from typing import Dict, List, Tuple

from oracle.dqn_oracle import CONVS, _col2im, adam_update, conv_forward, obs_to_float

PREFIX = "r2d2_atari_network"


@dataclasses.dataclass
class R2D2Config:
    num_actions: int = 18
    torso: str = "atari"        # "atari" (uint8 [84, 84, 4]) or "flat" (float [obs_dim])
    obs_dim: int = 0
    lstm_size: int = 512
    head_size: int = 512        # DuellingMLP hidden size
    burn_in_length: int = 40
    n_step: int = 5
    discount: float = 0.99
    importance_sampling_exponent: float = 0.2
    max_replay_size: int = 1_000_000
    max_priority_weight: float = 0.9
    target_update_period: int = 100
    learning_rate: float = 1e-3
    adam_epsilon: float = 1e-3
    store_lstm_state: bool = True

    @property
    def feat(self) -> int:
        return 7744 if self.torso == "atari" else self.obs_dim

    @property
    def embed(self) -> int:
        return self.feat + self.num_actions + 1


def tensor_shapes(cfg: R2D2Config) -> List[Tuple[str, Tuple[int, ...]]]:
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
            (f"{PREFIX}/duelling_q_network/hidden/w", (H, 2 * H2)),
            (f"{PREFIX}/duelling_q_network/hidden/b", (2 * H2,)),
            (f"{PREFIX}/duelling_q_network/mlp/linear_1/w", (H2, 1)),
            (f"{PREFIX}/duelling_q_network/mlp/linear_1/b", (1,)),
            (f"{PREFIX}/duelling_q_network/mlp_1/linear_1/w", (H2, A)),
            (f"{PREFIX}/duelling_q_network/mlp_1/linear_1/b", (A,))]
    return out


def _torso_names():
    return [f"{PREFIX}/atari_torso/{n.split('/')[-1]}" for n, _, _ in CONVS]


def _sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def signed_hyperbolic(x, eps=1e-3):
    """losses/r2d2.py:172-174."""
    return np.sign(x) * (np.sqrt(np.abs(x) + 1) - 1) + eps * x


def signed_parabolic(x, eps=1e-3):
    """losses/r2d2.py:177-180."""
    z = np.sqrt(1 + 4 * eps * (eps + 1 + np.abs(x))) / 2 / eps - 1 / 2 / eps
    return np.sign(x) * (np.square(z) - 1)


def signed_hyperbolic_f32(x):
    """_signed_hyperbolic_tx in TF's float32 arithmetic (eps * x with eps an f32 constant)."""
    f = np.float32
    x = np.asarray(x, f)
    return (np.sign(x) * (np.sqrt(np.abs(x) + f(1)) - f(1)) + f(1e-3) * x).astype(f)


def signed_parabolic_f32(x):
    """_signed_parabolic_tx in TF's float32 arithmetic: Python folds eps + 1, 4 * eps and
    1 / 2 / eps into the f32 constants 1.001, 0.004 and 500; then sqrt, / 2, / eps, - 500.
    The subtraction of 500 from ~501 leaves the result with an absolute resolution of
    ulp(512) = 6.1e-5: the reference's own f32 loss carries that rounding."""
    f = np.float32
    x = np.asarray(x, f)
    t = f(0.004) * (f(1.001) + np.abs(x))
    z = np.sqrt(f(1) + t) / f(2) / f(1e-3) - f(500)
    return (np.sign(x) * (np.square(z) - f(1))).astype(f)


def n_step_targets(r_t, pcont_t, bootstrap_value, n):
    """losses/r2d2.py:122-169 over [T, B] time-major arrays."""
    T, B = r_t.shape
    f = r_t.dtype
    r = np.concatenate([r_t, np.zeros((n - 1, B), f)], 0)
    pc = np.concatenate([pcont_t, np.ones((n - 1, B), f)], 0)
    last = bootstrap_value[T - 1:T]
    if T > n - 1:
        boot = np.concatenate([bootstrap_value[n - 1:T]] + [last] * (n - 1), 0)
    else:
        boot = np.concatenate([last] * T, 0)
    targets = boot
    for i in range(n - 1, -1, -1):
        targets = r[i:i + T] + pc[i:i + T] * targets
    return targets


def forward(cfg: R2D2Config, p, batch, dtype):
    """Unroll over all T steps of [B, T] from the batch's core state; q [B, T, A]."""
    f = dtype
    obs = batch["obs"]
    B, T = batch["action"].shape
    A, H, H2 = cfg.num_actions, cfg.lstm_size, cfg.head_size
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
    gx = (emb @ p[f"{PREFIX}/lstm/w_i"].astype(f) + p[f"{PREFIX}/lstm/b"].astype(f))
    gx = gx.reshape(B, T, 4 * H)
    wh = p[f"{PREFIX}/lstm/w_h"].astype(f)
    if cfg.store_lstm_state:
        h, c = batch["h0"].astype(f), batch["c0"].astype(f)
    else:
        h, c = np.zeros((B, H), f), np.zeros((B, H), f)
    cache["h0"], cache["c0"] = h, c
    hs, cs, gates = np.zeros((B, T, H), f), np.zeros((B, T, H), f), np.zeros((B, T, 4 * H), f)
    for t in range(T):
        z = gx[:, t] + h @ wh
        i, fg, g, o = (_sigmoid(z[:, :H]), _sigmoid(z[:, H:2 * H]), np.tanh(z[:, 2 * H:3 * H]),
                       _sigmoid(z[:, 3 * H:]))
        c = fg * c + i * g
        h = o * np.tanh(c)
        hs[:, t], cs[:, t] = h, c
        gates[:, t] = np.concatenate([i, fg, g, o], axis=1)
    hflat = hs.reshape(B * T, H)
    D = f"{PREFIX}/duelling_q_network"
    hid = np.maximum(hflat @ p[f"{D}/hidden/w"].astype(f) + p[f"{D}/hidden/b"].astype(f), 0)
    v = hid[:, :H2] @ p[f"{D}/mlp/linear_1/w"].astype(f) + p[f"{D}/mlp/linear_1/b"].astype(f)
    adv = hid[:, H2:] @ p[f"{D}/mlp_1/linear_1/w"].astype(f) + p[f"{D}/mlp_1/linear_1/b"].astype(f)
    q = v + (adv - adv.mean(axis=-1, keepdims=True))
    cache.update(feats=feats, emb=emb, hs=hs, cs=cs, gates=gates, hid=hid)
    return q.reshape(B, T, A), cache


def transformed_loss(cfg: R2D2Config, q, tq, batch, dtype=np.float32):
    """losses/r2d2.py:29-119 on the suffix q values q / tq [L, B, A] (time-major, online /
    target); dtype float32 = TF's arithmetic (the transforms with f32 constants, the n-step
    folds r + pcont target), float64 = exact.  Returns (errors, targets) [L - 1, B]."""
    f = dtype
    BI, n, A = cfg.burn_in_length, cfg.n_step, cfg.num_actions
    q, tq = np.asarray(q, f), np.asarray(tq, f)
    act = np.swapaxes(batch["action"][:, BI:], 0, 1)  # [L, B]
    rew = np.swapaxes(batch["reward"][:, BI:], 0, 1)[:-1].astype(np.float32).astype(f)
    disc = np.swapaxes(batch["discount"][:, BI:], 0, 1)[:-1].astype(np.float32)
    pcont = (disc * np.float32(cfg.discount)).astype(f)  # f32 discounts * python float
    greedy = np.argmax(q, axis=-1)                    # first maximal index, as tf.argmax
    pi = np.eye(A, dtype=f)[greedy]
    par = signed_parabolic_f32 if f == np.float32 else signed_parabolic
    hyp = signed_hyperbolic_f32 if f == np.float32 else signed_hyperbolic
    with np.errstate(invalid="ignore", over="ignore"):
        bootstrap = np.zeros(pi[1:].shape[:2], f)   # sum over actions in order
        ptq = par(tq[1:])
        for j in range(A):
            bootstrap = (bootstrap + pi[1:, :, j] * ptq[:, :, j]).astype(f)
        targets = n_step_targets(rew, pcont, bootstrap, n).astype(f)
    finite = np.isfinite(targets)
    targets = np.where(finite, targets, 0.0).astype(f)
    a_tm1 = act[:-1]
    qa = np.take_along_axis(q[:-1], a_tm1[..., None], -1)[..., 0]
    errors = np.where(finite, qa - hyp(targets), 0.0).astype(f)
    return errors, targets


def loss_and_grads(cfg: R2D2Config, params, target, batch, dtype=np.float64, masks=None,
                   loss_dtype=np.float32):
    """Forward + backward of R2D2Learner._step; returns (outputs, grads).  The networks run
    in `dtype`; the transformed loss in `loss_dtype` (float32: TF's arithmetic, whose value
    transforms have an absolute resolution of ~6e-5, see signed_parabolic_f32).  masks:
    optional ReLU patterns {"x1", "x2", "x3", "hid"} replacing (x > 0) in the backward."""
    f = dtype
    B, T = batch["action"].shape
    A, BI = cfg.num_actions, cfg.burn_in_length
    L = T - BI
    q_on, cache = forward(cfg, params, batch, f)
    q_tg, _ = forward(cfg, target, batch, f)
    q = np.swapaxes(q_on[:, BI:], 0, 1)             # [L, B, A]
    tq = np.swapaxes(q_tg[:, BI:], 0, 1)
    act = np.swapaxes(batch["action"][:, BI:], 0, 1)  # [L, B]
    a_tm1 = act[:-1]
    errors, targets = transformed_loss(cfg, q, tq, batch, loss_dtype)
    errors = errors.astype(f)
    seq_loss = 0.5 * np.sum(np.square(errors), axis=0)  # [B]
    probs = np.asarray(batch["probabilities"], np.float64)
    iw = (1.0 / (cfg.max_replay_size * probs)) ** np.float64(cfg.importance_sampling_exponent)
    iw = (iw / iw.max()).astype(np.float32).astype(f)
    loss = np.mean(seq_loss * iw)
    dq = np.zeros((B, T, A), f)
    g_err = errors * iw[None, :] / B                  # d loss / d q[:-1][a]  [L-1, B]
    for t in range(L - 1):
        dq[np.arange(B), BI + t, a_tm1[t]] += g_err[t]
    grads = backward(cfg, params, batch, cache, dq.reshape(B * T, A), f, masks)
    prio = compute_priority(errors.astype(np.float32), cfg.max_priority_weight)
    out = dict(loss=loss, errors=errors, targets=targets, priorities=prio, q=q_on, target_q=q_tg,
               importance_weights=iw, hs=cache["hs"], dq=dq)
    return out, grads


def backward(cfg: R2D2Config, p, batch, cache, dq, f, masks=None):
    """Gradients of the step's loss; rows t < burn_in carry none (the burn-in is outside the
    gradient tape, learning.py:134-137: BPTT stops at t = burn_in)."""
    B, T = batch["action"].shape
    H, H2, BI = cfg.lstm_size, cfg.head_size, cfg.burn_in_length
    g = {}
    D = f"{PREFIX}/duelling_q_network"

    def relu_mask(name, x):
        if masks is not None and name in masks:
            return masks[name].reshape(x.shape)
        return x > 0

    hid = cache["hid"]
    dv = dq.sum(axis=1, keepdims=True)
    dadv = dq - dq.mean(axis=1, keepdims=True)
    wv = p[f"{D}/mlp/linear_1/w"].astype(f)
    wa = p[f"{D}/mlp_1/linear_1/w"].astype(f)
    g[f"{D}/mlp/linear_1/w"] = hid[:, :H2].T @ dv
    g[f"{D}/mlp/linear_1/b"] = dv.sum(0)
    g[f"{D}/mlp_1/linear_1/w"] = hid[:, H2:].T @ dadv
    g[f"{D}/mlp_1/linear_1/b"] = dadv.sum(0)
    dhid = np.concatenate([dv @ wv.T, dadv @ wa.T], axis=1) * relu_mask("hid", hid)
    hflat = cache["hs"].reshape(B * T, H)
    g[f"{D}/hidden/w"] = hflat.T @ dhid
    g[f"{D}/hidden/b"] = dhid.sum(0)
    dh_head = (dhid @ p[f"{D}/hidden/w"].astype(f).T).reshape(B, T, H)
    wh = p[f"{PREFIX}/lstm/w_h"].astype(f)
    gates, cs, hs = cache["gates"], cache["cs"], cache["hs"]
    dgates = np.zeros((B, T, 4 * H), f)
    dh_next = np.zeros((B, H), f)
    dc_next = np.zeros((B, H), f)
    for t in range(T - 1, BI - 1, -1):
        i, fg, gg, o = (gates[:, t, :H], gates[:, t, H:2 * H], gates[:, t, 2 * H:3 * H],
                        gates[:, t, 3 * H:])
        c = cs[:, t]
        c_prev = cs[:, t - 1] if t > 0 else cache["c0"]
        tc = np.tanh(c)
        dh = dh_head[:, t] + dh_next
        dc = dc_next + dh * o * (1 - tc * tc)
        dz = np.concatenate([dc * gg * i * (1 - i), dc * c_prev * fg * (1 - fg),
                             dc * i * (1 - gg * gg), dh * tc * o * (1 - o)], axis=1)
        dgates[:, t] = dz
        dh_next = dz @ wh.T
        dc_next = dc * fg
    h_prev = np.concatenate([cache["h0"][:, None], hs[:, :-1]], axis=1)
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


def r2d2_step(cfg: R2D2Config, state: dict, batch: dict, dtype=np.float64, masks=None):
    """One learner step.  state = {params, target, m, v, num_steps}."""
    out, grads = loss_and_grads(cfg, state["params"], state["target"], batch, dtype, masks)
    t = state["num_steps"] + 1
    new_p, new_m, new_v = {}, {}, {}
    for k in state["params"]:
        new_p[k], new_m[k], new_v[k] = adam_update(state["params"][k], grads[k], state["m"][k],
                                                   state["v"][k], t, cfg.learning_rate,
                                                   eps=cfg.adam_epsilon)
    target = state["target"]
    if state["num_steps"] % cfg.target_update_period == 0:
        target = {k: x.copy() for k, x in new_p.items()}
    return out, grads, dict(params=new_p, target=target, m=new_m, v=new_v, num_steps=t)


def init_params(cfg: R2D2Config, seed: int) -> Dict[str, np.ndarray]:
    """Sonnet-style initialisers (truncated normal, stddev 1 / sqrt(fan_in); zero biases)."""
    rng = np.random.default_rng(seed)
    out = {}
    for name, shape in tensor_shapes(cfg):
        if name.endswith("/b"):
            out[name] = np.zeros(shape, np.float32)
        else:
            fan_in = int(np.prod(shape[:-1]))
            x = rng.standard_normal(shape)
            x = np.clip(x, -2, 2) / np.sqrt(fan_in)
            out[name] = x.astype(np.float32)
    return out
