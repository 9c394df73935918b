"""Network descriptors for the native learners.

The reference builds Sonnet modules (acme/tf/networks/atari.py:36-69 DQNAtariNetwork,
acme/tf/networks/duelling.py:27-59 DuellingMLP, snt.nets.MLP in
examples/bsuite/run_dqn.py:46-49).  Here a network is a small descriptor: the learner's
HIP kernels implement the layers, and the descriptor fixes the architecture, the input
dtype and the initial parameters (Sonnet defaults: TruncatedNormal(stddev=1/sqrt(fan_in))
weights, zero biases).

Parameter naming follows the learner's flat buffer; `to_sonnet` /
`from_sonnet` translate the fused duelling hidden layer to/from Sonnet's separate
value/advantage MLP variables.
"""

from __future__ import annotations

import dataclasses
from typing import Dict, List, NamedTuple, Sequence, Tuple

import numpy as np


def truncated_normal(rng: np.random.Generator, shape, stddev: float) -> np.ndarray:
    """TruncatedNormal(0, stddev) cut at 2 stddev (snt.initializers.TruncatedNormal)."""
    out = rng.standard_normal(shape)
    bad = np.abs(out) > 2.0
    while bad.any():
        out[bad] = rng.standard_normal(int(bad.sum()))
        bad = np.abs(out) > 2.0
    return (out * stddev).astype(np.float32)


@dataclasses.dataclass(frozen=True)
class DQNAtariNetwork:
    """AtariTorso + DuellingMLP(num_actions, hidden_sizes=[512]) on uint8 [84, 84, 4]."""

    num_actions: int
    obs_dtype: str = "uint8"  # uint8 frames scaled by 1/255 inside conv1, or "float32"
    kind: str = dataclasses.field(default="nature", init=False)

    def tensor_shapes(self) -> List[Tuple[str, Tuple[int, ...]]]:
        A = self.num_actions
        return [
            ("atari_torso/conv2_d/w", (8, 8, 4, 32)), ("atari_torso/conv2_d/b", (32,)),
            ("atari_torso/conv2_d_1/w", (4, 4, 32, 64)), ("atari_torso/conv2_d_1/b", (64,)),
            ("atari_torso/conv2_d_2/w", (3, 3, 64, 64)), ("atari_torso/conv2_d_2/b", (64,)),
            ("duelling_q_network/hidden/w", (7744, 1024)), ("duelling_q_network/hidden/b", (1024,)),
            ("duelling_q_network/mlp/linear_1/w", (512, 1)),
            ("duelling_q_network/mlp/linear_1/b", (1,)),
            ("duelling_q_network/mlp_1/linear_1/w", (512, A)),
            ("duelling_q_network/mlp_1/linear_1/b", (A,)),
        ]

    @property
    def obs_shape(self) -> Tuple[int, ...]:
        return (84, 84, 4)

    def init(self, seed: int = 0) -> Dict[str, np.ndarray]:
        rng = np.random.default_rng(seed)
        out = {}
        for name, shape in self.tensor_shapes():
            if name.endswith("/b"):
                out[name] = np.zeros(shape, np.float32)
            else:
                fan_in = int(np.prod(shape[:-1]))
                out[name] = truncated_normal(rng, shape, 1.0 / np.sqrt(fan_in))
        # The fused hidden layer is two Linear(7744 -> 512) layers side by side: the
        # fan-in is 7744 for both halves, which the generic rule above already uses.
        return out

    def to_sonnet(self, params: Dict[str, np.ndarray]) -> Dict[str, np.ndarray]:
        """Splits the fused hidden layer into Sonnet's value/advantage MLP variables."""
        out = {k: v for k, v in params.items() if not k.startswith("duelling_q_network/hidden")}
        w, b = params["duelling_q_network/hidden/w"], params["duelling_q_network/hidden/b"]
        out["duelling_q_network/mlp/linear_0/w"] = w[:, :512]
        out["duelling_q_network/mlp/linear_0/b"] = b[:512]
        out["duelling_q_network/mlp_1/linear_0/w"] = w[:, 512:]
        out["duelling_q_network/mlp_1/linear_0/b"] = b[512:]
        return out

    def from_sonnet(self, variables: Dict[str, np.ndarray]) -> Dict[str, np.ndarray]:
        out = {k: v for k, v in variables.items() if "/linear_0/" not in k}
        out["duelling_q_network/hidden/w"] = np.concatenate(
            [variables["duelling_q_network/mlp/linear_0/w"],
             variables["duelling_q_network/mlp_1/linear_0/w"]], axis=1)
        out["duelling_q_network/hidden/b"] = np.concatenate(
            [variables["duelling_q_network/mlp/linear_0/b"],
             variables["duelling_q_network/mlp_1/linear_0/b"]])
        return out


@dataclasses.dataclass(frozen=True)
class MLP:
    """snt.Sequential([snt.Flatten(), snt.nets.MLP([*hidden, num_actions])])."""

    obs_dim: int
    hidden: Tuple[int, ...]
    num_actions: int
    obs_dtype: str = "float32"
    kind: str = dataclasses.field(default="mlp", init=False)

    def __init__(self, obs_dim: int, hidden: Sequence[int], num_actions: int,
                 obs_dtype: str = "float32"):
        object.__setattr__(self, "obs_dim", int(obs_dim))
        object.__setattr__(self, "hidden", tuple(int(h) for h in hidden))
        object.__setattr__(self, "num_actions", int(num_actions))
        object.__setattr__(self, "obs_dtype", obs_dtype)
        object.__setattr__(self, "kind", "mlp")

    def tensor_shapes(self):
        out, d = [], self.obs_dim
        for i, h in enumerate(list(self.hidden) + [self.num_actions]):
            out.append((f"mlp/linear_{i}/w", (d, h)))
            out.append((f"mlp/linear_{i}/b", (h,)))
            d = h
        return out

    @property
    def obs_shape(self) -> Tuple[int, ...]:
        return (self.obs_dim,)

    def init(self, seed: int = 0) -> Dict[str, np.ndarray]:
        rng = np.random.default_rng(seed)
        out = {}
        for name, shape in self.tensor_shapes():
            if name.endswith("/b"):
                out[name] = np.zeros(shape, np.float32)
            else:
                out[name] = truncated_normal(rng, shape, 1.0 / np.sqrt(shape[0]))
        return out

    def to_sonnet(self, params):
        return dict(params)

    def from_sonnet(self, variables):
        return dict(variables)


# ------------------------------------------------------------------ D4PG (control suite)


def _variance_scaling_uniform(rng, shape, scale: float, fan: int) -> np.ndarray:
    limit = np.sqrt(3.0 * scale / fan)
    return rng.uniform(-limit, limit, shape).astype(np.float32)


def _layer_norm_mlp_shapes(prefix: str, din: int, sizes: Sequence[int]):
    out = [(f"{prefix}/layer_norm_mlp/linear/w", (din, sizes[0])),
           (f"{prefix}/layer_norm_mlp/linear/b", (sizes[0],)),
           (f"{prefix}/layer_norm_mlp/layer_norm/scale", (sizes[0],)),
           (f"{prefix}/layer_norm_mlp/layer_norm/offset", (sizes[0],))]
    for i in range(1, len(sizes)):
        out += [(f"{prefix}/layer_norm_mlp/mlp/linear_{i - 1}/w", (sizes[i - 1], sizes[i])),
                (f"{prefix}/layer_norm_mlp/mlp/linear_{i - 1}/b", (sizes[i],))]
    return out


def _init_layer_norm_mlp(rng, shapes, out: Dict[str, np.ndarray]) -> None:
    # LayerNormMLP (acme/tf/networks/continuous.py:26-28, 55-65): VarianceScaling(
    # distribution='uniform', mode='fan_out', scale=0.333) weights, zero biases, unit
    # LayerNorm scale, zero offset.
    for name, shape in shapes:
        if name.endswith("/w"):
            out[name] = _variance_scaling_uniform(rng, shape, 0.333, shape[-1])
        elif name.endswith("/scale"):
            out[name] = np.ones(shape, np.float32)
        else:
            out[name] = np.zeros(shape, np.float32)


@dataclasses.dataclass(frozen=True)
class LayerNormMLPPolicy:
    """snt.Sequential([LayerNormMLP(sizes, activate_final=True),
    NearZeroInitializedLinear(act_dim), TanhToSpec(action_spec)])
    (examples/control_suite/run_d4pg.py:69-73)."""

    obs_dim: int
    act_dim: int
    layer_sizes: Tuple[int, ...] = (256, 256, 256)
    action_min: Tuple[float, ...] = ()
    action_max: Tuple[float, ...] = ()

    def __init__(self, obs_dim: int, act_dim: int, layer_sizes: Sequence[int] = (256, 256, 256),
                 action_min=-1.0, action_max=1.0):
        object.__setattr__(self, "obs_dim", int(obs_dim))
        object.__setattr__(self, "act_dim", int(act_dim))
        object.__setattr__(self, "layer_sizes", tuple(int(s) for s in layer_sizes))
        lo = np.broadcast_to(np.asarray(action_min, np.float32), (act_dim,))
        hi = np.broadcast_to(np.asarray(action_max, np.float32), (act_dim,))
        object.__setattr__(self, "action_min", tuple(float(x) for x in lo))
        object.__setattr__(self, "action_max", tuple(float(x) for x in hi))

    def tensor_shapes(self):
        s = list(self.layer_sizes)
        return _layer_norm_mlp_shapes("policy", self.obs_dim, s) + [
            ("policy/near_zero_initialized_linear/w", (s[-1], self.act_dim)),
            ("policy/near_zero_initialized_linear/b", (self.act_dim,))]

    def init(self, seed: int = 0) -> Dict[str, np.ndarray]:
        rng = np.random.default_rng(seed)
        out: Dict[str, np.ndarray] = {}
        shapes = self.tensor_shapes()
        _init_layer_norm_mlp(rng, shapes[:-2], out)
        # NearZeroInitializedLinear: VarianceScaling(1e-4) = truncated normal, fan_in
        # (continuous.py:30-35); stddev corrected for the 2-sigma truncation.
        (wn, ws), (bn, bs) = shapes[-2:]
        out[wn] = truncated_normal(rng, ws, np.sqrt(1e-4 / ws[0]) / 0.87962566103423978)
        out[bn] = np.zeros(bs, np.float32)
        return out


@dataclasses.dataclass(frozen=True)
class DistributionalCritic:
    """snt.Sequential([CriticMultiplexer(), LayerNormMLP(sizes, activate_final=True),
    DiscreteValuedHead(vmin, vmax, num_atoms)]) (examples/control_suite/run_d4pg.py:76-81)."""

    obs_dim: int
    act_dim: int
    layer_sizes: Tuple[int, ...] = (512, 512, 256)
    vmin: float = -150.0
    vmax: float = 150.0
    num_atoms: int = 51

    def __init__(self, obs_dim: int, act_dim: int, layer_sizes: Sequence[int] = (512, 512, 256),
                 vmin: float = -150.0, vmax: float = 150.0, num_atoms: int = 51):
        object.__setattr__(self, "obs_dim", int(obs_dim))
        object.__setattr__(self, "act_dim", int(act_dim))
        object.__setattr__(self, "layer_sizes", tuple(int(s) for s in layer_sizes))
        object.__setattr__(self, "vmin", float(vmin))
        object.__setattr__(self, "vmax", float(vmax))
        object.__setattr__(self, "num_atoms", int(num_atoms))

    def tensor_shapes(self):
        s = list(self.layer_sizes)
        return _layer_norm_mlp_shapes("critic", self.obs_dim + self.act_dim, s) + [
            ("critic/discrete_valued_head/linear/w", (s[-1], self.num_atoms)),
            ("critic/discrete_valued_head/linear/b", (self.num_atoms,))]

    def init(self, seed: int = 0) -> Dict[str, np.ndarray]:
        rng = np.random.default_rng(seed)
        out: Dict[str, np.ndarray] = {}
        shapes = self.tensor_shapes()
        _init_layer_norm_mlp(rng, shapes[:-2], out)
        # DiscreteValuedHead's snt.Linear default: TruncatedNormal(1 / sqrt(fan_in)).
        (wn, ws), (bn, bs) = shapes[-2:]
        out[wn] = truncated_normal(rng, ws, 1.0 / np.sqrt(ws[0]))
        out[bn] = np.zeros(bs, np.float32)
        return out

    @property
    def values(self) -> np.ndarray:
        step = (self.vmax - self.vmin) / (self.num_atoms - 1)
        return (self.vmin + np.arange(self.num_atoms) * step).astype(np.float32)


def make_d4pg_networks(obs_dim: int, action_spec, policy_layer_sizes=(256, 256, 256),
                       critic_layer_sizes=(512, 512, 256), vmin: float = -150.0,
                       vmax: float = 150.0, num_atoms: int = 51) -> Dict[str, object]:
    """make_networks of examples/control_suite/run_d4pg.py:53-88 (observation network =
    identity; tf2_utils.batch_concat of a flat observation)."""
    act_dim = int(np.prod(action_spec.shape))
    return {
        "policy": LayerNormMLPPolicy(obs_dim, act_dim, policy_layer_sizes,
                                     action_spec.minimum, action_spec.maximum),
        "critic": DistributionalCritic(obs_dim, act_dim, critic_layer_sizes, vmin, vmax,
                                       num_atoms),
        "observation": "identity",
    }


# ------------------------------------------------------------------ IMPALA (Atari)


class LSTMState(NamedTuple):
    """snt.LSTMState: the core state carried by the IMPALA actor and stored in extras."""
    hidden: np.ndarray
    cell: np.ndarray


@dataclasses.dataclass(frozen=True)
class IMPALAAtariNetwork:
    """IMPALAAtariNetwork (acme/tf/networks/atari.py:115-144): OAREmbedding(AtariTorso) ->
    snt.LSTM(lstm_size) -> Linear(head_size) -> ReLU -> PolicyValueHead(num_actions).
    torso="flat" replaces the AtariTorso by the identity over a float observation vector
    of obs_dim features (small configurations and tests)."""

    num_actions: int
    lstm_size: int = 256
    head_size: int = 256
    torso: str = "atari"
    obs_dim: int = 0

    @property
    def feat(self) -> int:
        return 7744 if self.torso == "atari" else self.obs_dim

    @property
    def obs_dtype(self) -> str:
        return "uint8" if self.torso == "atari" else "float32"

    def tensor_shapes(self):
        H, H2, A = self.lstm_size, self.head_size, self.num_actions
        pre = "impala_atari_network"
        out = []
        if self.torso == "atari":
            out += [(f"{pre}/atari_torso/conv2_d/w", (8, 8, 4, 32)),
                    (f"{pre}/atari_torso/conv2_d/b", (32,)),
                    (f"{pre}/atari_torso/conv2_d_1/w", (4, 4, 32, 64)),
                    (f"{pre}/atari_torso/conv2_d_1/b", (64,)),
                    (f"{pre}/atari_torso/conv2_d_2/w", (3, 3, 64, 64)),
                    (f"{pre}/atari_torso/conv2_d_2/b", (64,))]
        D = self.feat + A + 1
        out += [(f"{pre}/lstm/w_i", (D, 4 * H)), (f"{pre}/lstm/w_h", (H, 4 * H)),
                (f"{pre}/lstm/b", (4 * H,)), (f"{pre}/linear/w", (H, H2)),
                (f"{pre}/linear/b", (H2,)), (f"{pre}/policy_value/w", (H2, A + 1)),
                (f"{pre}/policy_value/b", (A + 1,))]
        return out

    def init(self, seed: int = 0) -> Dict[str, np.ndarray]:
        """Sonnet defaults: conv / linear TruncatedNormal(1/sqrt(fan_in)), zero biases;
        snt.LSTM w_i ~ TruncatedNormal(1/sqrt(input)), w_h ~ TruncatedNormal(1/sqrt(H)),
        bias zero with forget_bias 1.0 folded into the forget-gate slice."""
        rng = np.random.default_rng(seed)
        out = {}
        H = self.lstm_size
        for name, shape in self.tensor_shapes():
            if name.endswith("lstm/b"):
                b = np.zeros(shape, np.float32)
                b[H:2 * H] = 1.0
                out[name] = b
            elif name.endswith("/b"):
                out[name] = np.zeros(shape, np.float32)
            else:
                fan_in = int(np.prod(shape[:-1]))
                out[name] = truncated_normal(rng, shape, 1.0 / np.sqrt(fan_in))
        return out

    def initial_state(self, batch_size: int) -> LSTMState:
        z = np.zeros((batch_size, self.lstm_size), np.float32)
        return LSTMState(z, z.copy())


# ------------------------------------------------------------------ R2D2 (Atari)


@dataclasses.dataclass(frozen=True)
class R2D2AtariNetwork:
    """R2D2AtariNetwork (acme/tf/networks/atari.py:72-112): OAREmbedding(AtariTorso) ->
    snt.LSTM(lstm_size) -> DuellingMLP(num_actions, [head_size]) (duelling.py:26-59).  The
    duelling MLP's two first layers are one fused [lstm_size, 2 head_size] tensor
    [value | advantage] (as DQNAtariNetwork's).  torso="flat": the identity over a float
    observation vector of obs_dim features."""

    num_actions: int
    lstm_size: int = 512
    head_size: int = 512
    torso: str = "atari"
    obs_dim: int = 0

    @property
    def feat(self) -> int:
        return 7744 if self.torso == "atari" else self.obs_dim

    @property
    def obs_dtype(self) -> str:
        return "uint8" if self.torso == "atari" else "float32"

    def tensor_shapes(self):
        H, H2, A = self.lstm_size, self.head_size, self.num_actions
        pre = "r2d2_atari_network"
        out = []
        if self.torso == "atari":
            out += [(f"{pre}/atari_torso/conv2_d/w", (8, 8, 4, 32)),
                    (f"{pre}/atari_torso/conv2_d/b", (32,)),
                    (f"{pre}/atari_torso/conv2_d_1/w", (4, 4, 32, 64)),
                    (f"{pre}/atari_torso/conv2_d_1/b", (64,)),
                    (f"{pre}/atari_torso/conv2_d_2/w", (3, 3, 64, 64)),
                    (f"{pre}/atari_torso/conv2_d_2/b", (64,))]
        D = self.feat + A + 1
        q = f"{pre}/duelling_q_network"
        out += [(f"{pre}/lstm/w_i", (D, 4 * H)), (f"{pre}/lstm/w_h", (H, 4 * H)),
                (f"{pre}/lstm/b", (4 * H,)),
                (f"{q}/hidden/w", (H, 2 * H2)), (f"{q}/hidden/b", (2 * H2,)),
                (f"{q}/mlp/linear_1/w", (H2, 1)), (f"{q}/mlp/linear_1/b", (1,)),
                (f"{q}/mlp_1/linear_1/w", (H2, A)), (f"{q}/mlp_1/linear_1/b", (A,))]
        return out

    init = IMPALAAtariNetwork.init
    initial_state = IMPALAAtariNetwork.initial_state
