"""ctypes binding of libacme_hip.so (the C ABI declared in include/acme_hip.h).

The product path has no CPU fallback: if the library is missing or cannot be loaded
on a GPU machine, `lib()` raises.  torch is imported first so that the HIP runtime the
library links against (SONAME libamdhip64.so.7) resolves to the one torch already
loaded — one runtime, one device context, shared pointers and streams.
"""

from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must load the HIP runtime before libacme_hip.so)

_HERE = os.path.dirname(os.path.abspath(__file__))
# ACME_LIB_PATH: an alternative build (experiments); the in-tree library by default.
LIB_PATH = os.environ.get("ACME_LIB_PATH") or os.path.join(_HERE, "libacme_hip.so")

ACME_OK = 0
ACME_ERR_INVALID = -1
ACME_ERR_HIP = -2
ACME_ERR_EMPTY = -3
ACME_ERR_OOM = -4

SEMANTICS_TF = 0
SEMANTICS_JAX = 1

MATMUL_F32 = 0
MATMUL_X6 = 1

MAX_FIELDS = 16
MAX_MLP_LAYERS = 8
D4PG_MAX_LAYERS = 4
D4PG_MAX_ACT = 16
D4PG_MAX_ATOMS = 64

c_i32, c_i64, c_u64, c_f32, c_f64, c_vp = (ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64,
                                          ctypes.c_float, ctypes.c_double, ctypes.c_void_p)


class ReplayConfig(ctypes.Structure):
    _fields_ = [("capacity", c_i64), ("sampler", c_i32), ("num_fields", c_i32),
                ("priority_exponent", c_f64), ("seed", c_u64),
                ("field_bytes", c_i64 * MAX_FIELDS)]


class DQNConfig(ctypes.Structure):
    _fields_ = [("network", c_i32), ("obs_dtype", c_i32), ("num_actions", c_i32),
                ("max_batch", c_i32), ("obs_dim", c_i32), ("num_hidden", c_i32),
                ("hidden", c_i32 * MAX_MLP_LAYERS), ("discount", c_f32),
                ("importance_sampling_exponent", c_f32), ("learning_rate", c_f32),
                ("huber_loss_parameter", c_f32), ("adam_beta1", c_f32), ("adam_beta2", c_f32),
                ("adam_epsilon", c_f32), ("target_update_period", c_i32),
                ("max_abs_reward", c_f32), ("semantics", c_i32)]


class TransitionBatch(ctypes.Structure):
    _fields_ = [("o_tm1", c_vp), ("a_tm1", c_vp), ("r_t", c_vp), ("d_t", c_vp), ("o_t", c_vp),
                ("probabilities", c_vp), ("batch", c_i64), ("global_min_probability", c_vp),
                ("mean_over", c_i64), ("obs_f16", c_vp), ("inputs_event", c_vp)]


class DQNOutputs(ctypes.Structure):
    _fields_ = [("loss", c_vp), ("td_error", c_vp), ("priorities", c_vp), ("q_tm1", c_vp)]


class D4PGConfig(ctypes.Structure):
    _fields_ = [("obs_dim", c_i32), ("act_dim", c_i32), ("max_batch", c_i32),
                ("num_policy_layers", c_i32), ("policy_sizes", c_i32 * D4PG_MAX_LAYERS),
                ("num_critic_layers", c_i32), ("critic_sizes", c_i32 * D4PG_MAX_LAYERS),
                ("num_atoms", c_i32), ("vmin", c_f32), ("vmax", c_f32),
                ("action_min", c_f32 * D4PG_MAX_ACT), ("action_max", c_f32 * D4PG_MAX_ACT),
                ("discount", c_f32), ("target_update_period", c_i32),
                ("policy_learning_rate", c_f32), ("critic_learning_rate", c_f32),
                ("adam_beta1", c_f32), ("adam_beta2", c_f32), ("adam_epsilon", c_f32),
                ("clipping", c_i32), ("layer_norm_epsilon", c_f32)]


class D4PGBatch(ctypes.Structure):
    _fields_ = [("o_tm1", c_vp), ("a_tm1", c_vp), ("r_t", c_vp), ("d_t", c_vp), ("o_t", c_vp),
                ("batch", c_i64)]


class D4PGOutputs(ctypes.Structure):
    _fields_ = [("critic_loss", c_vp), ("policy_loss", c_vp)]


IMPALA_TORSO_ATARI = 0
IMPALA_TORSO_FLAT = 1


class IMPALAConfig(ctypes.Structure):
    _fields_ = [("torso", c_i32), ("obs_dim", c_i32), ("num_actions", c_i32),
                ("max_batch", c_i32), ("max_sequence_length", c_i32), ("lstm_size", c_i32),
                ("head_size", c_i32), ("discount", c_f32), ("entropy_cost", c_f32),
                ("baseline_cost", c_f32), ("max_abs_reward", c_f32),
                ("max_gradient_norm", c_f32), ("learning_rate", c_f32), ("adam_beta1", c_f32),
                ("adam_beta2", c_f32), ("adam_epsilon", c_f32), ("semantics", c_i32)]


class R2D2Config(ctypes.Structure):
    _fields_ = [("torso", c_i32), ("obs_dim", c_i32), ("num_actions", c_i32),
                ("max_batch", c_i32), ("max_sequence_length", c_i32), ("burn_in_length", c_i32),
                ("lstm_size", c_i32), ("head_size", c_i32), ("n_step", c_i32),
                ("store_lstm_state", c_i32), ("target_update_period", c_i32),
                ("reserved", c_i32), ("max_replay_size", c_i64),
                ("max_priority_weight", ctypes.c_double),
                ("importance_sampling_exponent", ctypes.c_double), ("discount", c_f32),
                ("learning_rate", c_f32), ("adam_beta1", c_f32), ("adam_beta2", c_f32),
                ("adam_epsilon", c_f32)]


class R2D2Outputs(ctypes.Structure):
    _fields_ = [("loss", c_vp), ("errors", c_vp), ("priorities", c_vp)]


class SequenceBatch(ctypes.Structure):
    _fields_ = [("observation", c_vp), ("prev_action", c_vp), ("prev_reward", c_vp),
                ("action", c_vp), ("reward", c_vp), ("discount", c_vp),
                ("behaviour_logits", c_vp), ("h0", c_vp), ("c0", c_vp),
                ("state_stride", c_i64), ("batch", c_i64), ("sequence_length", c_i64)]


_SIGS = {
    "acme_last_error": (ctypes.c_char_p, []),
    "acme_tune_set": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int32]),
    "acme_version": (ctypes.c_char_p, []),
    "acme_target_arch": (ctypes.c_char_p, []),
    "acme_set_matmul_engine": (c_i32, [c_i32]),
    "acme_matmul_engine": (c_i32, []),
    "acme_dense_forward": (c_i32, [c_vp, c_i64, c_i64, c_vp, c_vp, c_i64, c_i32, c_vp, c_vp]),
    "acme_dense_forward_staged": (c_i32, [c_vp, c_i64, c_i64, c_vp, c_vp, c_i64, c_i32, c_vp,
                                          c_i32, c_i32, c_i32, c_vp]),
    "acme_replay_create": (c_i32, [ctypes.POINTER(ReplayConfig), ctypes.POINTER(c_vp)]),
    "acme_replay_destroy": (c_i32, [c_vp]),
    "acme_replay_insert": (c_i32, [c_vp, ctypes.POINTER(c_vp), c_i64, c_vp, c_i32, c_vp, c_vp]),
    "acme_replay_stage_capacity": (c_i64, [c_vp]),
    "acme_replay_stage": (c_i32, [c_vp, c_i64, ctypes.POINTER(c_vp)]),
    "acme_replay_commit": (c_i32, [c_vp, c_i64, c_vp, c_vp, c_vp]),
    "acme_replay_sync_inserts": (c_i32, [c_vp]),
    "acme_host_register": (c_i32, [c_vp, c_i64]),
    "acme_event_create": (c_i32, [ctypes.POINTER(c_vp)]),
    "acme_event_destroy": (c_i32, [c_vp]),
    "acme_event_record": (c_i32, [c_vp, c_vp]),
    "acme_stream_wait_event": (c_i32, [c_vp, c_vp]),
    "acme_event_query": (c_i32, [c_vp]),
    "acme_event_synchronize": (c_i32, [c_vp]),
    "acme_host_unregister": (c_i32, [c_vp]),
    "acme_nstep_writer_create": (c_i32, [c_vp, c_i32, c_f32, c_i64, c_i64, c_i64, c_vp]),
    "acme_nstep_writer_destroy": (c_i32, [c_vp]),
    "acme_nstep_writer_start": (c_i32, [c_vp, c_vp]),
    "acme_nstep_writer_add": (c_i32, [c_vp, c_vp, c_f32, c_f32, c_vp, c_i32, c_f64]),
    "acme_nstep_writer_flush": (c_i32, [c_vp]),
    "acme_nstep_writer_reset": (c_i32, [c_vp]),
    "acme_nstep_writer_pending": (c_i64, [c_vp]),
    "acme_replay_fill_synthetic": (c_i32, [c_vp, c_i64, c_i32, c_i32, c_u64, c_vp]),
    "acme_replay_sample": (c_i32, [c_vp, c_i64, c_u64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "acme_replay_gather": (c_i32, [c_vp, c_vp, c_i64, ctypes.POINTER(c_vp), c_vp]),
    "acme_replay_total": (c_i32, [c_vp, c_vp, c_vp]),
    "acme_replay_sample_share": (c_i32, [c_vp, c_i64, c_u64, c_f64, c_vp, c_vp, c_vp, c_vp, c_vp,
                                         ctypes.POINTER(c_vp), c_vp]),
    "acme_replay_sample_share_frames": (c_i32, [c_vp, c_i64, c_u64, c_f64, c_vp, c_vp, c_vp, c_vp,
                                                c_vp, ctypes.POINTER(c_vp), c_vp, c_vp]),
    "acme_replay_sample_gather": (c_i32, [c_vp, c_i64, c_u64, c_vp, c_vp, c_vp, c_vp, c_vp,
                                          ctypes.POINTER(c_vp), c_vp]),
    "acme_replay_sample_gather_frames": (c_i32, [c_vp, c_i64, c_u64, c_vp, c_vp, c_vp, c_vp,
                                                 c_vp, ctypes.POINTER(c_vp), c_vp, c_vp]),
    "acme_replay_pipe_open": (c_i32, [c_vp, ctypes.POINTER(c_i32)]),
    "acme_replay_pipe_close": (c_i32, [c_vp, c_i32]),
    "acme_replay_pipe_flush": (c_i32, [c_vp, c_i32]),
    "acme_replay_sample_gather_pipe": (c_i32, [c_vp, c_i32, c_i64, c_u64, c_vp, c_vp, c_vp, c_vp,
                                               c_vp, ctypes.POINTER(c_vp), c_vp]),
    "acme_r2d2_priorities": (c_i32, [c_vp, c_i32, c_i32, ctypes.c_double, c_vp, c_vp]),
    "acme_r2d2_importance_weights": (c_i32, [c_vp, c_i32, c_i64, ctypes.c_double, c_vp, c_vp]),
    "acme_frames_expand": (c_i32, [c_vp, c_i64, c_i64, c_i32, c_vp, c_i64, c_vp, c_vp]),
    "acme_replay_update_priorities": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_vp]),
    "acme_replay_update_priorities_gated": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_vp, c_vp]),
    "acme_replay_size": (c_i64, [c_vp]),
    "acme_replay_capacity": (c_i64, [c_vp]),
    "acme_replay_debug_leaves": (c_i32, [c_vp, ctypes.POINTER(c_vp), ctypes.POINTER(c_vp),
                                         ctypes.POINTER(c_vp)]),
    "acme_replay_storage": (c_i32, [c_vp, c_i32, ctypes.POINTER(c_vp)]),
    "acme_replay_inserted": (c_i64, [c_vp]),
    "acme_replay_restore": (c_i32, [c_vp, c_i64, c_vp]),
    "acme_dqn_create": (c_i32, [ctypes.POINTER(DQNConfig), ctypes.POINTER(c_vp)]),
    "acme_dqn_destroy": (c_i32, [c_vp]),
    "acme_dqn_num_params": (c_i64, [c_vp]),
    "acme_dqn_flat_size": (c_i64, [c_vp]),
    "acme_dqn_num_tensors": (c_i32, [c_vp]),
    "acme_dqn_tensor_info": (c_i32, [c_vp, c_i32, ctypes.POINTER(c_i64), ctypes.POINTER(c_i64),
                                     ctypes.POINTER(c_i32), ctypes.POINTER(c_i64),
                                     ctypes.POINTER(ctypes.c_char_p)]),
    "acme_dqn_bind": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "acme_dqn_params_changed": (c_i32, [c_vp]),
    "acme_dqn_plane_overflow": (c_i32, [c_vp, ctypes.POINTER(c_i32), c_i32]),
    "acme_dqn_skipped_steps": (c_i64, [c_vp]),
    "acme_dqn_guard_state": (c_i32, [c_vp, ctypes.POINTER(c_i64)]),
    "acme_dqn_verdict_timeouts": (c_i32, [c_vp, ctypes.POINTER(c_i64)]),
    "acme_dqn_set_applied_steps": (c_i32, [c_vp, c_i64]),
    "acme_dqn_skip_word": (c_i32, [c_vp, ctypes.POINTER(c_vp)]),
    "acme_dqn_set_reissue": (c_i32, [c_vp, c_i32]),
    "acme_dqn_verdicts_issued": (c_i64, [c_vp]),
    "acme_dqn_step_verdict": (c_i32, [c_vp, c_i64, ctypes.POINTER(c_i32)]),
    "acme_dqn_set_data_parallel_gate": (c_i32, [c_vp, c_i32]),
    "acme_dqn_dense_grads_ready": (c_i32, [c_vp, c_vp]),
    "acme_dqn_dp_init": (c_i32, [c_vp, c_vp, c_i32]),
    "acme_dqn_dp_step": (c_i32, [c_vp, ctypes.POINTER(TransitionBatch), ctypes.POINTER(DQNOutputs),
                                 c_vp]),
    "acme_nccl_get_unique_id": (c_i32, [c_vp]),
    "acme_nccl_comm_init": (c_i32, [c_vp, c_i32, c_i32, ctypes.POINTER(c_vp)]),
    "acme_nccl_comm_destroy": (c_i32, [c_vp]),
    "acme_dqn_scale_state": (c_i32, [c_vp, c_vp, c_i32, ctypes.POINTER(c_i32)]),
    "acme_dqn_set_scale_state": (c_i32, [c_vp, c_vp, c_i32]),
    "acme_dqn_forward_backward": (c_i32, [c_vp, ctypes.POINTER(TransitionBatch),
                                          ctypes.POINTER(DQNOutputs), c_vp]),
    "acme_dqn_apply": (c_i32, [c_vp, c_vp]),
    "acme_dqn_forward_backward_stage": (c_i32, [c_vp, ctypes.POINTER(TransitionBatch),
                                                ctypes.POINTER(DQNOutputs), c_i32, c_vp]),
    "acme_dqn_grad_split": (c_i32, [c_vp, ctypes.POINTER(c_i64)]),
    "acme_dqn_step": (c_i32, [c_vp, ctypes.POINTER(TransitionBatch), ctypes.POINTER(DQNOutputs),
                              c_vp]),
    "acme_dqn_step_update": (c_i32, [c_vp, ctypes.POINTER(TransitionBatch),
                                     ctypes.POINTER(DQNOutputs), c_vp, c_vp, c_vp, c_vp]),
    "acme_dqn_q_values": (c_i32, [c_vp, c_vp, c_i64, c_i32, c_vp, c_vp]),
    "acme_dqn_num_steps": (c_i64, [c_vp]),
    "acme_dqn_debug_buffer": (c_i32, [c_vp, ctypes.c_char_p, ctypes.POINTER(c_vp),
                                      ctypes.POINTER(c_i64)]),
    "acme_dqn_set_num_steps": (c_i32, [c_vp, c_i64]),
    "acme_min_f64": (c_i32, [c_vp, c_i64, c_vp, c_vp]),
    "acme_r2d2_create": (c_i32, [ctypes.POINTER(R2D2Config), ctypes.POINTER(c_vp)]),
    "acme_r2d2_destroy": (c_i32, [c_vp]),
    "acme_r2d2_flat_size": (c_i64, [c_vp]),
    "acme_r2d2_num_tensors": (c_i32, [c_vp]),
    "acme_r2d2_tensor_info": (c_i32, [c_vp, c_i32, ctypes.POINTER(c_i64), ctypes.POINTER(c_i64),
                                      ctypes.POINTER(c_i32), ctypes.POINTER(c_i64),
                                      ctypes.POINTER(ctypes.c_char_p)]),
    "acme_r2d2_bind": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "acme_r2d2_step": (c_i32, [c_vp, ctypes.POINTER(SequenceBatch), c_vp,
                               ctypes.POINTER(R2D2Outputs), c_vp]),
    "acme_r2d2_params_changed": (c_i32, [c_vp]),
    "acme_r2d2_scale_state": (c_i32, [c_vp, c_vp, c_i32, ctypes.POINTER(c_i32)]),
    "acme_r2d2_set_scale_state": (c_i32, [c_vp, c_vp, c_i32]),
    "acme_r2d2_skipped_steps": (c_i64, [c_vp]),
    "acme_r2d2_guard_state": (c_i32, [c_vp, ctypes.POINTER(c_i64)]),
    "acme_r2d2_skip_word": (c_vp, [c_vp]),
    "acme_r2d2_set_applied_steps": (c_i32, [c_vp, c_i64]),
    "acme_r2d2_num_steps": (c_i64, [c_vp]),
    "acme_r2d2_set_num_steps": (c_i32, [c_vp, c_i64]),
    "acme_r2d2_set_lstm_unroll": (c_i32, [c_vp, c_i32]),
    "acme_r2d2_debug_buffer": (c_i32, [c_vp, ctypes.c_char_p, ctypes.POINTER(c_vp),
                                       ctypes.POINTER(c_i64)]),
    "acme_impala_create": (c_i32, [ctypes.POINTER(IMPALAConfig), ctypes.POINTER(c_vp)]),
    "acme_impala_destroy": (c_i32, [c_vp]),
    "acme_impala_flat_size": (c_i64, [c_vp]),
    "acme_impala_num_tensors": (c_i32, [c_vp]),
    "acme_impala_tensor_info": (c_i32, [c_vp, c_i32, ctypes.POINTER(c_i64), ctypes.POINTER(c_i64),
                                        ctypes.POINTER(c_i32), ctypes.POINTER(c_i64),
                                        ctypes.POINTER(ctypes.c_char_p)]),
    "acme_impala_bind": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp]),
    "acme_impala_params_changed": (c_i32, [c_vp]),
    "acme_impala_step": (c_i32, [c_vp, ctypes.POINTER(SequenceBatch), c_vp, c_vp]),
    "acme_impala_set_lstm_unroll": (c_i32, [c_vp, c_i32]),
    "acme_impala_plane_overflow": (c_i32, [c_vp, ctypes.POINTER(c_i32), c_i32]),
    "acme_impala_skipped_steps": (c_i64, [c_vp]),
    "acme_impala_guard_state": (c_i32, [c_vp, ctypes.POINTER(c_i64)]),
    "acme_impala_set_applied_steps": (c_i32, [c_vp, c_i64]),
    "acme_impala_scale_state": (c_i32, [c_vp, c_vp, c_i32, ctypes.POINTER(c_i32)]),
    "acme_impala_set_scale_state": (c_i32, [c_vp, c_vp, c_i32]),
    "acme_impala_policy_step": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp,
                                        c_vp, c_vp, c_vp]),
    "acme_impala_set_policy_planes": (c_i32, [c_vp, c_i32]),
    "acme_impala_num_steps": (c_i64, [c_vp]),
    "acme_impala_set_num_steps": (c_i32, [c_vp, c_i64]),
    "acme_impala_debug_buffer": (c_i32, [c_vp, ctypes.c_char_p, ctypes.POINTER(c_vp),
                                         ctypes.POINTER(c_i64)]),
    "acme_d4pg_create": (c_i32, [ctypes.POINTER(D4PGConfig), ctypes.POINTER(c_vp)]),
    "acme_d4pg_destroy": (c_i32, [c_vp]),
    "acme_d4pg_flat_size": (c_i64, [c_vp]),
    "acme_d4pg_policy_size": (c_i64, [c_vp]),
    "acme_d4pg_num_tensors": (c_i32, [c_vp]),
    "acme_d4pg_tensor_info": (c_i32, [c_vp, c_i32, ctypes.POINTER(c_i64), ctypes.POINTER(c_i64),
                                      ctypes.POINTER(c_i32), ctypes.POINTER(c_i64),
                                      ctypes.POINTER(ctypes.c_char_p)]),
    "acme_d4pg_bind": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "acme_d4pg_step": (c_i32, [c_vp, ctypes.POINTER(D4PGBatch), ctypes.POINTER(D4PGOutputs),
                               c_vp]),
    "acme_d4pg_policy": (c_i32, [c_vp, c_vp, c_i64, c_i32, c_vp, c_vp]),
    "acme_d4pg_num_steps": (c_i64, [c_vp]),
    "acme_d4pg_set_num_steps": (c_i32, [c_vp, c_i64]),
    "acme_d4pg_debug_buffer": (c_i32, [c_vp, ctypes.c_char_p, ctypes.POINTER(c_vp),
                                       ctypes.POINTER(c_i64)]),
    "acme_profile_enable": (c_i32, [c_i32]),
    "acme_profile_reset": (c_i32, []),
    "acme_profile_num_sections": (c_i32, []),
    "acme_profile_query_peak": (c_i32, [c_i32, ctypes.POINTER(c_f64)]),
    "acme_profile_query": (c_i32, [c_i32, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(c_f64),
                                   ctypes.POINTER(c_i64), ctypes.POINTER(c_f64),
                                   ctypes.POINTER(c_f64)]),
    "acme_adam_update": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, c_f32, c_f32, c_f32, c_f32, c_i64,
                                 c_vp]),
}

EXPORTED_SYMBOLS = tuple(_SIGS)

_lib = None
_lock = threading.Lock()


class AcmeError(RuntimeError):
    pass


def lib() -> ctypes.CDLL:
    """Loads libacme_hip.so (raises if absent: there is no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError(
                    f"{LIB_PATH} not found: run `python -m acme_amd._build` (or "
                    "__graft_entry__.build()) to compile the HIP library for gfx950.")
            L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
            for name, (res, args) in _SIGS.items():
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _lib = L
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc == ACME_OK:
        return
    msg = lib().acme_last_error().decode(errors="replace")
    if what:
        msg = f"{what}: {msg}"
    if rc == ACME_ERR_INVALID:
        raise ValueError(msg)
    if rc == ACME_ERR_OOM:
        raise MemoryError(msg)
    raise AcmeError(msg)


def require_gpu() -> None:
    if not torch.cuda.is_available():
        raise RuntimeError("acme_amd's learner and replay run on an AMD GPU (gfx950); "
                           "no GPU is visible and there is no CPU fallback.")


def stream_ptr(stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


class OrderEvent:
    """A device-scope stream-order event (acme_event_*), used like torch.cuda.Event for
    record / wait / query between streams of one device.  torch's events fence at system
    scope, which writes back and invalidates the caches: ~6 us of the recording stream's
    time on MI355X.  Completion only: the host must not read device-written memory on the
    strength of query() / synchronize()."""

    def __init__(self):
        self._lib = lib()
        h = ctypes.c_void_p()
        check(self._lib.acme_event_create(ctypes.byref(h)), "event create")
        self._h = h

    def record(self, stream=None) -> None:
        check(self._lib.acme_event_record(self._h, stream_ptr(stream)), "event record")

    def wait(self, stream=None) -> None:
        check(self._lib.acme_stream_wait_event(stream_ptr(stream), self._h), "event wait")

    def query(self) -> bool:
        rc = self._lib.acme_event_query(self._h)
        if rc < 0:
            check(rc, "event query")
        return rc == 1

    def synchronize(self) -> None:
        check(self._lib.acme_event_synchronize(self._h), "event synchronize")

    @property
    def handle(self) -> int:
        """The raw hipEvent_t (for C entry points that take an event)."""
        return int(self._h.value)

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h is not None and h.value:
            try:
                self._lib.acme_event_destroy(h)
            except Exception:  # interpreter shutdown
                pass


def ptr(t) -> int:
    return 0 if t is None else int(t.data_ptr())


_PROFILING = False


def set_profiling(on: bool) -> None:
    """Turns the library's section profiler on/off (acme_profile_enable).  While it is on,
    Python-side producers (the prefetching dataset) also issue on the caller's stream, so
    every profiled kernel runs alone."""
    global _PROFILING
    check(lib().acme_profile_enable(1 if on else 0), "profile enable")
    _PROFILING = bool(on)


def profiling() -> bool:
    return _PROFILING
