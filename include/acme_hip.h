/*
 * acme_hip.h — C ABI of the MI355X-native Acme learner core (libacme_hip.so).
 *
 * Plain C types only (no torch / HIP types in the signatures): device buffers are
 * `void*` device pointers, streams are `void*` (a hipStream_t, NULL = default).
 * Every function returns ACME_OK (0) or a negative acme_status and leaves a message
 * in a thread-local buffer (acme_last_error()).
 *
 * What each entry point replaces in the reference (tmtlakmal/acme @ 2025-02-05):
 *
 *   acme_replay_*       the Reverb table/server the agents construct
 *                       (acme/agents/tf/dqn/agent.py:95-102 Prioritized + Fifo + MinSize;
 *                        acme/agents/tf/d4pg/agent.py:96-102 Uniform) and
 *     _insert           reverb.Writer.append + create_item, driven by
 *                       NStepTransitionAdder._write (acme/adders/reverb/transition.py:374-378)
 *     _sample/_gather   reverb.ReplayDataset + tf.data batch (acme/datasets/reverb.py:93-139)
 *                       producing ReplaySample(info=SampleInfo(key, probability,
 *                       table_size, priority), data=...)  (acme/testing/fakes.py:249-260)
 *     _update_priorities reverb.TFClient.update_priorities
 *                       (acme/agents/tf/dqn/learning.py:151-154) and
 *                       Client.mutate_priorities (acme/agents/jax/dqn/learning.py:131-134)
 *   acme_dqn_*          DQNLearner._step (acme/agents/tf/dqn/learning.py:112-168):
 *                       three Q forwards, double-Q n-step TD, Huber, f64 IS weights,
 *                       backward, snt.Adam, post-step periodic target copy.
 *
 * Threading: one learner stream; acme_replay_insert / _stage / _commit may be called from
 * actor threads (internal mutex).  Host inserts run on the table's own side stream; the
 * table orders them against every stream that samples, gathers or updates priorities
 * (see acme_replay_insert), with no per-step event on the learner stream.
 */
#ifndef ACME_HIP_H_
#define ACME_HIP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum acme_status {
  ACME_OK = 0,
  ACME_ERR_INVALID = -1, /* bad argument -> ValueError */
  ACME_ERR_HIP = -2,     /* HIP runtime failure -> RuntimeError */
  ACME_ERR_EMPTY = -3,   /* sampling below the table's min size -> RuntimeError */
  ACME_ERR_OOM = -4      /* device allocation failure -> MemoryError */
} acme_status;

const char* acme_last_error(void);

/* Tuning / experiment switch `key` (the ACME_V_<key> environment variable, read once per
 * process) set to `value` for the rest of the process; 0 restores the default.  Not part
 * of the reference interface: kernel-variant selection for tests and sweeps. */
int acme_tune_set(const char* key, int32_t value);
/* Library version string (build id). */
const char* acme_version(void);
/* Name of the GPU the library was built for ("gfx950"). */
const char* acme_target_arch(void);

/* Stream-order events between streams of one device (hipEventDisableTiming |
 * hipEventDisableSystemFence): the record is a device-scope release, so it costs the
 * recording stream no cache writeback; query / synchronize report completion only (the
 * host must not read device-written memory on their strength).  Used by the dataset's
 * prefetch ordering; the learners create theirs internally.  query: 1 complete, 0 pending. */
int acme_event_create(void** ev);
int acme_event_destroy(void* ev);
int acme_event_record(void* ev, void* stream);
int acme_stream_wait_event(void* stream, void* ev);
int acme_event_query(void* ev);
int acme_event_synchronize(void* ev);

/* Matmul engine of the learners' dense layers (process-wide; default from the
 * ACME_MATMUL environment variable, "x6" unless it says "f32"):
 *   ACME_MATMUL_X6  f32 operands split exactly into three bf16 planes, six bf16 MFMAs
 *                   per 16-deep k step, f32 accumulation: f32-equivalent error
 *                   (csrc/gemm_x6.h), 2.7x the MFMA rate of
 *   ACME_MATMUL_F32 v_mfma_f32_32x32x2_f32 (exact f32 products, csrc/gemm.h). */
enum { ACME_MATMUL_F32 = 0, ACME_MATMUL_X6 = 1 };
int acme_set_matmul_engine(int32_t engine);
int32_t acme_matmul_engine(void);
/* One dense layer on the current engine: y[rows, out] = act(x[rows, in] @ w[in, out] + b)
 * (act: 0 none, 1 relu, 2 elu, 3 tanh); in and out multiples of 4.  Device pointers. */
int acme_dense_forward(const float* x, int64_t rows, int64_t in, const float* w, const float* b,
                       int64_t out, int32_t act, float* y, void* stream);
/* The same layer on the staged f32 engine (csrc/gemm.h, 32 x 32 tiles of one wave per k-group)
 * at stage depth bk and wk k-groups, (bk, wk) in {(16, 8), (32, 4), (32, 8), (16, 16)};
 * multi != 0 runs it through the multi-problem kernel the D4PG backward launches use
 * (gemm_f32_multi_kernel).  Tests of the engine's configurations. */
int acme_dense_forward_staged(const float* x, int64_t rows, int64_t in, const float* w,
                              const float* b, int64_t out, int32_t act, float* y, int32_t bk,
                              int32_t wk, int32_t multi, void* stream);

/* ------------------------------------------------------------------ replay -- */

#define ACME_MAX_FIELDS 16

enum { ACME_SAMPLER_UNIFORM = 0, ACME_SAMPLER_PRIORITIZED = 1 };

typedef struct acme_replay_config {
  int64_t capacity;          /* max_size of the table (FIFO eviction beyond it)     */
  int32_t sampler;           /* ACME_SAMPLER_*                                      */
  int32_t num_fields;        /* number of flattened data fields per item            */
  double priority_exponent;  /* Prioritized(alpha); ignored for uniform             */
  uint64_t seed;             /* Philox key for sampling                             */
  int64_t field_bytes[ACME_MAX_FIELDS]; /* bytes per item of each field (mult. of 4) */
} acme_replay_config;

typedef struct acme_replay acme_replay;

int acme_replay_create(const acme_replay_config* cfg, acme_replay** out);
int acme_replay_destroy(acme_replay* r);

/* Insert n items (replaces Writer.append + create_item, adders/reverb/transition.py:119-165,
 * one item per environment step; Reverb's insert RPC).  fields[f] points at
 * n * field_bytes[f] contiguous bytes, on the host when src_on_device == 0, else on the
 * device.  priorities: n raw priorities (host, NULL = 1.0).  out_keys (host, optional): the
 * keys assigned.  Items go to ring slots (insert_count + i) % capacity (Fifo remover).
 * Host rows are packed into the table's pinned staging ring, uploaded (hipMemcpyAsync on
 * an upload stream, unordered against readers) into the chunk's device mirror, and landed
 * into the ring slots by one scatter launch on the table's side stream, followed by the
 * tree refresh; the call returns without waiting.  The landing is ordered after the upload,
 * the work already issued on `stream` and on every stream that has used the table; every
 * later sample / gather / update_priorities (any stream) is ordered after it, so a reader
 * waits for the landing, not for the PCIe transfer.  Device rows are copied on `stream`
 * itself. */
int acme_replay_insert(acme_replay* r, const void* const* fields, int64_t n,
                       const double* priorities, int32_t src_on_device,
                       uint64_t* out_keys, void* stream);

/* Zero-copy form of the host insert: acme_replay_stage hands out pinned host pointers
 * field_ptrs[f] with room for n <= acme_replay_stage_capacity(r) items (blocking only while
 * that staging chunk's previous copies are in flight); the caller writes the rows there
 * and acme_replay_commit(r, m <= n, ...) issues them exactly as acme_replay_insert does. */
int64_t acme_replay_stage_capacity(acme_replay* r);
int acme_replay_stage(acme_replay* r, int64_t n, void** field_ptrs);
int acme_replay_commit(acme_replay* r, int64_t n, const double* priorities, uint64_t* out_keys,
                       void* stream);
/* Host wait for every issued insert (tests, checkpoints, shutdown). */
int acme_replay_sync_inserts(acme_replay* r);
/* Page-locks caller memory (hipHostRegister) so copies from it are DMA without staging,
 * e.g. the shared-memory blocks actor processes write observations into; unregister
 * before the memory is unmapped. */
int acme_host_register(void* p, int64_t bytes);
int acme_host_unregister(void* p);

/* N-step transition writer: the native NStepTransitionAdder (acme/adders/reverb/
 * transition.py:119-172; replaces its _write / _write_last + Writer.append / create_item)
 * for a transition table (fields o_tm1, a, f32 R, f32 D, o_t).  The adder passes each
 * environment step's raw fields: _start(first observation) on add_first, _add(action,
 * reward, discount, next observation, last, priority) on add.  The writer keeps the last
 * n_step steps, writes every item the reference writes (window head = oldest step; windows
 * of 1, 2, ... steps at an episode's start; on the last step the drain of shrinking windows)
 * as rows of its own pinned chunk of rows_per_chunk items, and commits a full chunk exactly
 * as acme_replay_commit does (side-stream copies, no host wait).  R and D accumulate in f32
 * in the reference's order.  obs_bytes / action_bytes: payload bytes (<= the field's row
 * bytes; the rest of a row stays zero).  _flush commits the pending rows; _reset (adder.reset
 * without a last step) commits them and drops the window; _pending: rows not yet committed.
 * One thread adds; _flush / _pending may be called from any thread. */
typedef struct acme_nstep_writer acme_nstep_writer;
int acme_nstep_writer_create(acme_replay* r, int32_t n_step, float discount, int64_t obs_bytes,
                             int64_t action_bytes, int64_t rows_per_chunk,
                             acme_nstep_writer** out);
int acme_nstep_writer_destroy(acme_nstep_writer* w);
int acme_nstep_writer_start(acme_nstep_writer* w, const void* observation);
int acme_nstep_writer_add(acme_nstep_writer* w, const void* action, float reward,
                          float discount, const void* next_observation, int32_t last,
                          double priority);
int acme_nstep_writer_flush(acme_nstep_writer* w);
int acme_nstep_writer_reset(acme_nstep_writer* w);
int64_t acme_nstep_writer_pending(acme_nstep_writer* w);

/* Fill n items with synthetic data generated on the device (benchmark/test helper,
 * no host traffic).  layout: 0 = DQN Atari transition (o_tm1 u8, a i32, r f32, d f32,
 * o_t u8), 1 = control transition with f32 fields
 * (o f32, a f32, r f32, d f32, o_t f32; config 3).  All priorities set to 1.0. */
int acme_replay_fill_synthetic(acme_replay* r, int64_t n, int32_t layout,
                               int32_t num_actions, uint64_t seed, void* stream);

/* Draw `batch` items.  Device outputs: slots (i64), keys (u64), probabilities (f64,
 * P(i) = p_i^alpha / sum_j p_j^alpha or 1/size), table_size (i64), priorities (f64).
 * Any output pointer except slots may be NULL.  step_counter selects the Philox
 * counter block, so (seed, step_counter) fully determines the draw. */
int acme_replay_sample(acme_replay* r, int64_t batch, uint64_t step_counter,
                       int64_t* slots, uint64_t* keys, double* probabilities,
                       int64_t* table_size, double* priorities, void* stream);

/* Copy the items at `slots` into batch-major device buffers out_fields[f]
 * (batch * field_bytes[f] bytes each). */
int acme_replay_gather(acme_replay* r, const int64_t* slots, int64_t batch,
                       void* const* out_fields, void* stream);

/* acme_replay_sample then acme_replay_gather as one unit: no insert is committed between
 * the draw and the row copy, so every gathered row is the row of the key reported for it
 * even while actor threads insert (the two separate calls leave that to the caller). */
int acme_replay_sample_gather(acme_replay* r, int64_t batch, uint64_t step_counter,
                              int64_t* slots, uint64_t* keys, double* probabilities,
                              int64_t* table_size, double* priorities, void* const* out_fields,
                              void* stream);

/* acme_replay_sample_gather for the transition layout (two equal uint8 fields, e.g. o_tm1 /
 * o_t) that also writes the exact f16 copy of both fields that the DQN plane path reads
 * (frames_f16: [2 * batch][field_bytes] u16, rows [0, batch) the first field, [batch,
 * 2 * batch) the second; 16-B aligned), in the same launch; pass it to the learner as
 * acme_transition_batch.obs_f16.  Errors for other layouts. */
int acme_replay_sample_gather_frames(acme_replay* r, int64_t batch, uint64_t step_counter,
                                     int64_t* slots, uint64_t* keys, double* probabilities,
                                     int64_t* table_size, double* priorities,
                                     void* const* out_fields, uint16_t* frames_f16,
                                     void* stream);

/* Pipelined sample + gather for a prefetching reader (round 6; the reference's prefetched
 * dataset iterator, acme/datasets/reverb.py:136-137, issues draws ahead of their use).
 * acme_replay_sample_gather_pipe draws a batch exactly as acme_replay_sample_gather (same
 * keys, slots, probabilities and rows) but copies its rows in the pipe's NEXT call, in the
 * same launch as that call's draw, so the draw's dependent tree loads overlap a row copy.
 * A batch's rows are therefore complete only after the following call on its pipe (or
 * acme_replay_pipe_flush); every operation that writes table rows (insert, commit,
 * synthetic fill, acme_replay_storage) issues the pending copies first, so each batch
 * gets the rows of its drawn keys.  A pipe is one reader on one stream; the transition
 * layout only (two equal big fields): other layouts sample + gather at once.
 * acme_replay_pipe_close drops a pending copy (its batch was never handed out). */
int acme_replay_pipe_open(acme_replay* r, int32_t* pipe);
int acme_replay_pipe_close(acme_replay* r, int32_t pipe);
int acme_replay_pipe_flush(acme_replay* r, int32_t pipe);
int acme_replay_sample_gather_pipe(acme_replay* r, int32_t pipe, int64_t batch,
                                   uint64_t step_counter, int64_t* slots, uint64_t* keys,
                                   double* probabilities, int64_t* table_size,
                                   double* priorities, void* const* out_fields, void* stream);

/* Data-parallel global-probability sampling: one table per rank holds a
 * shard of the global replay.  acme_replay_total writes the shard's sampling mass S_r
 * (sum of p^alpha, or the item count for Uniform) to out[0] on the device; the ranks
 * all-gather the masses, allocate the global batch N * B in proportion (n_r / (N B) =
 * S_r / S), and each draws its share n_r from its own shard with
 * acme_replay_sample_share(prob_scale = n_r / (N B)), which reports
 * probability = prob_scale * p^alpha / S_r — the item's marginal probability of being
 * drawn by the global draw, p^alpha / S_global when the shares are proportional — and, when
 * out_fields is non-NULL, gathers the rows as acme_replay_sample_gather does. */
int acme_replay_total(acme_replay* r, double* out, void* stream);
int acme_replay_sample_share(acme_replay* r, int64_t batch, uint64_t step_counter,
                             double prob_scale, int64_t* slots, uint64_t* keys,
                             double* probabilities, int64_t* table_size, double* priorities,
                             void* const* out_fields, void* stream);
/* acme_replay_sample_share with the gather and the f16 frame copy of
 * acme_replay_sample_gather_frames (rows [0, batch) / [batch, 2 * batch) of frames_f16). */
int acme_replay_sample_share_frames(acme_replay* r, int64_t batch, uint64_t step_counter,
                                    double prob_scale, int64_t* slots, uint64_t* keys,
                                    double* probabilities, int64_t* table_size,
                                    double* priorities, void* const* out_fields,
                                    uint16_t* frames_f16, void* stream);

/* Frame-deduplicated observations: rebuild `batch` stacked
 * observations out[b] = stack(frames[idx[b][0..stack-1]], axis=-1) (uint8 HWC, as
 * acme/wrappers/frame_stacking.py:78-83 builds them) from a device frame ring
 * frames[num_frames][frame_bytes]; idx is int32 [batch][stack] on the device.  Replaces the
 * whole-stack storage of adders/reverb/transition.py:147-152 (replay/FrameTable). */
int acme_frames_expand(const uint8_t* frames, int64_t num_frames, int64_t frame_bytes,
                       int32_t stack, const int32_t* idx, int64_t batch, uint8_t* out,
                       void* stream);

/* R2D2 prioritized sequence replay, device arrays:
 * priorities out[b] = (f64)(eta * max_t |errors[t][b]| + (1 - eta) * mean_t |errors[t][b]|)
 *   in f32, errors [T][B] (acme/agents/tf/r2d2/learning.py:230-236, written back at :196-199);
 * importance weights out[b] = (f32)((1 / (N p_b))^beta / max_b (1 / (N p_b))^beta) in f64,
 *   N = max_replay_size (learning.py:178-183; the [T, B] weights are this, per sequence). */
int acme_r2d2_priorities(const float* errors, int32_t T, int32_t B, double eta, double* out,
                         void* stream);
int acme_r2d2_importance_weights(const double* probabilities, int32_t B,
                                 int64_t max_replay_size, double beta, float* out,
                                 void* stream);

/* Set priorities of the items identified by device arrays keys/priorities.  Keys no
 * longer in the table are ignored; for repeated keys the last one wins (Reverb
 * applies updates in order). */
int acme_replay_update_priorities(acme_replay* r, const uint64_t* keys,
                                  const double* priorities, int64_t n, void* stream);
/* The same behind a learner's skip word (acme_dqn_skip_word, a device word): the update
 * is dropped when the word is non-zero when the update runs on the device, i.e. when the
 * learner step that produced the priorities was skipped (plane overflow, below). */
int acme_replay_update_priorities_gated(acme_replay* r, const uint64_t* keys,
                                        const double* priorities, int64_t n,
                                        const uint32_t* skip_word, void* stream);

int64_t acme_replay_size(const acme_replay* r);
int64_t acme_replay_capacity(const acme_replay* r);
/* Device pointer to the sum-tree total (f64) — test/diagnostic use. */
int acme_replay_debug_leaves(const acme_replay* r, const double** leaf_values,
                             const double** raw_priorities, const uint64_t** keys);

/* Table state for checkpoints (optional replay state of acme/tf/savers.py's Checkpointer,
 * SURVEY §8(f) row 2).  acme_replay_storage: device pointer of field f's [capacity, bytes]
 * rows; acme_replay_inserted: items ever inserted (the next key).  acme_replay_restore:
 * after the caller wrote field rows, keys and raw priorities (device pointers from
 * acme_replay_storage / acme_replay_debug_leaves), sets the insert counter and rebuilds the
 * leaves (p^alpha) and every level of the sum tree on `stream`. */
int acme_replay_storage(acme_replay* r, int32_t field, void** out);
int64_t acme_replay_inserted(const acme_replay* r);
int acme_replay_restore(acme_replay* r, int64_t inserted, void* stream);

/* -------------------------------------------------------------------- DQN -- */

enum { ACME_NET_NATURE_DQN = 0, ACME_NET_MLP = 1 };
/* Which reference learner a config restates:
 *   ACME_SEMANTICS_TF   acme/agents/tf/{dqn,impala}/learning.py (snt.Adam, f64 IS weights,
 *                       post-step target copy when num_steps % period == 0);
 *   ACME_SEMANTICS_JAX  acme/agents/jax/{dqn,impala}/learning.py: DQN importance weights in
 *                       f32 before ** beta (dqn/learning.py:94-96), target copy when
 *                       (steps + 1) % period == 0 (:114-119, jax/utils.py:148-154), optix.adam's
 *                       update order; IMPALA optix.chain(clip_by_global_norm, adam)
 *                       (impala/agent.py:98-101). */
enum { ACME_SEMANTICS_TF = 0, ACME_SEMANTICS_JAX = 1 };
enum { ACME_OBS_U8_SCALED = 0, ACME_OBS_F32 = 1 };

#define ACME_MAX_MLP_LAYERS 8

typedef struct acme_dqn_config {
  int32_t network;           /* ACME_NET_*                                          */
  int32_t obs_dtype;         /* ACME_OBS_U8_SCALED: uint8 / 255 (AtariWrapper to_float) */
  int32_t num_actions;
  int32_t max_batch;
  /* Nature DQN: obs is [84, 84, 4] NHWC.  MLP: obs_dim inputs, hidden sizes below
   * (ReLU), final Linear(num_actions) (snt.nets.MLP([..., A])). */
  int32_t obs_dim;
  int32_t num_hidden;
  int32_t hidden[ACME_MAX_MLP_LAYERS];
  float discount;            /* agent discount, applied to the n-step D           */
  float importance_sampling_exponent;
  float learning_rate;
  float huber_loss_parameter;
  float adam_beta1, adam_beta2, adam_epsilon;
  int32_t target_update_period;
  float max_abs_reward;      /* reward clip (TF DQN clips to [-1, 1])               */
  int32_t semantics;         /* ACME_SEMANTICS_TF (default) or ACME_SEMANTICS_JAX    */
} acme_dqn_config;

typedef struct acme_dqn acme_dqn;

int acme_dqn_create(const acme_dqn_config* cfg, acme_dqn** out);
int acme_dqn_destroy(acme_dqn* l);
/* Number of f32 parameters (logical) and of the padded flat buffer the learner uses. */
int64_t acme_dqn_num_params(const acme_dqn* l);
int64_t acme_dqn_flat_size(const acme_dqn* l);
/* Per-tensor layout of the flat buffer: offsets/sizes (in floats) of tensor i. */
int32_t acme_dqn_num_tensors(const acme_dqn* l);
int acme_dqn_tensor_info(const acme_dqn* l, int32_t i, int64_t* offset, int64_t* numel,
                         int32_t* ndim, int64_t* shape4, const char** name);

/* Bind caller-owned device buffers (each acme_dqn_flat_size floats): online params,
 * target params, gradients, Adam first/second moments. */
int acme_dqn_bind(acme_dqn* l, float* params, float* target, float* grads, float* adam_m,
                  float* adam_v);
/* Declares that the caller wrote the bound params / target buffers directly (restore,
 * broadcast, initialisation): the learner's derived copies of them (the scaled f16
 * parameter planes of the uint8 Nature path) are rebuilt, and the activation / gradient
 * plane scales recalibrated, before the next use.  The learner's own updates (step /
 * apply) need no call. */
int acme_dqn_params_changed(acme_dqn* l);
/* Plane-range check of the uint8 Nature path (synchronises the device): *overflow = 1 if
 * some plane tensor written since the last reset exceeded f16's range at its scale (its
 * maximum grew more than 2^8-fold within one step; the results of that step are then not
 * exact), else 0.  reset != 0 clears the flag. */
int acme_dqn_plane_overflow(acme_dqn* l, int32_t* overflow, int32_t reset);
/* Step guard of the plane path (the skip-on-overflow rule of automatic mixed precision):
 * a step in which some f16 plane write overflowed (a tensor's maximum grew more than about
 * 2^8-fold since the previous step) changes no parameter, Adam moment, Adam count, target
 * or replay priority; its end-of-step rescale sets every scale from the step's true maxima,
 * so the next step runs exactly.  Adam's t counts applied updates (acme_dqn_guard_state
 * out4[0] + 1); num_steps (the target period) counts step calls.
 *   acme_dqn_skipped_steps: steps skipped so far among those the device has finished
 *     (a pinned host word the device writes; no synchronisation).
 *   acme_dqn_guard_state: synchronises; out4 = {applied, skipped, last step skipped,
 *     last q_values call overflowed (repeat it: the scales were reset from its maxima)}.
 *   acme_dqn_set_applied_steps: restore Adam's count (checkpoints).
 *   acme_dqn_skip_word: the device word acme_replay_update_priorities_gated reads after
 *     a step (NULL without the plane path).
 *   acme_dqn_set_data_parallel_gate: the ranks skip together: stage 1 writes this rank's
 *     decision into a padding word of the torso gradient bucket [0, grad_split), which the
 *     caller's all-reduce of that bucket combines before acme_dqn_apply (acme_dqn_dp_init
 *     enables it). */
int64_t acme_dqn_skipped_steps(const acme_dqn* l);
int acme_dqn_guard_state(acme_dqn* l, int64_t* out4);
int acme_dqn_set_applied_steps(acme_dqn* l, int64_t n);
int acme_dqn_skip_word(const acme_dqn* l, const uint32_t** out);
int acme_dqn_set_data_parallel_gate(acme_dqn* l, int32_t enable);
/* Re-issue of skipped steps (DQNLearner.step: every call applies one update, as
 * acme/agents/tf/dqn/learning.py:147-161 does).  Every step's verdict gets a sequence number
 * (acme_dqn_verdicts_issued: how many were issued so far) and is published by the device
 * into a pinned 64-entry ring; acme_dqn_step_verdict reads verdict `seq` without a
 * synchronisation: *state = -1 not decided yet, 0 applied, 1 skipped.
 * acme_dqn_set_reissue(l, 1): a skipped step holds every later step skipped (nothing they
 * compute from the un-updated parameters is applied) until the next calibration
 * (acme_dqn_params_changed), so the caller can re-issue the held batches in order; a target
 * copy due on a skipped step is not made (the re-issued step makes it). */
int acme_dqn_set_reissue(acme_dqn* l, int32_t enable);
/* Priority write-backs inside the step (acme_dqn_step_update) that gave up waiting for the
 * step's verdict (a bounded spin) and so wrote no priority although the step may have been
 * applied; synchronises.  Never expected; DQNLearner raises RuntimeError when it is non-zero. */
int acme_dqn_verdict_timeouts(acme_dqn* l, int64_t* out);
int64_t acme_dqn_verdicts_issued(const acme_dqn* l);
int acme_dqn_step_verdict(const acme_dqn* l, int64_t seq, int32_t* state);
/* The plane scales (powers of two) as learner state for checkpoints: acme_dqn_scale_state
 * writes *count floats to out (when out is non-NULL and capacity suffices);
 * acme_dqn_set_scale_state restores them after acme_dqn_params_changed, so the resumed
 * steps are bit-identical to the uninterrupted run instead of recalibrating. */
int acme_dqn_scale_state(const acme_dqn* l, float* out, int32_t capacity, int32_t* count);
int acme_dqn_set_scale_state(acme_dqn* l, const float* in, int32_t count);

typedef struct acme_transition_batch {
  const void* o_tm1;   /* [B, obs...]  u8 or f32 */
  const int32_t* a_tm1;/* [B] */
  const float* r_t;    /* [B] n-step return */
  const float* d_t;    /* [B] n-step discount */
  const void* o_t;     /* [B, obs...] */
  const double* probabilities; /* [B] f64 sampling probabilities (info.probability) */
  int64_t batch;
  /* If non-NULL: the minimum probability over the GLOBAL batch (data-parallel),
   * else the local batch minimum is used for the IS-weight max. */
  const double* global_min_probability;
  /* Denominator of the batch mean (loss and its gradient): 0 = batch.  A data-parallel
   * rank holding a share of a global batch of N * mean_over rows passes the nominal
   * per-rank batch, so that the all-reduce mean of the ranks' gradients is the global
   * batch's mean whatever the shares. */
  int64_t mean_over;
  /* Optional (uint8 Nature network): the exact f16 copy of [o_tm1; o_t], [2B][obs bytes]
   * u16, as acme_replay_sample_gather_frames writes it; the learner then skips its own
   * conversion (same bits).  NULL: the learner converts. */
  const uint16_t* obs_f16;
  /* Optional (hipEvent_t): an event at which every input of the batch (fields and
   * obs_f16) is complete, e.g. the prefetching dataset's ready event of the batch.  The
   * uint8 Nature plane path then starts the target forward on its second stream from this
   * event alone, without ordering it after the caller's stream, so it can overlap the end
   * of the previous step (its Adam); the learner falls back to ordering after the caller's
   * stream when that stream has written target state since the last step (a target copy,
   * a q_values call, new parameters, calibration) or when it converts the frames itself.
   * The caller must not write the target network's buffers, the learner's scale records
   * or the batch's inputs on another stream meanwhile.  NULL: ordered after the caller's
   * stream. */
  void* inputs_event;
} acme_transition_batch;

typedef struct acme_dqn_outputs {
  float* loss;         /* [1] device: mean weighted Huber loss */
  float* td_error;     /* [B] device (optional) */
  double* priorities;  /* [B] device |td| as f64 (optional) */
  float* q_tm1;        /* [B, A] device (optional) online q(o_tm1) */
} acme_dqn_outputs;

/* Forward + backward: fills grads (flat) and outputs.  Does not touch params. */
int acme_dqn_forward_backward(acme_dqn* l, const acme_transition_batch* batch,
                              const acme_dqn_outputs* out, void* stream);
/* The same work in two stages, for data parallelism that overlaps the gradient
 * all-reduce with the rest of the backward pass: stage 0 = forwards, loss, head and
 * dense-layer backward (writes grads[grad_split:]); stage 1 = torso backward (writes
 * grads[:grad_split]; a no-op for MLP networks, whose grad_split is 0).  Stage 0 may itself
 * be issued as stage 2 (the forwards) then stage 3 or 4 (loss, head and dense backward, the
 * same batch), so that batch->global_min_probability is only read from stage 3 on. */
int acme_dqn_forward_backward_stage(acme_dqn* l, const acme_transition_batch* batch,
                                    const acme_dqn_outputs* out, int32_t stage, void* stream);
int acme_dqn_grad_split(const acme_dqn* l, int64_t* split);
/* Stage 4 (acme_dqn_forward_backward_stage) is stage 3 without ordering the caller's stream
 * after the dense gradients grads[grad_split:] (computed beside it on the learner's second
 * stream); acme_dqn_dense_grads_ready makes `stream` wait for them, e.g. a collective
 * stream that all-reduces them while the caller's stream runs stage 1. */
int acme_dqn_dense_grads_ready(acme_dqn* l, void* stream);
/* Data parallelism over a caller-owned RCCL communicator (ncclComm_t; replaces a rank of
 * DQNLearner's torch.distributed path for non-Python callers): one rank per
 * GPU, each stepping on its share of the global batch (acme_transition_batch.mean_over =
 * the nominal per-rank batch).  acme_dqn_dp_step = min-probability all-reduce beside the
 * forwards, loss and dense backward, dense-gradient all-reduce (AVG) beside the torso
 * backward, torso-gradient all-reduce, Adam and the target copy, num_steps += 1; every
 * replica applies the same update.  RCCL is loaded at run time (librccl.so.1). */
int acme_dqn_dp_init(acme_dqn* l, void* nccl_comm, int32_t world_size);
int acme_dqn_dp_step(acme_dqn* l, const acme_transition_batch* batch,
                     const acme_dqn_outputs* out, void* stream);
/* Communicator helpers for callers that bring none: a 128-byte unique id made on one rank
 * and shared with the others, then one communicator per rank. */
int acme_nccl_get_unique_id(uint8_t* out128);
int acme_nccl_comm_init(const uint8_t* id128, int32_t world_size, int32_t rank, void** comm);
int acme_nccl_comm_destroy(void* comm);
/* Adam on (params, grads), then target <- params when num_steps % period == 0, then
 * num_steps += 1 (acme/agents/tf/dqn/learning.py:147-161). */
int acme_dqn_apply(acme_dqn* l, void* stream);
/* forward_backward + apply. */
int acme_dqn_step(acme_dqn* l, const acme_transition_batch* batch,
                  const acme_dqn_outputs* out, void* stream);
/* acme_dqn_step followed by the learner's priority write-back of the batch
 * (acme_replay_update_priorities(replay, keys, priorities, batch)), the order of
 * DQNLearner._step then the replay client's update (acme/agents/tf/dqn/learning.py:
 * 151-154).  On the uint8 Nature plane path the update is issued inside the step, on the
 * learner's second stream as soon as the loss has written the priorities, so it runs
 * beside the backward instead of after Adam; the step's final join orders it before the
 * caller's later work.  after_event (hipEvent_t, optional): the table's last device read
 * on another stream (a prefetching dataset's draw); the update waits for it on the stream
 * that issues it, as a caller of acme_replay_update_priorities orders its stream after
 * those draws.  Same results as the two calls. */
int acme_dqn_step_update(acme_dqn* l, const acme_transition_batch* batch,
                         const acme_dqn_outputs* out, acme_replay* replay,
                         const uint64_t* keys, void* after_event, void* stream);
/* Q forward only (online or target network) — actor/eval helper. */
int acme_dqn_q_values(acme_dqn* l, const void* obs, int64_t batch, int32_t use_target,
                      float* q_out, void* stream);
int64_t acme_dqn_num_steps(const acme_dqn* l);
/* Device pointer + element count of an internal f32 workspace (tests / diagnostics):
 * "x1" "x2" "x3" "hid" (online activations, 2B rows), "dzh" "dz3" "dz2" "dz1" (layer
 * pre-activation gradients, B rows), "q_on", "q_tg", "g". */
int acme_dqn_debug_buffer(const acme_dqn* l, const char* name, const float** out,
                          int64_t* count);
int acme_dqn_set_num_steps(acme_dqn* l, int64_t n);
/* Minimum of a device f64 array (for the data-parallel IS normaliser). */
int acme_min_f64(const double* x, int64_t n, double* out_dev, void* stream);

/* ------------------------------------------------------------------ D4PG -- */
/* Replaces D4PGLearner._step (acme/agents/tf/d4pg/learning.py:156-247) with the networks
 * of examples/control_suite/run_d4pg.py:60-81: policy = LayerNormMLP(policy_sizes,
 * activate_final) -> NearZeroInitializedLinear(act_dim) -> TanhToSpec; critic =
 * concat(obs, action) -> LayerNormMLP(critic_sizes, activate_final) ->
 * DiscreteValuedHead(vmin, vmax, num_atoms).  The observation network is the identity
 * (tf2_utils.batch_concat of a flat observation). */
#define ACME_D4PG_MAX_LAYERS 4
#define ACME_D4PG_MAX_ACT 16
#define ACME_D4PG_MAX_ATOMS 64

typedef struct acme_d4pg acme_d4pg;

typedef struct acme_d4pg_config {
  int32_t obs_dim;              /* flat observation size (<= 64 - act_dim) */
  int32_t act_dim;              /* <= ACME_D4PG_MAX_ACT */
  int32_t max_batch;
  int32_t num_policy_layers;    /* LayerNormMLP sizes, 2..ACME_D4PG_MAX_LAYERS */
  int32_t policy_sizes[ACME_D4PG_MAX_LAYERS];
  int32_t num_critic_layers;
  int32_t critic_sizes[ACME_D4PG_MAX_LAYERS];
  int32_t num_atoms;            /* <= ACME_D4PG_MAX_ATOMS */
  float vmin, vmax;
  float action_min[ACME_D4PG_MAX_ACT];  /* TanhToSpec bounds (spec.minimum / maximum) */
  float action_max[ACME_D4PG_MAX_ACT];
  float discount;
  int32_t target_update_period;
  float policy_learning_rate, critic_learning_rate;
  float adam_beta1, adam_beta2, adam_epsilon;
  int32_t clipping;             /* dqda norm clip 1.0 + global-norm clip 40 (learning.py:211-237) */
  float layer_norm_epsilon;     /* Sonnet LayerNorm default 1e-5 */
} acme_d4pg_config;

typedef struct acme_d4pg_batch {
  const float* o_tm1;  /* [B, obs_dim] */
  const float* a_tm1;  /* [B, act_dim] */
  const float* r_t;    /* [B] */
  const float* d_t;    /* [B] */
  const float* o_t;    /* [B, obs_dim] */
  int64_t batch;
} acme_d4pg_batch;

typedef struct acme_d4pg_outputs {
  float* critic_loss;  /* [1] device (optional) */
  float* policy_loss;  /* [1] device (optional) */
} acme_d4pg_outputs;

int acme_d4pg_create(const acme_d4pg_config* cfg, acme_d4pg** out);
int acme_d4pg_destroy(acme_d4pg* l);
/* Flat buffers hold the policy tensors, then the critic tensors (64-float aligned). */
int64_t acme_d4pg_flat_size(const acme_d4pg* l);
/* Floats [0, policy_size) are the policy's (its own Adam and global-norm clip). */
int64_t acme_d4pg_policy_size(const acme_d4pg* l);
int32_t acme_d4pg_num_tensors(const acme_d4pg* l);
int acme_d4pg_tensor_info(const acme_d4pg* l, int32_t i, int64_t* offset, int64_t* numel,
                          int32_t* ndim, int64_t* shape4, const char** name);
int acme_d4pg_bind(acme_d4pg* l, float* params, float* target, float* grads, float* adam_m,
                   float* adam_v);
/* One learner step: target <- online when num_steps % period == 0, num_steps += 1,
 * critic + policy losses and gradients, global-norm clipping, two Adams. */
int acme_d4pg_step(acme_d4pg* l, const acme_d4pg_batch* batch, const acme_d4pg_outputs* out,
                   void* stream);
/* Policy forward (actor / evaluation): actions [rows, act_dim]. */
int acme_d4pg_policy(acme_d4pg* l, const float* obs, int64_t rows, int32_t use_target,
                     float* actions, void* stream);
int64_t acme_d4pg_num_steps(const acme_d4pg* l);
int acme_d4pg_set_num_steps(acme_d4pg* l, int64_t n);
/* Internal device workspaces (tests): "p_a" (dpg actions), "t_a" (target actions),
 * "c_logits" (online critic logits, 2B rows: [q_tm1; dpg]), "t_logits", "dlogits",
 * "dqda", "norms" (policy / critic gradient global norms before clipping). */
int acme_d4pg_debug_buffer(const acme_d4pg* l, const char* name, const float** out,
                           int64_t* count);

/* ---------------------------------------------------------------- IMPALA -- */
/* Replaces IMPALALearner._step (acme/agents/tf/impala/learning.py:97-169) with
 * IMPALAAtariNetwork (acme/tf/networks/atari.py:115-144): OAREmbedding(AtariTorso) ->
 * snt.LSTM(lstm_size) -> Linear(head_size) -> ReLU -> PolicyValueHead(num_actions).
 * The policy and value layers are one fused [head_size, A + 1] tensor (column A = value). */
#define ACME_IMPALA_TORSO_ATARI 0 /* uint8 [84, 84, 4] frames, scaled 1/255 inside conv1 */
#define ACME_IMPALA_TORSO_FLAT 1  /* float [obs_dim] vector used as the torso output */

typedef struct acme_impala acme_impala;

typedef struct acme_impala_config {
  int32_t torso;
  int32_t obs_dim;              /* FLAT torso only */
  int32_t num_actions;          /* <= 63 */
  int32_t max_batch;            /* sequences per step (B) */
  int32_t max_sequence_length;  /* T */
  int32_t lstm_size;            /* multiple of 8, max_batch * (lstm_size + 32) <= 12288 */
  int32_t head_size;            /* multiple of 4 */
  float discount, entropy_cost, baseline_cost;
  float max_abs_reward;         /* INFINITY = no reward clipping (learning.py:70-71) */
  float max_gradient_norm;      /* 1e10 = effectively none (learning.py:72-73) */
  float learning_rate, adam_beta1, adam_beta2, adam_epsilon;
  int32_t semantics;            /* ACME_SEMANTICS_TF (default) or ACME_SEMANTICS_JAX */
} acme_impala_config;

/* One batch of sequences, batch-major [B, T, ...] as the dataset yields them. */
typedef struct acme_sequence_batch {
  const void* observation;      /* [B, T, 84, 84, 4] u8 or [B, T, obs_dim] f32 */
  const int32_t* prev_action;   /* [B, T] OAR observation: previous action */
  const float* prev_reward;     /* [B, T] OAR observation: previous reward */
  const int32_t* action;        /* [B, T] */
  const float* reward;          /* [B, T] */
  const float* discount;        /* [B, T] */
  const float* behaviour_logits;/* [B, T, A] extras['logits'] */
  const float* h0;              /* core_state hidden at t = 0: row b at h0 + b * state_stride */
  const float* c0;              /* core_state cell at t = 0 */
  int64_t state_stride;         /* floats between consecutive rows of h0 / c0 */
  int64_t batch;                /* B <= max_batch */
  int64_t sequence_length;      /* T, 2 <= T <= max_sequence_length */
} acme_sequence_batch;

int acme_impala_create(const acme_impala_config* cfg, acme_impala** out);
int acme_impala_destroy(acme_impala* l);
int64_t acme_impala_flat_size(const acme_impala* l);
int32_t acme_impala_num_tensors(const acme_impala* l);
int acme_impala_tensor_info(const acme_impala* l, int32_t i, int64_t* offset, int64_t* numel,
                            int32_t* ndim, int64_t* shape4, const char** name);
int acme_impala_bind(acme_impala* l, float* params, float* grads, float* adam_m, float* adam_v);
/* Declares that the caller wrote the bound params buffer directly (restore, broadcast): the
 * plane scales (the parameter planes' scale lags one step behind the parameters' maximum,
 * like the activations') are recalibrated before the next step.  The learner's own updates
 * need no call. */
int acme_impala_params_changed(acme_impala* l);
/* One SGD step; metrics (device, optional) = [loss, critic_loss, entropy_loss,
 * policy_gradient_loss] as logged by learning.py:162-167. */
int acme_impala_step(acme_impala* l, const acme_sequence_batch* batch, float* metrics,
                     void* stream);
/* Plane-range check of the Atari plane path (as acme_dqn_plane_overflow). */
int acme_impala_plane_overflow(acme_impala* l, int32_t* overflow, int32_t reset);
/* Step guard (as acme_dqn_guard_state): a step whose plane writes overflowed, or whose
 * one-launch LSTM unroll timed out, applies no update (Adam's device count stays);
 * out4 = {applied, skipped, last step skipped, LSTM timeouts so far}.
 * acme_impala_skipped_steps reads the pinned host mirror (no synchronisation). */
int64_t acme_impala_skipped_steps(const acme_impala* l);
int acme_impala_guard_state(acme_impala* l, int64_t* out4);
/* Adam's device count (checkpoint restore; acme_impala_set_num_steps sets it to n too). */
int acme_impala_set_applied_steps(acme_impala* l, int64_t n);
/* Plane scales as learner state (as acme_dqn_scale_state / acme_dqn_set_scale_state): a
 * resumed run restores them after acme_impala_params_changed instead of recalibrating. */
int acme_impala_scale_state(const acme_impala* l, float* out, int32_t capacity, int32_t* count);
int acme_impala_set_scale_state(acme_impala* l, const float* in, int32_t count);
/* The LSTM unroll of this learner: 0 (default) = one launch each for the forward and the
 * backward when lstm_size = 256 and the batch is at most 64 sequences
 * (workgroups own 4 sequences x 16 units and exchange h / dh partials as tagged granules;
 * spins bounded, debug buffer "lstm_timeout"), per-step launches otherwise; 1 = always
 * per-step launches. */
int acme_impala_set_lstm_unroll(acme_impala* l, int32_t mode);
/* One network step for `rows` independent actors (IMPALAActor.select_action): inputs
 * obs [rows, ...], prev_action / prev_reward [rows], state h / c [rows, lstm_size];
 * outputs logits [rows, A], values [rows], next state h_out / c_out. */
int acme_impala_policy_step(acme_impala* l, const void* obs, const int32_t* prev_action,
                            const float* prev_reward, const float* h, const float* c,
                            int64_t rows, float* logits, float* values, float* h_out,
                            float* c_out, void* stream);
/* Policy steps of this (actor-side) network on the plane engine: torso and W_i read f16
 * planes (the learner's f32-equivalent engine, csrc/gemm_p3.h) at scales rescaled after
 * every call from its maxima (calibrated by three passes on the first call); at least 64
 * rows.  For networks that run policy steps only: a learner's own scales are its steps'. */
int acme_impala_set_policy_planes(acme_impala* l, int32_t on);
int64_t acme_impala_num_steps(const acme_impala* l);
int acme_impala_set_num_steps(acme_impala* l, int64_t n);
/* "logits" "values" [B*T] batch-major rows, "vs" "pg_adv" [(T-1)*B] time-major,
 * "h" [B*T, H], "dpv" [B*T, A+1], "grad_norm" [1]. */
int acme_impala_debug_buffer(const acme_impala* l, const char* name, const float** out,
                             int64_t* count);

/* ------------------------------------------------------------------ R2D2 -- */
/* Replaces R2D2Learner._step (acme/agents/tf/r2d2/learning.py:112-200) with
 * R2D2AtariNetwork (acme/tf/networks/atari.py:72-112): OAREmbedding(AtariTorso, or the
 * observation vector with ACME_IMPALA_TORSO_FLAT) -> snt.LSTM(lstm_size) ->
 * DuellingMLP(num_actions, [head_size]) (duelling.py:26-59; its two first layers are one
 * fused [lstm_size, 2 head_size] tensor [value | advantage], as the DQN learner's).  The
 * step: burn-in of both networks over the first burn_in_length steps from the stored core
 * state (no gradient), online and target unrolls over the rest, greedy double-Q
 * transformed n-step loss (losses/r2d2.py:29-169), importance weights (1 / (N p))^beta
 * / max, snt.Adam(learning_rate, epsilon = adam_epsilon), target <- online when
 * num_steps % target_update_period == 0 after the update, priorities eta max_t |e| +
 * (1 - eta) mean_t |e| (learning.py:230-236). */
typedef struct acme_r2d2 acme_r2d2;

typedef struct acme_r2d2_config {
  int32_t torso;                /* ACME_IMPALA_TORSO_ATARI or ACME_IMPALA_TORSO_FLAT */
  int32_t obs_dim;              /* FLAT torso only */
  int32_t num_actions;
  int32_t max_batch;            /* sequences per step (B) */
  int32_t max_sequence_length;  /* T = burn_in + trace + 1, <= 256 */
  int32_t burn_in_length;
  int32_t lstm_size;            /* multiple of 8 (512 in R2D2AtariNetwork) */
  int32_t head_size;            /* multiple of 8 (512) */
  int32_t n_step;               /* bootstrap_n (learning.py:65: 5) */
  int32_t store_lstm_state;     /* 1: core state from extras (h0 / c0), 0: zeros */
  int32_t target_update_period;
  int32_t reserved;
  int64_t max_replay_size;      /* N of the importance weights */
  double max_priority_weight;   /* eta; eta and 1 - eta are rounded to f32 from double */
  double importance_sampling_exponent;  /* beta: the f64 weights' exponent (learning.py:181) */
  float discount;
  float learning_rate, adam_beta1, adam_beta2, adam_epsilon;  /* epsilon 1e-3 (:78) */
} acme_r2d2_config;

typedef struct acme_r2d2_outputs {
  float* loss;          /* [1] (optional) */
  float* errors;        /* [T - burn_in - 1][B] time-major, extra.errors (optional) */
  double* priorities;   /* [B] (optional) */
} acme_r2d2_outputs;

int acme_r2d2_create(const acme_r2d2_config* cfg, acme_r2d2** out);
int acme_r2d2_destroy(acme_r2d2* l);
int64_t acme_r2d2_flat_size(const acme_r2d2* l);
int32_t acme_r2d2_num_tensors(const acme_r2d2* l);
int acme_r2d2_tensor_info(const acme_r2d2* l, int32_t i, int64_t* offset, int64_t* numel,
                          int32_t* ndim, int64_t* shape4, const char** name);
int acme_r2d2_bind(acme_r2d2* l, float* params, float* target, float* grads, float* adam_m,
                   float* adam_v);
/* The caller wrote params / target directly (initialisation, restore): the Atari plane path
 * recalibrates its scales before the next step (as acme_impala_params_changed). */
int acme_r2d2_params_changed(acme_r2d2* l);
/* Plane scales as learner state (as acme_dqn_scale_state / acme_dqn_set_scale_state): a
 * checkpoint restored with them resumes bit-identically (0 floats without the plane path). */
int acme_r2d2_scale_state(const acme_r2d2* l, float* out, int32_t capacity, int32_t* count);
int acme_r2d2_set_scale_state(acme_r2d2* l, const float* in, int32_t count);
/* Step guard (as the DQN / IMPALA learners'): a step whose plane writes overflowed (Atari
 * plane path) or whose one-launch LSTM timed out applies no update; out3 = {applied,
 * skipped, last step skipped}; acme_r2d2_skipped_steps reads a pinned host mirror;
 * acme_r2d2_skip_word is the device word that gates the step's priority write-back
 * (acme_replay_update_priorities_gated). */
int64_t acme_r2d2_skipped_steps(const acme_r2d2* l);
int acme_r2d2_guard_state(acme_r2d2* l, int64_t* out3);
const uint32_t* acme_r2d2_skip_word(const acme_r2d2* l);
/* Adam's step count (updates applied; checkpoint restore after acme_r2d2_set_num_steps). */
int acme_r2d2_set_applied_steps(acme_r2d2* l, int64_t n);
/* One learner step on a batch of sequences (acme_sequence_batch: batch-major [B, T] fields;
 * behaviour_logits unused; h0 / c0 = extras['core_state'] at t = 0) with the sample's
 * probabilities [B] (f64). */
int acme_r2d2_step(acme_r2d2* l, const acme_sequence_batch* batch, const double* probabilities,
                   const acme_r2d2_outputs* out, void* stream);
int64_t acme_r2d2_num_steps(const acme_r2d2* l);
int acme_r2d2_set_num_steps(acme_r2d2* l, int64_t n);
/* mode 0 (default): the LSTM unroll and BPTT in one launch each when lstm_size is 256 or 512
 * and ceil(B / 4) * lstm_size / 16 <= 256; 1: one launch per time step (tests). */
int acme_r2d2_set_lstm_unroll(acme_r2d2* l, int32_t mode);
/* "q" / "target_q" [(T - burn_in) * B, A] time-major suffix rows, "h" [T * B, H]
 * time-major, "g" [(T - burn_in) * B] d loss / d q[a], "hid", "x1" "x2" "x3", "lstm_timeout"
 * (the one-launch unroll's sticky spin-timeout word; the loss reads NaN once it is set). */
int acme_r2d2_debug_buffer(const acme_r2d2* l, const char* name, const float** out,
                           int64_t* count);

/* ----------------------------------------------------------- elementwise ops -- */

/* ------------------------------------------------------------- profiling -- */
/* Section profiler: when enabled, every kernel section records a HIP event pair on the
 * stream it is launched on, tagged with its algorithmic FLOPs / HBM bytes. */
int acme_profile_enable(int32_t on);
int acme_profile_reset(void);
int32_t acme_profile_num_sections(void);
int acme_profile_query(int32_t i, const char** name, double* total_ms, int64_t* count,
                       double* flops, double* bytes);
/* TFLOP/s ceiling of the arithmetic path section i runs on (f32 MFMA 157.3; the exact
 * plane engines 2500 / MFMA terms per product: 833.3 for three terms, 1250 for two);
 * 0 for non-GEMM sections. */
int acme_profile_query_peak(int32_t i, double* peak_tflops);

/* snt.optimizers.Adam update over a flat f32 buffer (t = 1-based step). */
int acme_adam_update(float* params, const float* grads, float* m, float* v, int64_t n,
                     float lr, float beta1, float beta2, float eps, int64_t t,
                     void* stream);

#ifdef __cplusplus
}
#endif

#endif /* ACME_HIP_H_ */
