/*
 * fqlpop.h -- C ABI of the MI355X-native FQL population trainer (libfqlpop.so).
 *
 * The reference's boundary for this path is a Python object API, not an FFI
 * (SURVEY.md section 8b): the callers use FQLAgent.create / update /
 * total_loss / sample_actions / config and flax (to|from)_state_dict of the
 * un-vendored `fql` submodule [EXT].  Each entry point below cites the
 * reference call site it replaces.  The Python shim
 * `flow-q-learning_amd/fql/agents/fql.py` binds these with ctypes (see
 * INTEGRATION.md); nothing here uses torch or C++ types.
 *
 * Conventions
 *   - every function returns 0 on success or a negative FQLPOP_E* code; the
 *     message of the last failure on the calling thread is fqlpop_last_error();
 *   - the handle owns all device memory (params, Adam moments, target critic,
 *     dataset copy, activations, info); host pointers are borrowed for the
 *     duration of the call only;
 *   - calls are stream-ordered on the handle's streams; functions that return
 *     data to the host (read_info, get_state, sample_actions) synchronise;
 *   - one handle per host thread.
 *   - "member" indices are population slots 0..n_members-1.
 */
#ifndef FQLPOP_H
#define FQLPOP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FQLPOP_OK 0
#define FQLPOP_E_ARG (-1)      /* bad argument / shape */
#define FQLPOP_E_HIP (-2)      /* HIP runtime failure */
#define FQLPOP_E_STATE (-3)    /* call not valid in the current state */
#define FQLPOP_E_UNSUPPORTED (-4)

/* Number of float slots per member in the info buffers (13 used for train,
 * 10 for val, in the order of FQLPOP_INFO_*). */
#define FQLPOP_INFO_STRIDE 16
enum {
    FQLPOP_INFO_CRITIC_LOSS = 0, FQLPOP_INFO_Q_MEAN, FQLPOP_INFO_Q_MAX, FQLPOP_INFO_Q_MIN,
    FQLPOP_INFO_ACTOR_LOSS, FQLPOP_INFO_BC_FLOW_LOSS, FQLPOP_INFO_DISTILL_LOSS,
    FQLPOP_INFO_Q_LOSS, FQLPOP_INFO_Q, FQLPOP_INFO_MSE,
    FQLPOP_INFO_GRAD_MAX, FQLPOP_INFO_GRAD_MIN, FQLPOP_INFO_GRAD_NORM
};

/* Which state buffer get_state/set_state address. */
enum { FQLPOP_STATE_PARAMS = 0, FQLPOP_STATE_ADAM_M = 1, FQLPOP_STATE_ADAM_V = 2 };

/* Mirrors trainer/config.py:5-22 (AgentConfig) for the fields update() reads. */
typedef struct fqlpop_config {
    int obs_dim;           /* ob_dims[-1]; set by FQLAgent.create from ex_observations */
    int action_dim;        /* set by FQLAgent.create from ex_actions */
    int hidden_dim;        /* width of every hidden layer (actor_hidden_dims == value_hidden_dims) */
    int num_hidden;        /* number of hidden layers (4) */
    int batch_size;        /* AgentConfig.batch_size (256 / 1024) */
    int num_qs;            /* critic ensemble size (2) */
    int layer_norm;        /* critic LayerNorm (scripts pass --agent.layer_norm) */
    int actor_layer_norm;  /* actor LayerNorm (False) */
    int flow_steps;        /* Euler steps (10) */
    int q_agg_min;         /* q_agg == "min" (else "mean") */
    int normalize_q_loss;  /* normalize_q_loss */
    float discount;        /* 0.99 */
    float tau;             /* 0.005 */
    float lr;              /* Adam learning rate 3e-4 */
    int use_graph;         /* capture each step into a hipGraph (1) or launch eagerly (0) */
} fqlpop_config;

typedef struct fqlpop fqlpop_t;

/* Message of the last failed call on this thread ("" if none). */
const char* fqlpop_last_error(void);

/* Engine options: process-wide defaults read by every later fqlpop_create.  They
 * select alternate code paths and stream schedules with the same results
 * (bit-identical, or the per-layer / unfused paths within the parity tolerance),
 * for tests and profiling; there is no reference counterpart.  Names:
 *   euler_fused, stream_fwd, stream_bwd, fused_adam, serial  (0/1)
 *   dw_tile_critic / dw_tile_actor (0..10), adam_nt (0..3),
 *   split (0 off, 1 auto, 2 / 4 / 8: small populations run the streamed forwards, the
 *   Euler flow and the critic / one-step backwards as clusters of 2-8 blocks per 16-column
 *   tile; bit-identical to the unsplit kernels),
 *   small_sched (0/1: up to 256 16-column tiles per step, the target critic and the
 *   critic's TD-column backward run on a fourth stream; bit-identical),
 *   split_sites, split_blocks (per-site split factors and the block cap of a split forward,
 *   for A/B runs),
 *   hw_queues (1..1024, default 4): the GPU_MAX_HW_QUEUES the caller runs the HIP runtime
 *   with.  Below 4 the step is captured on one stream: ROCm 7's graph launch can index past
 *   its pool of branch streams when more than one shares the launch stream's hardware queue.
 *   A caller that sets GPU_MAX_HW_QUEUES passes it here (the Python Population does).
 *   em_seq_sweep (0/1, default 1; read by fqlpop_emtrain_create): multistep env-model
 *   training as a forward and a backward sweep per 16 sequences plus a dW GEMM (0: the
 *   round-5 kernel with dW inside the time loop; same oracle tolerance).
 * The defaults are the measured-fastest configuration.  Unknown names or values
 * out of range: FQLPOP_E_ARG.  (Round 3's schedule experiments that measured slower --
 * streams, prio, cdw_sb, dw_stagger, xstep, bc_late, fuse_dq, early_join -- were
 * removed.)  The production library reads no environment variable; result-changing
 * timing switches exist only in diagnostic builds. */
int fqlpop_set_engine_option(const char* name, int value);
int fqlpop_get_engine_option(const char* name, int* value);
int fqlpop_reset_engine_options(void);
/* The split plan a population of n_members created now with `cfg` would run (no GPU call):
 * blocks per 16-column tile of each split launch site, 1 = the unsplit kernel, in site order
 * {BC forward, Euler flow, one-step forward, target critic, critic forward, critic backward
 * (its Q-loss columns under the 4th-stream schedule), one-step backward, critic
 * TD-column backward (4th-stream schedule only)} (blocks_per_tile[8]), and whether the
 * 4th-stream schedule runs.  The step checks each launch against this plan.
 * [no reference counterpart: engine introspection] */
int fqlpop_split_plan(const fqlpop_config* cfg, int n_members, int* blocks_per_tile, int* small_sched);
/* Streams (parallel graph branches) a population created now would capture its step on:
 * 4 (sM, sF, sB, sX), or 1 when engine option serial is set or hw_queues < 4.  The HIP
 * runtime's graph launch indexes past its branch-stream pool when more branches than
 * hardware queues share the launch stream's queue; the capture refuses
 * (FQLPOP_E_STATE) a step with more branches than hw_queues.  No GPU call.  [no reference
 * counterpart: engine introspection] */
int fqlpop_step_streams(int* n_streams);
/* 1 in a diagnostic build (make DIAG=1 / PHASE=1), 0 in the production library. */
int fqlpop_diagnostic_build(void);

/* Replaces FQLAgent.create(seed, ex_obs, ex_act, config)  [EXT]
 * (called at trainer/experiment.py:44-49, utils/agent.py:24-29) for a whole
 * population: allocates the device state for n_members members, member i
 * with alpha alphas[i] and seed seeds[i]; params are initialised on device
 * (Glorot-uniform kernels, zero biases, unit LN scale, target := critic). */
int fqlpop_create(const fqlpop_config* cfg, int n_members, const float* alphas,
                  const uint64_t* seeds, int device, fqlpop_t** out);

/* Frees every device allocation of the handle. */
int fqlpop_destroy(fqlpop_t* h);

/* Replaces the ReplayBuffer/Dataset behind OfflineTaskWithRealEvaluations
 * (task/offline_task_real.py:26-36; sampled at :38-43).  which = 0 train,
 * 1 val.  Row-major host arrays obs[n][obs_dim], act[n][action_dim], rew[n],
 * mask[n], next_obs[n][obs_dim]; copied into an HBM-resident buffer.  If
 * on_device != 0 the pointers are device pointers on the handle's device. */
int fqlpop_set_dataset(fqlpop_t* h, int which, const float* obs, const float* act,
                       const float* rew, const float* mask, const float* next_obs,
                       int64_t n_rows, int on_device);

/* Selects the members that step()/total_loss() advance (SuccessiveHalving
 * pruning, hpo/successive_halving.py:67-101; Experiment.stop at
 * trainer/trainer.py:114-116).  mask[n_members], nonzero = active. */
int fqlpop_set_active(fqlpop_t* h, const uint8_t* mask);

/* Replaces n_steps iterations of the Experiment.train hot loop
 * (trainer/experiment.py:106-109): for every active member, sample a
 * minibatch on device (uniform with replacement, Philox keyed by the member
 * seed and update count) and run agent.update(batch) [EXT FQLAgent.update]. */
int fqlpop_step(fqlpop_t* h, int n_steps);

/* agent.update(batch) (trainer/experiment.py:109) on a host batch: one
 * update of every active member.  batch: per active member (in slot order)
 * the row-major block [obs B*D][act B*A][rew B][mask B][next_obs B*D].
 * noise: NULL => drawn on device (Philox keyed by member seed and update
 * count); else the parity mode: per active member
 * [z_next B*A][x0 B*A][t B][z_d B*A][z_metric B*A].  Host pointers. */
int fqlpop_step_injected(fqlpop_t* h, const float* batch, const float* noise);

/* Replaces agent.total_loss(val_batch, grad_params=None)
 * (trainer/experiment.py:114-115): losses of every active member, no update.
 * batch NULL => sample from the val dataset (which = 1, or the train
 * dataset if no val dataset was set); noise NULL => device RNG; else
 * injected as in fqlpop_step_injected. Results via fqlpop_read_info(h, 1, .). */
int fqlpop_total_loss(fqlpop_t* h, const float* batch, const float* noise);

/* Copies info[n_members][FQLPOP_INFO_STRIDE] of the last train step (which=0)
 * or last total_loss (which=1) to the host; synchronises.  Replaces the
 * update_info / val_info dicts (trainer/experiment.py:109,115). */
int fqlpop_read_info(fqlpop_t* h, int which, float* out);

/* Replaces agent.sample_actions(observations=obs, seed=..)
 * (evaluator/evaluation.py:58-64,94): clip(onestep(s, z), -1, 1) for n rows of
 * member `member`.  noise[n][action_dim] (host) or NULL => z ~ N(0,1) from
 * Philox(seed).  obs[n][obs_dim], out[n][action_dim] host arrays. */
int fqlpop_sample_actions(fqlpop_t* h, int member, const float* obs, int64_t n,
                          const float* noise, uint64_t seed, float* out);

/* Number of floats of one member's flat state (flax tree order: networks
 * actor_bc_flow, actor_onestep_flow, critic, target_critic; leaves sorted as
 * flax does).  which = FQLPOP_STATE_*; M/V have the same layout as PARAMS
 * (target leaves are zero in M/V). */
int fqlpop_state_size(fqlpop_t* h, int64_t* n_floats);

/* flax.serialization.to_state_dict / from_state_dict of one member
 * (trainer/experiment.py:61-63,92,135; utils/agent.py:35): copy the flat
 * state out of / into device memory; synchronises. */
int fqlpop_get_state(fqlpop_t* h, int member, int which, float* flat, int64_t n);
int fqlpop_set_state(fqlpop_t* h, int member, int which, const float* flat, int64_t n);

/* Adam step count of a member (optax count == number of updates). */
int fqlpop_get_count(fqlpop_t* h, int member, int32_t* count);
int fqlpop_set_count(fqlpop_t* h, int member, int32_t count);

/* Per-member alpha and seed (ExperimentConfig.alpha/seed,
 * trainer/config.py:25-28); re-initialises params when reinit != 0. */
int fqlpop_set_member(fqlpop_t* h, int member, float alpha, uint64_t seed, int reinit);

/* Leaf table of the flat state: name (e.g. "critic/Dense_0/kernel"), offset
 * and shape (up to 3 dims, ndim returned).  i in [0, fqlpop_num_leaves). */
int fqlpop_num_leaves(fqlpop_t* h, int* n);
int fqlpop_leaf_info(fqlpop_t* h, int i, char* name, int name_cap, int64_t* offset,
                     int* ndim, int64_t* shape3);

/* Waits for all work of the handle.  Reports (once) a split launch that gave up; the
 * members it stepped stay poisoned: fqlpop_step / _step_injected refuse while an active
 * member is poisoned, fqlpop_get_state / _get_count refuse for a poisoned member and
 * fqlpop_read_info while any is, until fqlpop_set_state has restored the member's params,
 * Adam m and Adam v (or fqlpop_set_member reinit).  [EXT: a JAX error surfaces at the next
 * blocking call of the reference's jitted update] */
int fqlpop_sync(fqlpop_t* h);
/* Test hook: sets the handle's split-error word exactly as a split launch whose hand-off
 * wait gave up does (kernels.hip sp_fail), so the error path above can be exercised without
 * a fault.  FQLPOP_E_STATE if the population runs no split launch.  [no reference
 * counterpart] */
int fqlpop_debug_fail_split(fqlpop_t* h);

/* Measurement hook for bench.py: replays the dominant kernel (the hidden-
 * layer forward GEMM of the Euler flow, all active members in one launch)
 * `iters` times on its own stream between HIP events; returns the mean
 * duration (us) and the algorithmic FLOPs of one launch. */
int fqlpop_time_dominant_kernel(fqlpop_t* h, int iters, double* avg_us, double* flops);

/* In-step timing probe of the dominant kernel (bench.py's roofline): while
 * enabled, every Euler-flow hidden-layer GEMM launch inside fqlpop_step
 * stamps the 100 MHz s_memrealtime clock at the start and end of each of its
 * blocks; a launch lasts max(end) - min(start).  read_probe returns the total
 * (us) and number of launches timed since set_probe (which resets them), and
 * if clock_check != NULL the last fqlpop_time_dominant_kernel cross-check:
 * [0] one isolated launch timed by HIP events, [1] the same by its stamps. */
int fqlpop_set_probe(fqlpop_t* h, int enable);
/* The dominant kernel of fqlpop_step (bench.py's roofline row): its kernel
 * symbol (for profiler filters), algorithmic FLOPs and unique HBM bytes of one
 * launch over the active members. */
int fqlpop_dominant_kernel_info(fqlpop_t* h, char* name, int name_cap, double* flops, double* bytes);
int fqlpop_read_probe(fqlpop_t* h, double* total_us, int64_t* launches, double* clock_check);
/* Probe coverage since set_probe: blocks whose start and end stamps were both written, and
 * blocks launched, summed over the timed launches (equal when every block of every timed
 * launch stamped; the stamps are cleared after each read).  [no reference counterpart] */
int fqlpop_probe_coverage(fqlpop_t* h, int64_t* blocks_seen, int64_t* blocks_expected);

/* ---------------------------------------------------------------------
 * World-model rollout evaluation (BASELINE config 5).
 * Replaces the per-step Python loop of evaluator/evaluation.py:75-114 driving
 * task/offline_task_simulated.py:85-107 (state predictor + termination
 * predictor loaded by utils/envmodel.py:10-56) with ONE device launch for all
 * active members.  Env-model shapes (envmodel/baseline.py:17-37,
 * envmodel/multistep.py:35-54 uses the same cell, envmodel/termination_predictor.py:9-21). */
typedef struct fqlpop_envmodel_config {
    int obs_dim, action_dim;
    int sp_num_hidden;      /* BaselineStatePredictor hidden_dims (multistep default 128,256,128) */
    int sp_hidden[7];
    int tp_num_hidden;      /* TerminationPredictor hidden_dims (default 128,128) */
    int tp_hidden[7];
} fqlpop_envmodel_config;

/* Float counts of the flat parameter vectors in flax leaf order:
 * state predictor  Dense_0/bias, Dense_0/kernel, ..., Dense_n/kernel, LayerNorm_0/bias, LayerNorm_0/scale;
 * termination      Dense_0/bias, Dense_0/kernel, ..., Dense_m/kernel  (kernels [in][out]). */
int fqlpop_envmodel_param_count(const fqlpop_envmodel_config* cfg, int64_t* n_sp, int64_t* n_tp);

/* Upload the env model (utils/envmodel.py:load_model for "baseline"/"multistep"
 * and "termination_predictor"); host arrays, copied. */
int fqlpop_set_env_model(fqlpop_t* h, const fqlpop_envmodel_config* cfg, const float* sp_params, int64_t n_sp,
                         const float* tp_params, int64_t n_tp);

/* Roll every ACTIVE member's one-step policy in the env model from init_obs
 * [n_envs][obs_dim] until each env terminated (termination logit > 0: success 1)
 * or max_steps (truncated: success 0).  noise: NULL (z ~ N(0,1) from Philox keyed
 * by seed and the member seed) or host [n_active][max_steps][n_envs][action_dim].
 * out: host [n_active][n_envs][2] = (success, episode length); out_obs: NULL or
 * host [n_active][n_envs][obs_dim], the observation after the last step run.
 * Active members in slot order.  Needs hidden_dim 512; synchronises. */
int fqlpop_rollout(fqlpop_t* h, const float* init_obs, int n_envs, int max_steps, uint64_t seed,
                   const float* noise, float* out, float* out_obs);

/* One env-model step for given actions (task/offline_task_simulated.py:85-90:
 * state_predictor(obs, actions) then termination_predictor(next_obs)): obs
 * [n][obs_dim], actions [n][action_dim] -> next_obs [n][obs_dim], logits [n]
 * (terminated = logit > 0).  Host arrays; synchronises. */
int fqlpop_envmodel_step(fqlpop_t* h, const float* obs, const float* actions, int n, float* next_obs, float* logits);

/* ---------------------------------------------------------------------------
 * Env-model trainer: the reference's world-model
 * trainers, one fused GPU step per train_step.
 *   FQLPOP_EM_STATE_PREDICTOR: StatePredictorTrainer.train_step
 *     (envmodel/state_predictor_trainer.py:67-95) on BaselineStatePredictor
 *     (envmodel/baseline.py:25-37) with state_prediction_loss
 *     (envmodel/loss.py:80-111, reconstruction_weight 0 as train_env_model.py:37-44
 *     binds it; termination_weight > 0 scores the predicted next observation with
 *     a frozen termination predictor, fqlpop_emtrain_set_frozen_termination).
 *   FQLPOP_EM_TERMINATION: TerminationPredictorTrainer.train_step
 *     (envmodel/termination_predictor_trainer.py:55-76) on TerminationPredictor
 *     (envmodel/termination_predictor.py:14-21, input dropout) with focal_loss
 *     (envmodel/loss.py:33-66, train_env_model.py:79).
 *   Optimiser: optax.adam(optax.cosine_decay_schedule(init_lr, steps))
 *     (state_predictor_trainer.py:57-61).
 * Parameters are flat vectors in flax leaf order (path-sorted): Dense_i/bias,
 * Dense_i/kernel ([in][out]) ..., then LayerNorm_0/bias, LayerNorm_0/scale. */
enum { FQLPOP_EM_STATE_PREDICTOR = 0, FQLPOP_EM_TERMINATION = 1, FQLPOP_EM_MULTISTEP = 2 };
/* FQLPOP_EM_MULTISTEP: the same trainer on MultistepStatePredictor
 *   (envmodel/multistep.py:31-54, train_env_model.py:46-66): the baseline cell scanned
 *   over sequence_length steps from observations[:, 0] (each prediction is the next
 *   step's observation), state_prediction_loss over all B x T predictions, gradients by
 *   backpropagation through time.  Batches are [B][T][..]; device sampling draws
 *   MultistepLoader windows (utils/data_loader.py:25-39): a uniform episode of
 *   episode_length rows, a uniform start in [0, episode_length - T). */
#define FQLPOP_EM_LOG_STRIDE 8
/* logs: state predictor  [loss, next_observation_loss, termination_loss,
 *                         true_termination_loss, false_termination_loss]
 *       termination      [loss, true_loss, false_loss, accuracy, precision, recall]
 *       (accuracy / precision / recall: eval only; envmodel/termination_predictor_trainer.py:78-112) */
typedef struct fqlpop_emtrain_config {
    int kind;                      /* FQLPOP_EM_* */
    int obs_dim, action_dim;
    int num_hidden;
    int hidden_dims[8];            /* --model.hidden_dims, default (128, 256, 128) (argparser.py:184-189) */
    int batch_size;                /* multiple of 16 (256) */
    int steps;                     /* cosine decay horizon (TrainerConfig.steps) */
    float init_lr;                 /* 1e-3 */
    float termination_weight;      /* state predictor (argparser default 1.0; baseline scripts 0) */
    float true_termination_weight; /* 30 */
    float focal_alpha, focal_gamma;/* 0.25, 2 */
    float dropout_rate;            /* 0.1 */
    uint64_t seed;                 /* device sampling and the fixed dropout mask */
    int tp_num_hidden;             /* frozen termination predictor (termination_weight > 0) */
    int tp_hidden_dims[8];
    int sequence_length;           /* FQLPOP_EM_MULTISTEP: T (--sequence_length, 256) */
    int episode_length;            /* FQLPOP_EM_MULTISTEP device sampling: rows per episode (1000) */
} fqlpop_emtrain_config;
typedef struct fqlpop_emtrain fqlpop_emtrain_t;

int fqlpop_emtrain_param_count(const fqlpop_emtrain_config* cfg, int64_t* n_params);
/* Replaces TrainState.create(params=model.init(...), tx=adam(schedule)) of the
 * trainers' __init__; params are the initial flat parameters (host, copied). */
int fqlpop_emtrain_create(const fqlpop_emtrain_config* cfg, const float* params, int64_t n_params, int device,
                          fqlpop_emtrain_t** out);
int fqlpop_emtrain_destroy(fqlpop_emtrain_t* h);
/* utils/envmodel.py load_model("termination_predictor") of the state trainer's __init__. */
int fqlpop_emtrain_set_frozen_termination(fqlpop_emtrain_t* h, const float* tp_params, int64_t n);
/* The StepLoader's dataset (utils/data_loader.py:47-52), uploaded once: rows sampled on
 * device (uniform with replacement, Philox keyed by seed and step). */
int fqlpop_emtrain_set_dataset(fqlpop_emtrain_t* h, const float* obs, const float* act, const float* rew,
                               const float* next_obs, int64_t n_rows);
/* n_steps train_steps on device-sampled batches (asynchronous). */
int fqlpop_emtrain_step(fqlpop_emtrain_t* h, int n_steps);
/* One train_step on a host batch [batch_size][..]; keep_mask: NULL (the handle's fixed
 * Philox dropout mask) or [batch_size][obs_dim] bytes (termination kind). Synchronises. */
int fqlpop_emtrain_step_injected(fqlpop_emtrain_t* h, const float* obs, const float* act, const float* rew,
                                 const float* next_obs, const uint8_t* keep_mask);
/* eval_step on a host batch (no dropout, no update): logs[FQLPOP_EM_LOG_STRIDE]. */
int fqlpop_emtrain_eval(fqlpop_emtrain_t* h, const float* obs, const float* act, const float* rew,
                        const float* next_obs, float* logs);
/* Logs of the last train step; synchronises. */
int fqlpop_emtrain_read_logs(fqlpop_emtrain_t* h, float* logs);
/* which = FQLPOP_STATE_PARAMS / _ADAM_M / _ADAM_V; flax.serialization.to_bytes source
 * (train_env_model.py:132-134). Synchronises. */
int fqlpop_emtrain_get_params(fqlpop_emtrain_t* h, int which, float* out, int64_t n);
int fqlpop_emtrain_get_count(fqlpop_emtrain_t* h, int64_t* count);
int fqlpop_emtrain_sync(fqlpop_emtrain_t* h);

/* Algorithmic GEMM FLOPs of one member-update at the handle's config
 * (SURVEY.md 8d formula). */
double fqlpop_flops_per_member_step(const fqlpop_config* cfg);

#ifdef __cplusplus
}
#endif
#endif /* FQLPOP_H */
