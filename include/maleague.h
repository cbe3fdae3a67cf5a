/*
 * maleague.h -- C ABI of the MI355X-native hot path of PMatthaei/ma-league (libmaleague.so, gfx950).
 *
 * Every entry point takes plain device pointers (HBM, allocated by the caller: PyTorch's caching
 * allocator in the Python host package), sizes, and a hipStream_t passed as void*. Kernels are
 * enqueued on that stream; no call allocates, frees or synchronises (graph-capturable), except
 * where noted. Return value: 0 on success, nonzero on error; mlg_last_error() holds the message.
 *
 * Reference interfaces each entry point replaces (file:line in /root/reference):
 *   mlg_rollout        ParallelStepper.run / reset  src/steppers/parallel_stepper.py:82-216
 *   mlg_rollout_selfplay SelfPlayParallelStepper.run src/steppers/self_play_parallel_stepper.py:73-201
 *                      (+ SelfPlayStepper.run src/steppers/self_play_stepper.py:44-147,
 *                         build_pre_transition_data src/steppers/utils/stepper_utils.py:4-24)
 *                      + EnvWorker step/reset       src/steppers/utils/env_worker_process.py:27-71
 *                      + BasicMAC.select_actions    src/marl/controllers/basic_controller.py:29-36
 *                      + EpsilonGreedy.select       src/marl/components/action_selectors.py:44-62
 *                      + maenv TeamsEnv.step/get_obs/get_state/get_avail_actions (external)
 *   mlg_env_reset      EnvWorker "reset" command    src/steppers/utils/env_worker_process.py:54-60
 *   mlg_env_step       EnvWorker "step" command     src/steppers/utils/env_worker_process.py:32-53
 *   mlg_env_observe    TeamsEnv get_obs/get_state/get_avail_actions (env_worker_process.py:41-42)
 *   mlg_agent_forward  DRQNAgentNetwork.forward     src/marl/modules/agents/drqn_agent.py:29-35
 *   mlg_mac_forward    BasicMAC.forward + _build_inputs  src/marl/controllers/basic_controller.py:38-50,80-92
 *   mlg_select_actions EpsilonGreedyActionSelector.select src/marl/components/action_selectors.py:44-62
 *   mlg_pack_agent     (layout step feeding the above; no reference counterpart)
 *   mlg_qmix_forward   QMixer.forward               src/marl/modules/mixers/qmix.py:41-59
 *   mlg_refil_*        REFIL (config 5): see the REFIL section below
 *   mlg_qlearner_*     QLearner.train               src/marl/learners/q_learner.py:34-131
 *                      + clip_grad_norm_ + RMSprop.step (q_learner.py:104-105, learner.py:25-31)
 */
#ifndef MALEAGUE_H
#define MALEAGUE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MLG_MAXU 64 /* max units per env (large.json has 50) */

/* Frozen synthetic TeamsEnv spec v1. Built on the host from env_args. */
typedef struct {
    int32_t U;             /* total units (both teams) */
    int32_t n_agents;      /* policy-controlled units = env_info["n_agents"] */
    int32_t n_actions;     /* 5 + U */
    int32_t grid;          /* env_args.grid_size */
    int32_t episode_limit; /* env_info["episode_limit"] */
    int32_t stochastic;    /* env_args.stochastic_spawns */
    int32_t policy_team;   /* first non-scripted plan team (stepper_utils.py:48-55) */
    int32_t n_policy_teams;
    int32_t team[MLG_MAXU];
    int32_t role[MLG_MAXU];  /* TANK 0, HEALER 1, ADC 2 */
    int32_t melee[MLG_MAXU]; /* RANGED 0, MELEE 1 */
    int32_t agent_unit[MLG_MAXU];
    int32_t scripted[2];
    uint64_t seed; /* per-env key = seed * 2^32 + env_index */
} MlgEnvSpec;

/* Device-resident env state, SoA, [B][U] int32 + per-env counters. */
typedef struct {
    int32_t *x, *y, *hp;   /* [B*U] */
    int32_t *t;            /* [B] step index within episode */
    uint32_t *episode;     /* [B] episodes started (RNG stream counter) */
    int32_t B;
} MlgEnvState;

/* EpisodeBatch transition tensors (scheme of ma_experiment.py:99-118), all [B][T1][...] row-major. */
typedef struct {
    float *state;          /* [B][T1][S] */
    float *obs;            /* [B][T1][N][d_obs] */
    int64_t *actions;      /* [B][T1][N][1] */
    int32_t *avail;        /* [B][T1][N][A] */
    float *reward;         /* [B][T1][1] */
    uint8_t *terminated;   /* [B][T1][1] */
    float *actions_onehot; /* [B][T1][N][A] */
    int64_t *filled;       /* [B][T1][1] */
    int32_t B, T1;
    /* Ring mode (mlg_rollout only): env b writes slot (ring_slot0 + b) % ring_size of tensors that hold
     * ring_size slots (the replay buffer itself -- zero-copy insert); full_write = 1 makes the kernel write
     * every byte of the slots it owns (zeros included), so the caller need not zero-initialise them. */
    int32_t ring_slot0, ring_size, full_write;
    /* Sampled view (learner entry points only): episode b lives in slot rows[b] of tensors holding more
     * slots (the replay buffer itself -- no gather copy); nullptr = identity. */
    const int32_t *rows;
    /* Full-write mode, optional [ring_size] (or [B] without a ring): per slot, the exclusive end of the rows
     * that may hold non-zero data (>= T1 = unknown, e.g. a fresh or externally written buffer). The rollout
     * zeroes only rows [L + 1, slot_extent) of a slot whose new episode has length L instead of [L + 1, T1),
     * and stores slot_extent = L + 1. nullptr = zero every tail row. */
    int32_t *slot_extent;
} MlgBatch;

/* Per-run episode summary written by mlg_rollout. */
typedef struct {
    int32_t *ep_len;   /* [B] env steps taken (t_env increment per env) */
    float *ret;        /* [B] episode return of the policy team (reward[0]) */
    int32_t *won;      /* [B][2] battle_won, policy team first */
    int32_t *draw;     /* [B] */
    uint64_t *agent_rows; /* optional [1], accumulated: agent rows the launch ran through the MFMA cell
                             (16-row tiles, padding included; living agents of running envs only) */
    float *ret_away;   /* optional [B] (mlg_rollout_selfplay): episode return of the away team (reward[1]) */
} MlgRunInfo;

/* Agent weights in canonical nn.Module layout (state_dict of DRQNAgentNetwork). */
typedef struct {
    const float *fc1_w, *fc1_b;     /* [H][d_in], [H] */
    const float *w_ih, *b_ih;       /* [3H][H], [3H] */
    const float *w_hh, *b_hh;       /* [3H][H], [3H] */
    const float *fc2_w, *fc2_b;     /* [A][H], [A] */
} MlgAgentParams;

typedef struct {
    int32_t d_obs, n_actions, n_agents, hidden, d_in;
    int32_t obs_last_action, obs_agent_id;
} MlgAgentDims;

/* Size in floats of the packed agent weight block used by the kernels. */
int64_t mlg_packed_agent_size(const MlgAgentDims *d);
int mlg_pack_agent(const MlgAgentDims *d, const MlgAgentParams *p, float *packed, void *stream);

int mlg_env_reset(const MlgEnvSpec *spec, MlgEnvState *st, void *stream);
int mlg_env_step(const MlgEnvSpec *spec, MlgEnvState *st, const int64_t *actions /*[B][N]*/,
                 float *reward /*[B][n_policy_teams]*/, int32_t *done /*[B]*/, int32_t *won /*[B][2]*/,
                 int32_t *draw /*[B]*/, void *stream);
int mlg_env_observe(const MlgEnvSpec *spec, const MlgEnvState *st, float *obs /*[B][N][8U]*/,
                    float *state /*[B][6U]*/, int32_t *avail /*[B][N][A]*/, void *stream);

/* One full ParallelStepper.run: reset all B envs, step until every env terminated, filling `batch`
 * (caller zero-initialised, like EpisodeBatch construction). epsilon already evaluated on the host
 * (DecayThenFlatSchedule.eval(t_env)); test_mode forces epsilon 0. */
int mlg_rollout(const MlgEnvSpec *spec, MlgEnvState *st, const MlgAgentDims *dims, const float *packed,
                MlgBatch *batch, MlgRunInfo *info, float epsilon, int32_t test_mode, void *stream);

/* One full SelfPlayParallelStepper.run: both plan teams are policy-controlled (spec->n_agents = 2 * nh, the
 * first nh agents are the home team). Home agents act with home_packed into `home`, away agents with
 * away_packed into `away` (obs / avail of each side's own agents; state, terminated and filled in both;
 * reward[0] -> home, reward[1] -> away, as stepper_utils.build_pre_transition_data splits them). dims
 * describe ONE side's MAC (n_agents = nh). Epsilon per side; the epsilon RNG stream index is the global
 * agent index (home 0..nh-1, away nh..2nh-1). info->ret_away receives the away returns. */
int mlg_rollout_selfplay(const MlgEnvSpec *spec, MlgEnvState *st, const MlgAgentDims *dims, const float *home_packed,
                         const float *away_packed, MlgBatch *home, MlgBatch *away, MlgRunInfo *info,
                         float eps_home, float eps_away, int32_t test_mode, void *stream);

/* Zero `count` EpisodeBatch slots starting at slot0 (mod ring_size) in every key -- one launch; the
 * ring-mode pre-fill that replaces constructing a zero EpisodeBatch. slot_bytes[8] = bytes per slot of
 * state, obs, actions, avail, reward, terminated, actions_onehot, filled. */
int mlg_zero_slots_bytes(const MlgBatch *batch, const int64_t *slot_bytes, int32_t slot0, int32_t count,
                         int32_t ring_size, void *stream);

/* DRQN forward over R rows: q[R][A], h_out[R][H] from inputs[R][d_in], h_in[R][H]. */
int mlg_agent_forward(const MlgAgentDims *d, const float *packed, const float *inputs, const float *h_in,
                      float *q, float *h_out, int32_t R, void *stream);

/* BasicMAC.forward(ep_batch, t): builds inputs from the batch at t (obs, onehot(a_{t-1}), agent id). */
int mlg_mac_forward(const MlgAgentDims *d, const float *packed, const MlgBatch *batch, int32_t t,
                    const float *h_in, float *q /*[B][N][A]*/, float *h_out, void *stream);

/* Epsilon-greedy over rows r of q[R][A] with avail[R][A] (int32). rng key per row:
 * keys[r / n_agents] with ctr(episode[r / n_agents], t, purpose, r % n_agents). */
int mlg_select_actions(const float *q, const int32_t *avail, int32_t R, int32_t A, int32_t n_agents,
                       const uint64_t *keys, const uint32_t *episodes, int32_t t, float epsilon,
                       int64_t *actions, int64_t *is_greedy, void *stream);

/* QMixer forward (hypernet_layers 1 or 2). */
typedef struct {
    const float *hw1_0w, *hw1_0b, *hw1_2w, *hw1_2b; /* hyper_w_1 (2 layers) or hyper_w_1 (1 layer: 0w/0b) */
    const float *hwf_0w, *hwf_0b, *hwf_2w, *hwf_2b;
    const float *hb1_w, *hb1_b;
    const float *v0_w, *v0_b, *v2_w, *v2_b;
    int32_t n_agents, state_dim, embed_dim, hypernet_embed, hypernet_layers;
} MlgQMixParams;
int mlg_qmix_forward(const MlgQMixParams *p, const float *agent_qs /*[R][N]*/, const float *states /*[R][S]*/,
                     float *q_tot /*[R]*/, int32_t R, void *stream);

/* ---- QLearner.train (q_learner.py:34-131) as one fused device pipeline --------------------------
 * Flat parameter vectors follow the nn.Module named_parameters() order:
 *   agent: fc1.weight [H][d_in], fc1.bias [H], gru.weight_ih [3H][H], gru.weight_hh [3H][H],
 *          gru.bias_ih [3H], gru.bias_hh [3H], fc2.weight [A][H], fc2.bias [A]
 *   qmix (hypernet_layers 2): hyper_w_1.{0.weight [HE][S], 0.bias, 2.weight [N*E][HE], 2.bias},
 *          hyper_w_final.{0.weight [HE][S], 0.bias, 2.weight [E][HE], 2.bias}, hyper_b_1.{weight [E][S], bias},
 *          V.{0.weight [E][S], 0.bias, 2.weight [1][E], 2.bias}
 * params/grads/square_avg = [agent | mixer]; target_params likewise (the target networks). */
typedef struct {
    int32_t B, T, N, A, d_obs, H, S, E, HE, hypernet_layers;
    int32_t mixer; /* 0 none (IQL), 1 vdn, 2 qmix */
    int32_t double_q, obs_last_action, obs_agent_id;
    float gamma, lr, optim_alpha, optim_eps, grad_norm_clip;
} MlgLearnerCfg;

typedef struct {
    MlgBatch batch;              /* the truncated sample: B episodes, T = max_t_filled timesteps (batch.T1 = stride) */
    float *params;               /* [n_agent + n_mixer] updated in place (RMSprop) */
    float *grads;                /* [n_agent + n_mixer] out: clipped gradients */
    float *square_avg;           /* [n_agent + n_mixer] RMSprop state */
    const float *target_params;  /* [n_agent + n_mixer] */
    float *workspace;            /* mlg_qlearner_workspace_floats() floats */
    float *stats;                /* [8] out: loss, grad_norm, td_error_abs, q_taken_mean, target_mean,
                                    mask_sum, count_nonzero(mask), 0 */
    /* optional (NULL = off), folded into the same launches instead of separate copies / adds: */
    float *target_sync;          /* [n_agent + n_mixer] receives the updated parameters (the target update
                                    q_learner.py:127-128 when it is due after this step; usually target_params) */
    double *trained_steps;       /* [1] += count_nonzero(mask) (Agent.trained_steps, q_learner.py:104) */
    const int32_t *host_rows;    /* HOST copy of the slot map (B <= 64): travels as a kernel argument,
                                    batch.rows is then ignored */
} MlgLearnerBufs;

int64_t mlg_qlearner_param_counts(const MlgLearnerCfg *c, int64_t *n_agent, int64_t *n_mixer);
int64_t mlg_qlearner_workspace_floats(const MlgLearnerCfg *c);
/* Largest batch (episodes) whose slot map may travel as MlgLearnerBufs.host_rows (a kernel argument). */
int mlg_qlearner_inline_rows(void);
int mlg_qlearner_train(const MlgLearnerCfg *c, const MlgLearnerBufs *b, void *stream);


/* ---- REFIL (config 5): entity scheme, EntityAttentionRNNAgent, FlexQMixer, REFILLearner ----------------- */
/* Entity env variant: base.U = 2S units, policy team 0 = units 0..S-1 (= the agents = entities
 * 0..S-1), scripted team 1 = S..2S-1; per episode k ~ U{min_agents..max_agents} active slots per team. */
typedef struct {
    MlgEnvSpec base;
    int32_t min_agents, max_agents;
} MlgEntityEnvSpec;

/* Entity-scheme EpisodeBatch, all [B][T1][...] row-major (REFIL scheme: no state / obs). */
typedef struct {
    float *entities;       /* [B][T1][NE][ED] */
    uint8_t *obs_mask;     /* [B][T1][NE][NE]  1 = entity not observable by the row entity */
    uint8_t *entity_mask;  /* [B][T1][NE]      1 = entity absent (padding) or dead */
    int64_t *actions;      /* [B][T1][NA][1] */
    int32_t *avail;        /* [B][T1][NA][A] */
    float *reward;         /* [B][T1][1] */
    uint8_t *terminated;   /* [B][T1][1] */
    float *actions_onehot; /* [B][T1][NA][A] */
    int64_t *filled;       /* [B][T1][1] */
    int32_t B, T1, ring_slot0, ring_size, full_write; /* as MlgBatch */
    const int32_t *rows;   /* sampled view (learner): episode b lives in slot rows[b]; nullptr = identity */
    int32_t *slot_extent;  /* as MlgBatch */
} MlgEntityBatch;

typedef struct {
    int32_t n_agents, n_entities, entity_shape, n_actions, entity_last_action;
    int32_t attn_embed_dim, attn_n_heads, rnn_hidden_dim;
} MlgRefilDims;

/* Packed EntityAttentionRNNAgent weights from the flat named_parameters() vector: fc1.weight [64][D0], fc1.bias,
 * attn.in_trans.weight [192][64], attn.out_trans.weight [64][64], attn.out_trans.bias, fc2.weight, fc2.bias,
 * rnn.weight_ih [192][64], rnn.weight_hh, rnn.bias_ih [192], rnn.bias_hh, fc3.weight [A][64], fc3.bias
 * (D0 = entity_shape + n_actions with entity_last_action). */
int64_t mlg_refil_packed_agent_size(const MlgRefilDims *d);
int mlg_refil_pack_agent(const MlgRefilDims *d, const float *flat, float *packed, void *stream);

/* One EntityAttentionRNNAgent.forward step (ts = 1) over R items: entities [R][NE][D0] (last-action one-hot
 * included), obs_mask [R][NE][NE], entity_mask [R][NE], h_in [R][NA][64] -> q [R][NA][A], h_out [R][NA][64]. */
int mlg_refil_agent_forward(const MlgRefilDims *d, const float *packed, const float *entities, const uint8_t *obs_mask,
                            const uint8_t *entity_mask, const float *h_in, float *q, float *h_out, int32_t R,
                            void *stream);

/* One ParallelStepper.run over the entity env with EntityMAC acting (entity_controller.py:11-30 with
 * t -> slice(t, t + 1); entity_rnn_agent.py:32-65; action_selectors.py:44-62). Same run semantics, ring /
 * full-write modes and run info as mlg_rollout. */
int mlg_refil_rollout(const MlgEntityEnvSpec *spec, MlgEnvState *st, const MlgRefilDims *d, const float *packed,
                      MlgEntityBatch *batch, MlgRunInfo *info, float epsilon, int32_t test_mode, void *stream);

/* EntityAttentionLayer.forward (src/marl/modules/layers/attention.py:24-79; in = embed = out = 64, 4 heads) over bs
 * items: x [bs][ne][64], pre_mask [bs][nq][ne], post_mask [bs][nq] (uint8, 1 = masked) -> y [bs][nq][64]. With
 * gy != nullptr also the backward of sum(y * gy): dx [bs][ne][64] written, dw_in [192][64], dw_out [64][64],
 * db_out [64] accumulated (atomic adds; caller zeroes). */
int mlg_refil_attention(const float *w_in, const float *w_out, const float *b_out, const float *x,
                        const uint8_t *pre_mask, const uint8_t *post_mask, int32_t bs, int32_t ne, int32_t nq,
                        int32_t n_heads, float *y, const float *gy, float *dx, float *dw_in, float *dw_out,
                        float *db_out, void *stream);

/* FlexQMixer (flex_qmix.py:55-117): packed = 4 AttentionHyperNet blocks from the flat named_parameters() vector
 * (hyper_w_1, hyper_w_final, hyper_b_1, V); forward over R rows: agent_qs [R][NA] (plain) or [R][2 NA] with the
 * imagine masks w_mask / i_mask [R][NE][NE] (both or neither), entities [R][NE][D0], entity_mask [R][NE]
 * -> q_tot [R]. softmax_mixing_weights selects softmax instead of abs mixing weights. */
int64_t mlg_refil_packed_mixer_size(const MlgRefilDims *d);
int mlg_refil_pack_mixer(const MlgRefilDims *d, const float *flat, float *packed, void *stream);
int mlg_refil_mixer_forward(const MlgRefilDims *d, const float *packed, const float *agent_qs, const float *entities,
                            const uint8_t *entity_mask, const uint8_t *w_mask, const uint8_t *i_mask,
                            int32_t softmax_mixing_weights, float *q_tot, int32_t R, void *stream);

/* REFILLearner.train (src/marl/learners/refil_learner.py:102-218) as one device pipeline: EntityMAC unrolls of the
 * plain / within / interact copies + target, FlexQMixer (flex_qmix.py:55-117) plain + imagined mixing, double-Q
 * targets, the lambda-mixed TD loss, all gradients, clip_grad_norm_ and RMSprop.
 * Flat parameters = [agent | mixer]; agent in named_parameters order (see mlg_refil_pack_agent); mixer =
 * hyper_w_1, hyper_w_final, hyper_b_1, V, each: fc1.weight [64][D0], fc1.bias, attn.in_trans.weight [192][64],
 * attn.out_trans.weight [64][64], attn.out_trans.bias, fc2.weight [32][64], fc2.bias [32]. */
typedef struct {
    int32_t B, T, n_agents, n_entities, entity_shape, n_actions, entity_last_action;
    int32_t attn_embed_dim, attn_n_heads, rnn_hidden_dim, hypernet_embed, mixing_embed_dim;
    int32_t double_q, softmax_mixing_weights, imagine;
    float gamma, lmbda, lr, optim_alpha, optim_eps, grad_norm_clip;
} MlgRefilLearnerCfg;

typedef struct {
    MlgEntityBatch batch;        /* B episodes, T timesteps used (batch.T1 = stride) */
    const uint8_t *groupA;       /* [B][NE] the imagine group draw per episode (entity_rnn_agent.py:95-97) */
    float *params;               /* [n_agent + n_mixer] updated in place (RMSprop) */
    float *grads;                /* [n_agent + n_mixer] out: clipped gradients */
    float *square_avg;           /* RMSprop state */
    const float *target_params;  /* target networks, same layout */
    float *workspace;            /* mlg_refil_workspace_floats() floats */
    float *stats;                /* [8] out: loss, im_loss, grad_norm, td_error_abs, q_taken_mean, target_mean,
                                    mask_sum, 0 */
    double *trained_steps;       /* optional [1] += mask_sum (Agent.trained_steps, refil_learner.py:176) */
    float *target_sync;          /* optional (NULL = off) [n_agent + n_mixer] receives the updated parameters in the
                                    optimizer launch: the target update when due after this step
                                    (refil_learner.py:181-183 -> _update_targets; usually target_params) */
    const int32_t *host_rows;    /* optional (NULL = off) HOST copy of the slot map (B <= mlg_qlearner_inline_rows()):
                                    travels as a kernel argument, batch.rows is then ignored */
} MlgRefilLearnerBufs;

int64_t mlg_refil_param_counts(const MlgRefilLearnerCfg *c, int64_t *n_agent, int64_t *n_mixer);
int64_t mlg_refil_workspace_floats(const MlgRefilLearnerCfg *c);
int mlg_refil_train(const MlgRefilLearnerCfg *c, const MlgRefilLearnerBufs *b, void *stream);
/* The imagine group draw of a train call (entity_rnn_agent.py:95-97: p_b = rand per episode, groupA[b][j] =
 * bernoulli(p_b)) on the device, counter-based from (seed, draw): one launch into groupA [B][NE]. */
int mlg_refil_draw_groups(int32_t B, int32_t NE, uint64_t seed, uint32_t draw, uint8_t *groupA, void *stream);

/* Diagnostic builds only (-DMLG_STAMPS): device buffer [grid][8 waves][16] u64 of per-phase cycle counts
 * of mlg_rollout. Returns nonzero in normal builds. */
int mlg_debug_set_stamps(void *ptr);
/* Diagnostic builds only (-DMLG_STAMPS): per-wave phase cycle counters of the learner recurrences. */
int mlg_debug_set_learner_stamps(void *ptr);
int mlg_refil_debug_set_stamps(void *ptr); /* same for mlg_refil_rollout: [grid][16] u64 */

/* League payoff bookkeeping of one batched self-play run (league_experiment_process.py:85-105, _extract_result +
 * _update_payoff per env): entry = the league's local payoff delta [GAMES, WIN, LOSS, DRAW, ...] of (home, away);
 * won [B][2] (policy team first), draw [B] as written by mlg_rollout_selfplay. DRAW if draw or both / no team won,
 * else WIN / LOSS by won[b][0]; GAMES += B when count_games (the reference never counts GAMES). One launch. */
int mlg_league_record_runs(const int32_t *won, const int32_t *draw, int32_t B, float *entry, int32_t count_games,
                           void *stream);

const char *mlg_last_error(void);
const char *mlg_version(void);

#ifdef __cplusplus
}
#endif
#endif
