/* asvrl.h -- C ABI of libasvrl.so, the MI355X (gfx950) kernels behind the rfarl training
 * hot path: the vectorised ASV marine-env step and the distributional Bellman update.
 *
 * The reference (pszenher/Distributional_RL_Decision_and_Control, rfarl/) is pure Python
 * and has no FFI; each entry point below replaces the Python function cited next to it
 * (paths relative to /root/reference/rfarl/rfarl/). The Python surfaces that call these
 * (MarineNavEnv3, Agent, Trainer) live in distributional_rl_decision_and_control_amd/ and
 * bind this header through ctypes (INTEGRATION.md shows the binding).
 *
 * Conventions
 *  - Every pointer argument is a DEVICE pointer unless its comment says "host".
 *    The caller owns all memory (allocated as torch tensors); the library keeps no state.
 *  - `stream` is a hipStream_t passed as void* (NULL = the default stream). All work is
 *    stream-ordered; no entry point synchronises the device.
 *  - Return value: 0 on success, nonzero on a bad argument or launch failure, with a
 *    thread-local message from asvrl_last_error(). No C++ exception crosses the ABI.
 *  - Two builds export this same header: libasvrl.so, whose learner kernels take bf16 MFMA
 *    operands (weight images, saved activations) with f32 accumulation, and libasvrl_f32.so,
 *    the same sources with every such operand f32 (the parity build). "bf16" in the comments
 *    below means the operand element type: f32 in libasvrl_f32.so (asvrl_operand_bytes()).
 */
#ifndef ASVRL_H
#define ASVRL_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ASVRL_ABI_VERSION 26

#define ASVRL_SELF_DIM 7   /* wamv.py:443-453 self observation */
#define ASVRL_OBJ_DIM 5    /* wamv.py:481,508 [px, py, vx, vy, r] */
#define ASVRL_MAX_OBJ 5    /* wamv.py:14 max_obj_num */
#define ASVRL_OBS_DIM 40   /* packed f32 obs row: self 7 | objects 5x5 | mask 5 | pad 3
                              (= replay_buffer.py:51-69 state_batch, padded to 16 B) */
#define ASVRL_TR_DIM 88    /* replay row: obs 40 | next obs 40 | action 2 | reward | done | pad 4 */
#define ASVRL_PER_DIM 48   /* prioritised replay slot: obs 40 | action | reward | nonterminal | timestep (i32) | pad 4 */

/* Robot state fields, field-major SoA: rs[f * (n_envs * max_robots) + e * max_robots + i] */
enum AsvRobotField {
  ASVRL_F_X = 0, ASVRL_F_Y, ASVRL_F_THETA,           /* wamv.py:92-94 */
  ASVRL_F_VR0, ASVRL_F_VR1, ASVRL_F_VR2,               /* velocity_r (wamv.py:95) */
  ASVRL_F_V0, ASVRL_F_V1, ASVRL_F_V2,                  /* velocity, one substep stale (:96) */
  ASVRL_F_TL, ASVRL_F_TR, ASVRL_F_LP, ASVRL_F_RP,      /* thrusts, thruster angles (:98-101) */
  ASVRL_F_GX, ASVRL_F_GY,                              /* goal (:129) */
  ASVRL_F_PHI,                                         /* COLREGs turn angle (:396) */
  ASVRL_F_RET,                                         /* discounted episode return (trainer.py:161) */
  ASVRL_NUM_FIELDS
};

/* Robot flag bits (u8 per robot) */
#define ASVRL_FLAG_DEACTIVATED 1u  /* wamv.py:132, written by trainer.py:168-170 */
#define ASVRL_FLAG_COLLISION 2u    /* wamv.py:130 */
#define ASVRL_FLAG_REACH_GOAL 4u   /* wamv.py:131 */
#define ASVRL_FLAG_COLREGS 8u      /* wamv.py:517-521 apply_COLREGs */

/* info codes of env.step (env.py:291-328) */
#define ASVRL_INFO_NORMAL 0
#define ASVRL_INFO_TOO_LONG 1
#define ASVRL_INFO_COLLISION 2
#define ASVRL_INFO_REACH_GOAL 3
#define ASVRL_INFO_DEACT_COLLISION 4
#define ASVRL_INFO_DEACT_GOAL 5
#define ASVRL_INFO_ABSENT 255      /* slot beyond the env's robot count */

/* Vehicle, perception and reward parameters (wamv.py:45-125, env.py:33-54). Passed by
 * value to the kernels; one set per env batch. */
typedef struct AsvParams {
  double dt;                 /* wamv.py:46 */
  int32_t N;                 /* wamv.py:47 substeps per action */
  int32_t episode_limit;     /* env.py:312 */
  double length, width;      /* wamv.py:51-52 */
  double r;                  /* collision radius = detect_r (wamv.py:53-54) */
  double goal_dis;           /* wamv.py:79 */
  double min_thrust, max_thrust; /* wamv.py:84-85 */
  double m, Izz;             /* wamv.py:103-104 */
  double xDotU, yDotV, yDotR, nDotR, nDotV, xU, xUU, yV, yVV, yR, yRV, yVR, yRR, nR, nRR, nV,
      nVV, nRV, nVR;         /* wamv.py:107-125 */
  double P[9];               /* inv(A^T A) A^T, A = M_RB + M_A (wamv.py:267-271), row-major,
                                computed on the host with the reference's numpy expression */
  double left_thrust_change[5], right_thrust_change[5]; /* wamv.py:86-88 discrete grid */
  double range, angle;       /* wamv.py:12-13 */
  double pos_std, vel_std, r_kappa, r_mean_ratio; /* wamv.py:22-25 */
  int32_t max_obj_num;       /* wamv.py:14 (<= ASVRL_MAX_OBJ) */
  int32_t _pad0;
  double timestep_penalty, COLREGs_penalty, collision_penalty, goal_reward; /* env.py:47-50 */
  double core_r;             /* env.py:35 vortex core radius */
} AsvParams;

/* A batch of E envs, resident in HBM. All arrays are caller-owned device memory. */
typedef struct AsvEnvState {
  int32_t n_envs, max_robots, max_obs, max_cores;
  double* rs;        /* [ASVRL_NUM_FIELDS][n_envs * max_robots] robot state (field-major SoA) */
  uint8_t* rflags;   /* [n_envs * max_robots] ASVRL_FLAG_* */
  int32_t* n_robots; /* [n_envs] robots placed by reset (<= max_robots; env.py:106-120 may place fewer) */
  int32_t* n_obs;    /* [n_envs] */
  int32_t* n_cores;  /* [n_envs] */
  int32_t* ep_ts;    /* [n_envs] episode_timesteps (env.py:64) */
  double* obstacles; /* [n_envs][max_obs][3] x, y, r (env.py:16-22) */
  double* cores;     /* [n_envs][max_cores][4] x, y, clockwise, Gamma (env.py:7-14) */
  const AsvParams* robot_params; /* optional [n_envs * max_robots]: each robot's own vehicle and
                                    perception parameters (reset_with_eval_config, env.py:553-607);
                                    NULL: `params` for every robot. The env-level members (episode
                                    limit, rewards, core radius) always come from `params`. Taken by the
                                    per-robot sweep layout (asvrl_env_step chooses it; layout 1 fails) */
} AsvEnvState;

/* Per-call control of asvrl_env_step. */
typedef struct AsvStepCtl {
  int32_t is_continuous;      /* env.step is_continuous_action (env.py:240) */
  int32_t do_dynamics;        /* 0: observation only (reset's get_observations, env.py:164) */
  int32_t trainer_deactivate; /* 1: apply trainer.py:157-172 in-kernel (deactivate on flags,
                                 episode-end test, discounted return) */
  int32_t noise_mode;         /* 0: injected draws (noise != NULL, parity with the reference's
                                 per-robot RandomState); 1: Philox-4x32-10 in registers, f64
                                 Box-Muller / von Mises; 2: Philox, f32 draws on the hardware
                                 transcendentals (the training path) */
  uint64_t seed, counter;     /* Philox key / per-step counter (noise_mode 1, 2) */
  const uint64_t* counter_dev; /* optional device counter added to `counter` (keeps a captured
                                  HIP graph drawing fresh noise on every replay) */
  double gamma;               /* discount for ASVRL_F_RET (trainer.py:161); 0 disables */
  const uint8_t* env_mask;    /* optional [n_envs]: only envs with mask != 0 are processed */
} AsvStepCtl;

/* Outputs of asvrl_env_step (device). Optional members may be NULL. */
typedef struct AsvStepOut {
  float* obs;        /* [n_envs*max_robots][ASVRL_OBS_DIM] packed f32 observation */
  double* obs64;     /* optional [n_envs*max_robots][32] f64 self(7)+objects(25) (compat path) */
  int8_t* obj_cnt;   /* [n_envs*max_robots] objects kept (0..5); -1 = (None, None) */
  double* reward;    /* [n_envs*max_robots] (env.py:242-328) */
  uint8_t* done;     /* [n_envs*max_robots] */
  uint8_t* info;     /* [n_envs*max_robots] ASVRL_INFO_* */
  uint8_t* env_done; /* optional [n_envs] trainer episode end (trainer.py:172) */
  double* stats;     /* optional [8] running sums over finished robot-episodes:
                        return, count, reach-goal, collision, timeout, env-episodes */
} AsvStepOut;

/* Reset parameters (env.py:33-54,72-164, curriculum values from the schedule). */
typedef struct AsvResetCfg {
  int32_t num_robots, num_obs, num_cores, _pad0;
  double min_start_goal_dis, width, height, clear_r;
  double obs_r_lo, obs_r_hi;       /* env.py:39 */
  double v_lo, v_hi;               /* env.py:38 core edge speed */
  double v_rel_max, p_rel;         /* env.py:36-37 */
} AsvResetCfg;

/* ---------------------------------------------------------------- env */

/* MarineNavEnv3.step (env.py:240-333) for every env of the batch in one launch: the N
 * Fossen substeps per robot (wamv.py:204-279, current field env.py:458-501), the sector
 * "LiDAR" object list with top-5 selection and collision test (wamv.py:436-529), COLREGs
 * (wamv.py:324-434) and reward/done/info (env.py:271-331).
 * actions: [n_envs*max_robots][2] f64; discrete actions pass the action index in [0].
 * noise (noise_mode 0): [n_envs*max_robots][max_obs + max_robots][5] f64 draws
 *   [n_px, n_py, n_vx, n_vy, vonmises] per candidate slot (slot k < max_obs: obstacle k,
 *   slot max_obs + j: robot j), in the order Perception makes them (wamv.py:27-40). */
int asvrl_env_step(const AsvParams* params, const AsvEnvState* state, const double* actions,
                   const double* noise, const AsvStepCtl* ctl, const AsvStepOut* out,
                   void* stream);

/* Launch shape of the env-step kernel (asvrl_env_step_ex). Zero members mean "choose":
 *   layout 0: automatic (pair-parallel perception when its LDS fits, else the per-robot sweep),
 *          1: pair-parallel (one lane per (robot, candidate) pair; fails if the LDS does not fit),
 *          2: per-robot sweep (one lane per robot, candidates in a serial loop);
 *   block  threads per workgroup of the pair layout (64, 128 or 256; 0: 256 lanes, or one wave from
 *          16384 envs when an env has at most 8 robots);
 *   envs_per_block  envs per workgroup of the pair layout (0: about 40 robots per group, about 120
 *          when an env has more than 8 robots). */
typedef struct AsvEnvLaunch {
  int32_t layout;
  int32_t block;
  int32_t envs_per_block;
  int32_t max_groups;   /* ABI 19: pair layout as launches of at most this many workgroups, one after another
                           (0 = one launch) -- the rollout's share of the chip beside a learner */
} AsvEnvLaunch;

/* asvrl_env_step with an explicit kernel shape (tests of every shipped layout, A/B tools);
 * launch == NULL is asvrl_env_step. Results do not depend on the shape. */
int asvrl_env_step_ex(const AsvParams* params, const AsvEnvState* state, const double* actions,
                      const double* noise, const AsvStepCtl* ctl, const AsvStepOut* out,
                      const AsvEnvLaunch* launch, void* stream);

/* MarineNavEnv3.reset (env.py:72-164) for envs with env_mask != 0, sampled on the device
 * with Philox (same rejection rules and iteration caps; not the reference's RandomState
 * stream -- the parity path resets on the host). Follow with asvrl_env_step(do_dynamics=0,
 * env_mask) to produce the reset observation. */
int asvrl_env_reset(const AsvParams* params, const AsvEnvState* state, const AsvResetCfg* cfg,
                    const uint8_t* env_mask, uint64_t seed, uint64_t counter,
                    const uint64_t* counter_dev, void* stream);

/* The training loop's auto-reset in ONE launch: for every env with env_mask[e] != 0, asvrl_env_reset's
 * sampler (one wave) followed by that env's reset observation, computed by the step kernel's phases with
 * ctl (do_dynamics = 0, env_mask = the same mask, Philox noise: noise_mode 1 or 2) into out -- the
 * same values as asvrl_env_reset + the masked asvrl_env_step, without the second launch over all envs.
 * Replaces, for the batched trainer, the reset() + get_observations() pair of MarineNavEnv3.reset
 * (env.py:72-164) that trainer.py calls at an episode end. Requires robot_params == NULL. */
int asvrl_env_reset_observe(const AsvParams* params, const AsvEnvState* state, const AsvResetCfg* cfg,
                            const uint8_t* env_mask, uint64_t seed, uint64_t counter,
                            const uint64_t* counter_dev, const AsvStepCtl* ctl, const AsvStepOut* out,
                            void* stream);

/* Ocean current of env.py:458-501 at n query points xy [n][2] for one env's cores
 * [n_cores][4] -> out [n][3]. Used for the initial velocity of reset_with_eval_config
 * (env.py:609-610); the step kernel evaluates the same field per substep. */
int asvrl_current_field(const double* cores, int32_t n_cores, double core_r, const double* xy,
                        int32_t n, double* out, void* stream);

/* ---------------------------------------------------------------- learner */

/* Quantile-Huber loss of agent.py:406-412 (+ calculate_huber_loss agent.py:701-707) and its
 * gradient w.r.t. the expected quantiles:
 *   delta[b,i,j] = qt[b,j] - qe[b,i]
 *   row_loss[b]  = (1/Np) sum_j sum_i |tau[b,i] - 1{delta<0}| * H_kappa(delta) / kappa
 *   loss[0]      = mean_b row_loss[b]
 *   dqe[b,i]     = grad_scale * d loss / d qe[b,i]
 * qt [B][Np], qe [B][N], tau [B][N] f32. loss may be NULL. */
int asvrl_quantile_huber(const float* qt, const float* qe, const float* tau, int32_t B, int32_t N,
                         int32_t Np, float kappa, float grad_scale, float* row_loss, float* loss,
                         float* dqe, void* stream);

/* C51 categorical projection of agent.py:616-631 (Tz, clamp, b, l/u with the l == u fix,
 * index_add_ of p(u - b) then p(b - l)), bit-identical to the reference's CPU f32 result.
 * pns_a [B][atoms], returns [B], nonterminal [B], support [atoms] -> m [B][atoms]. */
int asvrl_c51_project(const float* pns_a, const float* returns, const float* nonterminal,
                      const float* support, int32_t B, int32_t atoms, float vmin, float vmax,
                      float delta_z, float gamma_n, float* m, void* stream);
/* The same with returns[b * ld_ret] and nonterminal[b * ld_nt] (ABI 21): the columns of the replay rows
 * read in place (the Rainbow update's R^n and nonterminal columns, no copies). */
int asvrl_c51_project_ex(const float* pns_a, const float* returns, int64_t ld_ret, const float* nonterminal,
                         int64_t ld_nt, const float* support, int32_t B, int32_t atoms, float vmin, float vmax,
                         float delta_z, float gamma_n, float* m, void* stream);

/* ---------------------------------------------------------------- fused IQN critic (MFMA) */

/* Critic trunk weights of AC_IQN_model.py:392-408 (concat 256, hidden 128, 64 cosines), the
 * matrices pre-packed into bf16 MFMA A-operand fragments (64 lanes x 8 bf16 per
 * 32x32x16 fragment, in the k order the kernel's register chaining needs -- built by
 * critic_pack.py from the f32 nn.Linear weights). Biases / output row stay f32. */
typedef struct AsvCriticWeights {
  const void* wc_frag;   /* cos_embedding.weight  (256 x 64)  : 32 fragments */
  const void* w1_frag;   /* hidden_layer.weight   (128 x 256) : 64 fragments */
  const void* w2_frag;   /* hidden_layer_2.weight (128 x 128) : 32 fragments */
  const void* w2t_frag;  /* its transpose, for the backward   : 32 fragments */
  const void* w1t_frag;  /* hidden_layer.weight^T (256 x 128) : 64 fragments */
  const float* bc;       /* cos_embedding.bias [256] */
  const float* b1;       /* hidden_layer.bias [128] */
  const float* b2;       /* hidden_layer_2.bias [128] */
  const float* wo;       /* output_layer.weight [128] */
  const float* bo;       /* output_layer.bias [1] */
  /* f32 encoder parameters, read when an IO struct passes observation rows (obs != NULL): the
   * trunk kernels then compute F = observation_processor(obs) (AC_IQN_model.py:284-308,
   * IQN_model.py:80-96) and G = action_encoder(act) (AC_IQN_model.py:468-470) per sample in their
   * prologue instead of reading F / G. NULL when unused. */
  const float* self_w;   /* self_encoder.0.weight (56 x 7), .bias [56] */
  const float* self_b;
  const float* obj_w;    /* object_encoder.0.weight (40 x 5), .bias [40] */
  const float* obj_b;
  const float* ae_w;     /* action_encoder.0.weight (128 x 2), .bias [128] (AC-IQN critic only) */
  const float* ae_b;
} AsvCriticWeights;

/* bf16 row-major activations the TRAIN mode writes for the weight gradients
 * (dW = dZ^T X per layer), R = B*N rows. */
typedef struct AsvCriticActs {
  void* cos;   /* [R][64]   cos(tau pi k)            -> d cos_embedding.weight with dzc */
  void* h0;    /* [R][256]  F * c                    -> d hidden_layer.weight with dz1 */
  void* dzc;   /* [R][256]  dL/d(cos_embedding pre-activation) */
  void* h1g;   /* [R][128]  h1 * G                   -> d hidden_layer_2.weight with dz2 */
  void* dz1;   /* [R][128]  dL/d(hidden_layer pre-activation) */
  void* h2;    /* [R][128]  relu(hidden_layer_2)     -> d output_layer.weight with dq */
  void* dz2;   /* [R][128]  dL/d(hidden_layer_2 pre-activation) */
  float* dq;   /* [R]       dL/dq */
  float* wout_part; /* optional, AC-IQN TRAIN: [asvrl_critic_wout_groups(B, N)][129] per-workgroup
                       partials of output_layer's dW (128) | db, reduced in the kernel from f32 h2 and
                       dq (h2 and dq may then be NULL; reduce them with asvrl_partial_sums, nw 128, nb 1) */
} AsvCriticActs;

/* Number of [129] output-layer gradient partials asvrl_critic_train writes to acts->wout_part. */
int32_t asvrl_critic_wout_groups(int32_t B, int32_t N);

/* Fill the five bf16 fragment images of w (wc_frag .. w1t_frag) from the row-major f32
 * weights cos_embedding.weight (256 x 64), hidden_layer.weight (128 x 256) and
 * hidden_layer_2.weight (128 x 128) (AC_IQN_model.py:398-402). One launch. */
int asvrl_critic_pack(const float* wc, const float* w1, const float* w2, const AsvCriticWeights* w, void* stream);

/* Inputs / outputs of one critic launch. F (B x 256) = observation_processor features,
 * G (B x 128) = action_encoder features, taus (B x N); N in {8, 16, 32}. */
typedef struct AsvCriticIO {
  const float* F;          /* [B][256], or NULL with obs set */
  const float* G;          /* [B][128], or NULL with act set */
  const float* obs;        /* optional packed observation rows (ASVRL_OBS_DIM layout) at obs[b*ld_obs] */
  int64_t ld_obs;
  const float* act;        /* optional actions (2 f32) at act[b*ld_act] */
  int64_t ld_act;
  void* xb;                /* TRAIN optional: bf16 [B][32] copy of obs columns 0..31 (encoder wgrad operand) */
  const float* taus;
  int32_t B, N, Np;
  float kappa;
  const float* q_targets;  /* TRAIN: [B][Np], or NULL with q_next set: */
  const float* q_next;     /*   q_targets = rewards + gamma * q_next * (1 - dones) (agent.py:399-400) */
  const float* rewards;    /*   B values at stride ld_rd floats */
  const float* dones;
  int64_t ld_rd;
  float gamma;
  float dq;                /* ACTOR: dL/dq of every row (-1/(B*N) for actor_loss = -mean q) */
  float* q;                /* [B*N] (FWD: required) */
  float* row_loss;         /* TRAIN: [B*N], sums to B*Np*loss */
  float* dF;               /* TRAIN optional: dL/dF [B][256] */
  float* dG;               /* TRAIN / ACTOR optional: dL/dG [B][128] */
  void* dzF;               /* TRAIN optional: bf16 [B][256] dF * 1[F > 0] (encoder pre-activation grad) */
  float* dzG;              /* TRAIN optional: [B][128] dG * 1[G > 0] (action-encoder pre-activation grad) */
  const float* w_ae;       /* ACTOR with dA: action_encoder.weight [128][2] */
  float* dA;               /* ACTOR optional: dL/d(action) [B][2] = W_ae^T (dG * 1[G > 0]) */
  float* tile_loss;        /* optional [B*N/32]: per 32-row tile, TRAIN writes sum(row_loss) * loss_scale
                              (the critic loss with loss_scale = 1/(B*Np)), ACTOR sum(q) * loss_scale
                              (the actor loss with -1/(B*N)); sum them with asvrl_partial_sums
                              (a segment with nw = 1, groups = tiles) */
  float loss_scale;
} AsvCriticIO;

/* Critic.forward (AC_IQN_model.py:462-480): q [B*N]. */
int asvrl_critic_forward(const AsvCriticWeights* w, const AsvCriticIO* io, void* stream);

/* Critic update of train_AC_IQN (agent.py:395-414): forward, the quantile-Huber loss against
 * the targets and its backward in one launch; acts receive the activations for the weight
 * gradients. */
int asvrl_critic_train(const AsvCriticWeights* w, const AsvCriticIO* io, const AsvCriticActs* acts,
                       void* stream);

/* Per-workgroup weight-gradient partials of asvrl_critic_train_fused, [groups][M*K + M] per layer
 * (dW row-major in the layer's own feature order, then db); groups = asvrl_critic_fused_groups.
 * Sum them over the groups with asvrl_partial_sums (nw = M*K, nb = M, stride = M*K + M). */
typedef struct AsvCriticParts {
  float* cos_emb;   /* cos_embedding   (256 x 64): [groups][16384 + 256] */
  float* hidden;    /* hidden_layer    (128 x 256): [groups][32768 + 128] */
  float* hidden2;   /* hidden_layer_2  (128 x 128): [groups][16384 + 128] */
  float* out;       /* output_layer    (1 x 128):  [groups][128 + 1] */
  /* optional (ABI 16; asvrl_critic_train_fused only, NULL = not formed, then dzF / dzG / xb as
   * before): the encoders' gradients from the kernel's own per-sample dzF / dzG, without them
   * leaving the chip.
   * enc:  observation encoders, folded over the five objects (the contiguous layout of
   *       AC_IQN_model.py's self_encoder / object_encoder parameters):
   *       [groups][self_w 56x7 | self_b 56 | obj_w 40x5 | obj_b 40] = [groups][688]
   * aenc: action encoder (2 -> 128): [groups][w 128x2 | b 128] = [groups][384] */
  float* enc;
  float* aenc;
} AsvCriticParts;

/* Workgroups (= partial groups) of asvrl_critic_train_fused for B samples x N quantiles: one per
 * CU at most, each taking rounds of 64 rows (32 in the f32 build). */
int32_t asvrl_critic_fused_groups(int32_t B, int32_t N);

/* The critic update of train_AC_IQN (agent.py:395-414) WITH its trunk weight gradients, in one
 * persistent launch: encoders from io->obs / io->act, forward, quantile-Huber loss against
 * r + gamma q_next (1 - d) (io->q_next [B][N], rewards / dones at stride ld_rd), backward, and
 * per-workgroup dW / db partials of the four trunk layers (parts); per-sample dzF / dzG and xb for
 * the encoder gradients, per-tile loss partials (tile_loss) as asvrl_critic_train. N' must equal N;
 * B*N a multiple of the round size. No activation goes to HBM. */
int asvrl_critic_train_fused(const AsvCriticWeights* w, const AsvCriticIO* io, const AsvCriticParts* parts,
                             void* stream);

/* asvrl_critic_train_fused with the target critic's forward in the same launch (ABI 20; replaces the
 * separate asvrl_critic_forward(target) of train_AC_IQN, agent.py:396-400): each workgroup first computes
 * q_next = Critic_target(tio->obs, tio->act, tio->taus) (AC_IQN_model.py:462-480) for exactly the samples
 * its rounds update into io->q_next, then runs the update reading them. tw: the target critic (with its
 * encoders); tio: B and N as io. With kernel variant 4 (asvrl_critic_fused_variant) the target pass is
 * asvrl_critic_forward's own tile: q_next bit for bit what asvrl_critic_forward(tw, tio) gives; with variant 8
 * (the default where it applies) it is the update kernel's own forward phases: the same rounding points, f32 sums
 * in another order. */
int asvrl_critic_train_fused_tq(const AsvCriticWeights* w, const AsvCriticIO* io, const AsvCriticParts* parts,
                                const AsvCriticWeights* tw, const AsvCriticIO* tio, void* stream);

/* ABI 23: the kernel asvrl_critic_train_fused(_tq) launch where both forms take the shape (bf16 build, N = 32,
 * parts->enc and parts->aenc set, no dzF / dzG / xb): 8 = two waves per SIMD (512-thread workgroups), 4 = one
 * wave per SIMD (the round-5 kernel; the default: variant 8 measured 11 % slower). Results
 * agree within f32 summation order, not bit for bit.
 * v < 0 only queries; returns the previous setting, or -1 (asvrl_last_error) for any other v. Process-wide. */
int32_t asvrl_critic_fused_variant(int32_t v);

/* Actor update's critic pass (agent.py:419-425): forward, then the backward of
 * sum_rows dq * q to G (dG) and through the action encoder to the action (dA). */
int asvrl_critic_actor_grad(const AsvCriticWeights* w, const AsvCriticIO* io, void* stream);

/* ---------------------------------------------------------------- IQN (IQN_model.py, agent.py:227-256, 434-476) */

/* IQN_Policy has the critic's trunk without the action encoder (h1 feeds hidden_layer_2
 * directly, IQN_model.py:106-108) and an output_layer 128 -> A (A <= 32 actions). Its trunk
 * uses AsvCriticWeights (wo / bo unused); the head is described here. */
#define ASVRL_IQN_MAX_ACTIONS 32
typedef struct AsvIqnHead {
  const void* wo_frag;  /* output_layer.weight padded to 32 x 128, chained fragment order: 8 fragments */
  const float* wo;      /* output_layer.weight [A][128] f32 (the TRAIN backward) */
  const float* bo;      /* output_layer.bias [A] */
  int32_t n_actions;    /* A */
} AsvIqnHead;

/* Pack the trunk images (as asvrl_critic_pack) and the head image in one launch. */
int asvrl_iqn_pack(const float* wc, const float* w1, const float* w2, const float* wout,
                   const AsvCriticWeights* w, const AsvIqnHead* head, void* stream);

/* Inputs / outputs of one IQN launch. Rows are (sample b, tau n), R = B*N. */
typedef struct AsvIqnIO {
  const float* F;          /* [B][256] observation features, or NULL with obs set */
  const float* obs;        /* optional packed observation rows at obs[b*ld_obs] (encoders in-kernel) */
  int64_t ld_obs;
  void* xb;                /* TRAIN optional: bf16 [B][32] copy of obs columns 0..31 */
  const float* taus;       /* [B*N]; ACT: may be NULL = drawn in the kernel (Philox, uniform [0,1)) */
  int32_t B, N, Np;        /* N in {8,16,32} (ACT: N = K = 32); Np = target quantiles per sample (TRAIN) */
  float kappa;             /* Huber threshold (1.0, agent.py:458) */
  const float* q_next;     /* TRAIN: [B][Np] max over actions of the target quantiles (asvrl_iqn_forward_max) */
  const float* actions;    /* TRAIN: action index of sample b at actions[b*ld_rd] (f32, replay row column) */
  const float* rewards;    /* TRAIN: rewards[b*ld_rd] */
  const float* dones;      /* TRAIN: dones[b*ld_rd] */
  int64_t ld_rd;
  float gamma;
  float* q;                /* FORWARD_MAX: [R] max_a Q(row, a); TRAIN optional: [R] Q(row, a_b) */
  float* row_loss;         /* TRAIN optional: [R] sum over target quantiles of the quantile-Huber term */
  void* dzF;               /* TRAIN: bf16 [B][256] dL/dF * 1[F > 0] (encoder pre-activation grad) */
  void* dz_out;            /* TRAIN: bf16 [R][32] dL/d(output pre-activation): dq at the taken action, else 0 */
  float* tile_loss;        /* TRAIN optional: [R/32] per-tile sum(row_loss) * loss_scale */
  float loss_scale;
  /* ACT (act_iqn, agent.py:227-256): action = argmax_a mean_n Q(b, n, a), epsilon-greedy */
  double* act_out;         /* [B] action index as f64 at act_out[b*ld_act] */
  int64_t ld_act;
  const int64_t* step_dev; /* device step counter for the epsilon schedule and the RNG counter */
  double eps_steps_per_count, eps_total, eps_fraction, eps_initial, eps_final;
  uint64_t seed;
} AsvIqnIO;

/* Target pass of train_IQN (agent.py:451-452): q[row] = max_a Q(row, a). */
int asvrl_iqn_forward_max(const AsvCriticWeights* w, const AsvIqnHead* head, const AsvIqnIO* io, void* stream);

/* Local pass of train_IQN (agent.py:455-468): forward, gather at the taken action, the
 * quantile-Huber loss against r + gamma * q_next * (1 - d), and the whole trunk backward
 * (two launches). acts: h1g holds h1; dq is optional. */
int asvrl_iqn_train(const AsvCriticWeights* w, const AsvIqnHead* head, const AsvIqnIO* io,
                    const AsvCriticActs* acts, void* stream);

/* train_IQN's local pass (agent.py:455-468) WITH the trunk and output-layer weight gradients, in
 * one persistent launch (asvrl_critic_train_fused's kernel on IQN_Policy's trunk): encoders from
 * io->obs, forward, gather at io->actions, quantile-Huber loss, backward, per-workgroup partials
 * (parts; parts->out is [groups][32*128 + 32], output rows >= A zero), dzF / xb / tile_loss.
 * dz_out is not written; N' must equal N; groups = asvrl_critic_fused_groups(B, N). */
int asvrl_iqn_train_fused(const AsvCriticWeights* w, const AsvIqnHead* head, const AsvIqnIO* io,
                          const AsvCriticParts* parts, void* stream);
/* ABI 24: the same launch with train_IQN's target (agent.py:451-452: qnetwork_target(next_states, taus').max over
 * the actions) computed inside it first: each workgroup forms q_next for exactly the samples it updates (the
 * IQN_MAX tile of asvrl_iqn_forward_max, bit-identical) into io->q_next, then the update reads it. tw / thead:
 * the target network's images and head; tio: taus (the target's tau'), obs (next-observation rows), B and N as
 * io. Replaces asvrl_iqn_forward_max + asvrl_iqn_train_fused. */
int asvrl_iqn_train_fused_tq(const AsvCriticWeights* w, const AsvIqnHead* head, const AsvIqnIO* io,
                             const AsvCriticParts* parts, const AsvCriticWeights* tw, const AsvIqnHead* thead,
                             const AsvIqnIO* tio, void* stream);

/* act_iqn (agent.py:227-256) for every row of F with K = 32 quantile samples per state. */
int asvrl_iqn_act(const AsvCriticWeights* w, const AsvIqnHead* head, const AsvIqnIO* io, void* stream);

/* ---------------------------------------------------------------- replay (replay_buffer.py) */

/* ReplayBuffer.add (replay_buffer.py:22-24) for every robot that acted in the last step
 * (obj_cnt_next >= 0), in slot order, into a ring of `capacity` rows of ASVRL_TR_DIM f32.
 * ring_state: int64[2] = {head, size} in device memory (updated by the call, so the call
 * is capturable in a HIP graph). work: int32[ceil(n / 256) + 1] scratch, ZERO before the first call
 * (work[0] is the launch's arrival counter, work[1] the blocks' running row count; the call leaves both zero
 * again). One launch. */
int asvrl_replay_push(const float* obs_prev, const float* obs_next, const int8_t* obj_cnt_next,
                      const double* actions, int32_t action_dim, const double* reward,
                      const uint8_t* done, int32_t n, float* ring, int64_t capacity,
                      int64_t* ring_state, int32_t* work, void* stream);
/* asvrl_replay_push with actions rows action_ld doubles apart (the first action_dim used) that also
 * writes the new {head, size} to `snap` (int64[2], optional: the ring snapshot a concurrent learner
 * samples against) and increments *counter_inc (optional: the env step counter), in the same launch
 * (ABI 18). */
int asvrl_replay_push_ex(const float* obs_prev, const float* obs_next, const int8_t* obj_cnt_next,
                         const double* actions, int32_t action_dim, int64_t action_ld, const double* reward,
                         const uint8_t* done, int32_t n, float* ring, int64_t capacity,
                         int64_t* ring_state, int32_t* work, int64_t* snap, int64_t* counter_inc,
                         void* stream);

/* ReplayBuffer.sample (replay_buffer.py:26-45): gather B rows. With `indices` (host-chosen,
 * deque order: 0 = oldest) the rows are exactly those; with indices == NULL, B positions are
 * drawn uniformly (with replacement) by Philox(seed, counter + *counter_dev), skipping the
 * oldest entries that a push of up to `guard` rows running concurrently could overwrite
 * (guard = 0: none). ring_state may be a snapshot {head, size} taken before that push.
 * out [B][ASVRL_TR_DIM]; out_slots optional [B]. taus (optional): tau_sets x [B][tau_n] quantile
 * fractions U[0, 1) for the update (the torch.rand of AC_IQN_model.py:419 / IQN_model.py:62), drawn
 * from Philox(seed, counter + *counter_dev) in the same launch. */
int asvrl_replay_sample(const float* ring, int64_t capacity, const int64_t* ring_state,
                        const int64_t* indices, int32_t B, uint64_t seed, uint64_t counter,
                        const uint64_t* counter_dev, int64_t guard, float* out, int64_t* out_slots,
                        float* taus, int32_t tau_sets, int32_t tau_n, void* stream);

/* Host-side index copy helper for a ring with known (host) head/size: write rows given by
 * slot into the ring (used by the compat ReplayBuffer.add, one transition per call). */
int asvrl_replay_write_rows(const float* rows, const int64_t* slots, int32_t n, float* ring,
                            void* stream);

/* ---------------------------------------------------------------- prioritised n-step replay
 * Rainbow's ReplayMemory + SegmentTree (policy/replay_memory_rainbow.py:14-196) in HBM. All members
 * are device pointers the caller allocates (zero-initialised, maxp[0] = 1.0f); the struct itself is
 * read on the host at each call. */
typedef struct AsvPer {
  float* rows;          /* [capacity][ASVRL_PER_DIM] */
  float* tree;          /* [2 * tree_leaves - 1] sum tree, leaves at tree_leaves - 1 (:17) */
  int64_t* state;       /* [4] {index, full, reserved, anomaly count (rejections left after 64 redraws,
                           unsorted priority updates)} */
  int32_t* t;           /* [stride] per-stream timestep counter (ReplayMemory.t, :107,139) */
  float* maxp;          /* [1] SegmentTree.max (:22) */
  uint8_t* dirty;       /* [max(1, tree_leaves / 2048)] dirty 2048-leaf blocks (cleared by the rebuild) */
  int64_t capacity;     /* slots, a multiple of stride */
  int64_t tree_leaves;  /* next power of two >= capacity, <= 2^22 */
  int32_t stride;       /* slots per time step: 1 = the reference's single sequence; E*R = one stream per robot */
  int32_t n_step;       /* n (3, :105) */
  double discount;      /* 0.99 (:104) */
  float priority_weight;    /* beta 0.4 (:106) */
  float priority_exponent;  /* omega 0.5 (:107) */
  int32_t deferred;     /* 0: the reference's tree (every append at max priority, rejection sampling);
                           1: a slot's priority enters the tree when its n-step window is complete */
  int32_t _pad0;
} AsvPer;

/* ReplayMemory.append (:132-139) for n = m * stride rows (m time steps, rows time-major): robot
 * k % stride appends obs[k] (packed ASVRL_OBS_DIM row), action actions[k*action_dim], reward[k],
 * terminal done[k] at max priority when obj_cnt[k] >= 0, else a blank slot of priority 0 (deferred: the
 * priority is kept in the slot and set on the leaf n steps later, when the window is complete); then
 * the dirty subtrees are rebuilt and the ring advances by n. Three launches. */
int asvrl_per_push(const AsvPer* per, const float* obs, const int8_t* obj_cnt, const double* actions,
                   int32_t action_dim, const double* reward, const uint8_t* done, int32_t n, void* stream);
/* ABI 25: the same, and the device env-step counter step_counter[0] (int64) advanced by one in its last launch
 * (the batched loop's step count, trainer.py:172; NULL: not advanced) */
int asvrl_per_push_ex(const AsvPer* per, const float* obs, const int8_t* obj_cnt, const double* actions,
                      int32_t action_dim, const double* reward, const uint8_t* done, int32_t n, int64_t* step_counter,
                      void* stream);

/* ReplayMemory.sample (:157-192): B stratified draws (segment b: uniform in [b*seg, (b+1)*seg) with
 * seg = total / B in f32, the value in f64), SegmentTree.find, the validity rule of :163 (window
 * behind the write head, not the head slot, prob != 0), the n-step window with blanking at later
 * episode starts. uniforms (device f64 [B], optional): the reference's U(0,1) draws, one attempt;
 * otherwise Philox(seed, counter + *counter_dev) with up to 64 per-segment redraws.
 * out [B][ASVRL_TR_DIM]: obs 40 | n-th next obs 40 | action, 0 | R^n | nonterminal |
 * w = (cap * p)^-beta (before the batch-max normalisation) | p = prob / total | data index | 0.
 * out_tree_idx [B] int64: tree indices for asvrl_per_update. One launch. */
int asvrl_per_sample(const AsvPer* per, int32_t B, const double* uniforms, uint64_t seed, uint64_t counter,
                     const uint64_t* counter_dev, float* out, int64_t* out_tree_idx, void* stream);
/* ABI 25: the same, and each draw's weight also into weights[B] (contiguous, for asvrl_per_normalise). */
int asvrl_per_sample_ex(const AsvPer* per, int32_t B, const double* uniforms, uint64_t seed, uint64_t counter,
                        const uint64_t* counter_dev, float* out, int64_t* out_tree_idx, float* weights, void* stream);
/* ABI 25: weights / weights.max() (:191) into the weight column (84) of asvrl_per_sample_ex's B rows, from its
 * contiguous weights, in one launch (the quotients of the reference's expression bit for bit). */
int asvrl_per_normalise(float* rows, const float* weights, int32_t B, void* stream);

/* ReplayMemory.update_priorities (:194-196): leaf tree_idx[i] = values[i] ** priority_exponent
 * (raw != 0: values already exponentiated), duplicates resolved last-wins (tree_idx as sampled, in
 * non-decreasing order), SegmentTree.max updated, dirty subtrees rebuilt. Three launches. */
int asvrl_per_update(const AsvPer* per, const int64_t* tree_idx, const float* values, int32_t B, int32_t raw,
                     void* stream);
/* ABI 25: the same, and in its last launch values_mean[0] = the mean of values (a fixed summation order; the
 * train step's reported loss, agent.py:639) and learn_counter[0] (int64) += 1; either may be NULL. */
int asvrl_per_update_ex(const AsvPer* per, const int64_t* tree_idx, const float* values, int32_t B, int32_t raw,
                        float* values_mean, int64_t* learn_counter, void* stream);

/* ---------------------------------------------------------------- Rainbow (Rainbow_model.py, agent.py)
 * NoisyLinear weights and the dueling C51 head. A network's noisy tensors are described by up to 16
 * segments (weight, bias of each layer); off[k] is the flat offset of segment k (off[n] = total). */
#define ASVRL_MAX_NOISY_SEGS 16
typedef struct AsvNoisySeg {
  const float* mu;      /* weight_mu / bias_mu */
  const float* sigma;   /* weight_sigma / bias_sigma */
  float* eps;           /* weight_epsilon / bias_epsilon (written by asvrl_noisy_reset) */
  float* out;           /* composed mu + sigma * eps */
  const float* dout;    /* backward: gradient of out */
  float* dmu;           /* backward: written with dout */
  float* dsigma;        /* backward: written with dout * eps */
} AsvNoisySeg;

typedef struct AsvNoisySegs {
  int32_t n;
  int32_t _pad0;
  int64_t off[ASVRL_MAX_NOISY_SEGS + 1];
  AsvNoisySeg seg[ASVRL_MAX_NOISY_SEGS];
} AsvNoisySegs;

/* NoisyLinear.forward in training mode (Rainbow_model.py:47-51) for every segment: out = mu + sigma * eps;
 * backward != 0: dmu = dout, dsigma = dout * eps (assigned, the parameters' only use). One launch. */
int asvrl_noisy_compose(const AsvNoisySegs* segs, int32_t backward, void* stream);
/* ABI 26: the backward of asvrl_noisy_compose that also leaves the squared norm of the gradients it writes
 * (dmu^2 + dsigma^2) as asvrl_noisy_backward_norm_parts(segs) f64 per-workgroup partials in sq_parts (a fixed
 * order): with the reduction's own partials (asvrl_partial_sums_norm) the clip norm of asvrl_adam_step. */
int32_t asvrl_noisy_backward_norm_parts(const AsvNoisySegs* segs);
int asvrl_noisy_backward_norm(const AsvNoisySegs* segs, double* sq_parts, void* stream);

/* reset_noise() of every layer (Rainbow_model.py:35-45,141-145) with (weight, bias) segment pairs:
 * f(x) = sign(x) sqrt|x| of N(0, 1) Philox draws (seed, *counter_dev), eps_w = f(eps_out) f(eps_in)^T,
 * eps_b = f(eps_out), and out = mu + sigma * eps in the same launch. in/out_features: HOST int32
 * [n/2] (in <= 256). One workgroup per 16 output units. */
int asvrl_noisy_reset(const AsvNoisySegs* segs, const int32_t* in_features, const int32_t* out_features,
                      uint64_t seed, const int64_t* counter_dev, void* stream);

typedef struct AsvRainbowHeadIO {
  const float* v;           /* [N][ldv] value logits (51) */
  int64_t ldv;
  const float* a;           /* [N][lda] advantage logits (25 x 51, action-major) */
  int64_t lda;
  int32_t N, atoms, actions_n, _pad0;   /* atoms 51, actions_n 25 */
  const float* support;     /* [51] */
  /* act: argmax_a sum softmax(q[a]) z (agent.py:320), epsilon-greedy when step_dev != NULL */
  double* act_out;          /* optional [N] action as f64 at act_out[row * ld_act] */
  int64_t ld_act;
  int64_t* act_idx;         /* optional [N] greedy action (act) / a* input (pick) */
  const int64_t* step_dev;
  double eps_steps_per_count, eps_total, eps_fraction, eps_initial, eps_final;
  uint64_t seed;
  float* p_out;             /* pick: [N][51] softmax(q[a*]) */
  /* loss */
  const float* actions;     /* [N] at actions[row * ld_rd] (replay row column) */
  const float* weights;     /* [N] importance weights at weights[row * ld_rd] */
  int64_t ld_rd;
  const float* m;           /* [N][51] projected target distribution */
  float* loss;              /* [N] per-sample loss */
  float* dv;                /* [N][51] d(grad_scale * sum_b w_b loss_b) / dv */
  float* da;                /* [N][1275] ... / da */
  float grad_scale;         /* 1 / B for the mean */
  int32_t _pad1;
} AsvRainbowHeadIO;

/* Dueling head q = v + a - mean_a(a) (Rainbow_model.py:128-134) per row: softmax over atoms per action,
 * expected value, argmax (first maximum); epsilon-greedy exploration (agent.py:318-322) with the linear
 * schedule of the device step counter when step_dev != NULL. One wave per two rows. */
int asvrl_rainbow_act(const AsvRainbowHeadIO* io, void* stream);
/* p(s', a*) = softmax(q[a*]) (agent.py:611-612), a* = act_idx[row]. One wave per row. */
int asvrl_rainbow_pick(const AsvRainbowHeadIO* io, void* stream);
/* loss_b = -sum m log softmax(q[a_b]) (agent.py:633) and the gradients of grad_scale * sum_b w_b loss_b
 * with respect to v and a. One wave per row. */
int asvrl_rainbow_loss(const AsvRainbowHeadIO* io, void* stream);

/* Rainbow_Policy (Rainbow_model.py:56-139) as one kernel per 32-row tile: encoders, both streams, the
 * dueling combine and the C51 head, bf16 MFMA operands (f32 in libasvrl_f32.so). The weights are
 * fragment images packed from the COMPOSED NoisyLinear weights (asvrl_noisy_compose / _reset, then
 * asvrl_rainbow_pack), including the action-mean of output_layer_a (mean_k a[k] as one more layer). */
typedef struct AsvRainbowSrc {   /* f32 row-major [out][in] */
  const float *self_w, *self_b, *obj_w, *obj_b;            /* self_encoder.0 (56 x 7), object_encoder.0 (40 x 5) */
  const float *w_v1, *b_v1, *w_a1, *b_a1;                  /* hidden_layer_v / _a (128 x 256), composed */
  const float *w_v2, *b_v2, *w_a2, *b_a2;                  /* hidden_layer_v_2 / _a_2 (128 x 128) */
  const float *w_vo, *b_vo, *w_ao, *b_ao;                  /* output_layer_v (51 x 128), output_layer_a (1275 x 128) */
} AsvRainbowSrc;

/* The packed images (operand element type; biases f32). Sizes in elements: enc 8192, v1 / a1 32768,
 * v2 / a2 16384, vo / mo 8192, ao 204800; b_enc 256, b_v1p .. b_a2p 128, b_vop / b_mop 64, b_aop 1600.
 * The backward's transposed images (train only; may be NULL otherwise): vot / mot 8192 (mot holds
 * -mean_k), aot 204800, v2t / a2t 16384, v1t / a1t 32768. */
typedef struct AsvRainbowImgOut {
  void *enc, *v1, *a1, *v2, *a2, *vo, *mo, *ao;
  float *b_enc, *b_v1p, *b_a1p, *b_v2p, *b_a2p, *b_vop, *b_mop, *b_aop;
  void *vot, *mot, *aot, *v2t, *a2t, *v1t, *a1t;
} AsvRainbowImgOut;
typedef struct AsvRainbowImg {   /* the same buffers, read-only */
  const void *enc, *v1, *a1, *v2, *a2, *vo, *mo, *ao;
  const float *b_enc, *b_v1p, *b_a1p, *b_v2p, *b_a2p, *b_vop, *b_mop, *b_aop;
  const void *vot, *mot, *aot, *v2t, *a2t, *v1t, *a1t;
} AsvRainbowImg;

typedef struct AsvRainbowNetIO {
  const float* x;           /* [N] packed observation rows at x[row * ldx] (16-byte aligned, ldx >= 40) */
  int64_t ldx;
  int32_t N, _pad0;
  const float* support;     /* [51] */
  double* act_out;          /* act: [N] action as f64 at act_out[row * ld_act] */
  int64_t ld_act;
  int64_t* act_idx;         /* argmax: [N] greedy action out; pick: a* in; act: optional greedy out */
  const int64_t* step_dev;  /* act: epsilon schedule on the device step counter (NULL: greedy) */
  double eps_steps_per_count, eps_total, eps_fraction, eps_initial, eps_final;
  uint64_t seed;
  float* p_out;             /* pick: [N][51] softmax(q[a*]) */
  /* train (agent.py:613-636): loss and backward of mean_b w_b loss_b on the rows x (= s) */
  const float* actions;     /* [N] taken action at actions[row * ld_rd] (replay row column) */
  const float* weights;     /* [N] importance weights at weights[row * ld_rd] */
  int64_t ld_rd;
  const float* m;           /* [N][51] projected target distribution (asvrl_c51_project) */
  float grad_scale;         /* 1 / B */
  int32_t _pad1;
  float* loss;              /* [N] -sum m log softmax(q[a_b]) */
  /* saved activations (operand type, row-major, natural feature order): the weight-gradient inputs */
  void *xb, *f, *hv1, *ha1, *hv2, *ha2;   /* [N][32], [N][256], [N][128] x 4 */
  /* pre-activation gradients (operand type): dz of output_layer_v [N][64] (51 + zero pad), of
   * output_layer_a [N][1280] (1275 + zero pad), of the hidden layers [N][128] x 4, of the encoders [N][256] */
  void *dzv, *dza, *dz2v, *dz2a, *dz1v, *dz1a, *dzf;
} AsvRainbowNetIO;

/* Pack the encoders and composed noisy layers into AsvRainbowImgOut (one launch). */
int asvrl_rainbow_pack(const AsvRainbowSrc* src, const AsvRainbowImgOut* img, void* stream);
/* act_rainbow (agent.py:308-324) for every row: argmax_k sum softmax(q[k]) z, epsilon-greedy. */
int asvrl_rainbow_net_act(const AsvRainbowImg* w, const AsvRainbowNetIO* io, void* stream);
/* The double-Q argmax of train_Rainbow (agent.py:605-609): act_idx[row] = argmax_k Q[k]. */
int asvrl_rainbow_net_argmax(const AsvRainbowImg* w, const AsvRainbowNetIO* io, void* stream);
/* p(s', a*) of the target net (agent.py:610-612): p_out[row] = softmax(q[act_idx[row]]). */
int asvrl_rainbow_net_pick(const AsvRainbowImg* w, const AsvRainbowNetIO* io, void* stream);
/* The training pass of train_Rainbow (agent.py:613-636) on the online net: forward saving the
 * activations, loss_b = -sum m log softmax(q[a_b]), and the backward of grad_scale * sum_b w_b loss_b
 * down to the encoders' pre-activations (the weight gradients then come from asvrl_linear_wgrad_multi
 * over the saved activations / dz images, the encoders' by the fold). */
int asvrl_rainbow_net_train(const AsvRainbowImg* w, const AsvRainbowNetIO* io, void* stream);

/* ---------------------------------------------------------------- optimiser (agent.py) */

/* clip_grad_norm_(params, max_norm) followed by optim.Adam(lr, betas, eps).step() over one
 * flat f32 parameter buffer of n elements (agent.py:75-76,98 with the clips at
 * agent.py:415,426,471,636). grads are scaled in place by min(1, max_norm / (norm + 1e-6))
 * (max_norm <= 0: no clipping); *step (f32, device) is incremented before the bias
 * corrections are taken; norm_out (f32 device scalar, optional) receives the pre-clip global
 * norm that clip_grad_norm_ returns. work: >= 64 doubles of device scratch. Two launches,
 * no host synchronisation (capturable). */
int asvrl_adam_clip(float* params, float* grads, float* exp_avg, float* exp_avg_sq, int64_t n,
                    float* step, float lr, float beta1, float beta2, float eps, float max_norm,
                    float* norm_out, double* work, void* stream);

/* The second half of asvrl_adam_clip alone: clip + Adam with the squared norm given as nparts
 * f64 partial sums (asvrl_partial_sums_norm; every workgroup folds them in the same fixed order)
 * and *step already incremented. One launch. */
int asvrl_adam_step(float* params, float* grads, float* exp_avg, float* exp_avg_sq, int64_t n,
                    const float* step, float lr, float beta1, float beta2, float eps, float max_norm,
                    float* norm_out, const double* norm_parts, int32_t nparts, void* stream);

/* asvrl_adam_step that also writes every updated parameter into the bf16 MFMA weight images (ABI v10;
 * replaces the asvrl_critic_pack / asvrl_mlp_pack / asvrl_iqn_pack launch after the step, same values).
 * Segment: the rows x cols row-major weight at params[flat_off...]; element (r, c) goes to image position
 * (row0 + r + q*rep_row, col0 + c + q*rep_col) for q < nrep, swapped if transposed; f32 = 1 writes
 * image[row] as f32 (a bias copy, cols = 1), otherwise the bf16 fragment image of K columns (chained = 1:
 * an accumulator-fed layer's order). counter (optional): incremented once by the launch. */
#define ASVRL_MAX_PACK_SEGS 16
typedef struct AsvPackSeg {
  int64_t flat_off;
  void* image;
  int32_t rows, cols, K, chained;
  int32_t transposed, f32, row0, col0;
  int32_t nrep, rep_row, rep_col, reserved;
} AsvPackSeg;
int asvrl_adam_step_pack(float* params, float* grads, float* exp_avg, float* exp_avg_sq, int64_t n,
                         const float* step, float lr, float beta1, float beta2, float eps, float max_norm,
                         float* norm_out, const double* norm_parts, int32_t nparts, const AsvPackSeg* segs,
                         int32_t nseg, int64_t* counter, void* stream);

/* ---------------------------------------------------------------- Linear weight gradients */

/* grad_weight / grad_bias of an nn.Linear from bf16 activations over R rows (the backward's
 * dW = dZ^T X, db = dZ.sum(0), AC_IQN_model.py:398-404 layers): dw[m][k] = sum_r dz[r][m] x[r][k],
 * db[m] = sum_r dz[r][m] (db optional). dz (R x M, leading dim ldz) and x (R x K, ldx) are bf16
 * row-major, 16-byte aligned, ld multiples of 8; R a multiple of 32. (M, K) in {(256, 64),
 * (128, 256), (128, 128), (64, 64), (256, 32)}. accumulate = 0 overwrites dw/db, 1 adds. Deterministic
 * (fixed-order partial sums). work: asvrl_linear_wgrad_workspace(M, K) floats. */
int64_t asvrl_linear_wgrad_workspace(int32_t M, int32_t K);
int asvrl_linear_wgrad(const void* dz, int64_t ldz, const void* x, int64_t ldx, int32_t R, int32_t M,
                       int32_t K, float* dw, float* db, int32_t accumulate, float* work,
                       int64_t work_floats, void* stream);

/* The same without the final reduction: writes *groups_out partials of (M*K + M) floats each
 * into `partial` (asvrl_linear_wgrad_groups(R, M, K) of them); reduce later, possibly together
 * with other layers, with asvrl_partial_sums. */
int32_t asvrl_linear_wgrad_groups(int32_t R, int32_t M, int32_t K);
int asvrl_linear_wgrad_partial(const void* dz, int64_t ldz, const void* x, int64_t ldx, int32_t R, int32_t M,
                               int32_t K, float* partial, int64_t partial_floats, int32_t* groups_out,
                               void* stream);

/* Several layers' partials in ONE launch (ABI v9; replaces one partial launch per layer on side
 * streams joined back). Segment k writes groups_out[k] partials, bit-identical to its own launch
 * (same groups, same summation order):
 *   kind ASVRL_WGRAD_MFMA : asvrl_linear_wgrad_partial (bf16 dz, x); (M, K) in {(256, 64), (128, 256),
 *                           (128, 128), (256, 32), (32, 128)};
 *   kind ASVRL_WGRAD_VEC  : asvrl_linear_wgrad_vec_partial (dz = dq f32 with stride ldz, M = 1, K = 128);
 *   kind ASVRL_WGRAD_SMALL: asvrl_small_wgrad_partial (f32 dz, x; M | 256, K <= 4). */
#define ASVRL_MAX_WGRAD_SEGS 24
#define ASVRL_WGRAD_MFMA 0
#define ASVRL_WGRAD_VEC 1
#define ASVRL_WGRAD_SMALL 2
typedef struct AsvWgradSeg {
  const void* dz;
  int64_t ldz;
  const void* x;
  int64_t ldx;
  int32_t R, M, K, kind;
  float* partial;
  int64_t partial_floats;
} AsvWgradSeg;
int asvrl_linear_wgrad_multi(const AsvWgradSeg* segs, int32_t nseg, int32_t* groups_out, void* stream);

/* Every gradient of the Actor (AC_IQN_model.py:284-321) after asvrl_actor_backward, in ONE launch (ABI 19;
 * replaces asvrl_linear_wgrad_multi + asvrl_partial_sums_norm of agent.py:424-426's actor_loss.backward()):
 * hidden_layer / hidden_layer_2 weight and bias grads, output_layer's, the two observation encoders' (folded
 * from the 256 x 32 encoder image over the five object copies), the actor loss (sum of n_loss per-tile
 * partials), the squared-norm partials clip_grad_norm_ folds (asvrl_adam_step's norm_parts) and the Adam
 * step count (*step += 1). Each 32 x 32 output tile is reduced over S row splits by the split that arrives
 * last, in split order: deterministic, no partial buffer for another launch. Activations (operand dtype,
 * contiguous, 16-byte aligned): xb [B][32], h0 [B][256], h1, h2, dz2, dz1 [B][128], dz0 [B][256]; dout f32
 * [B][2]. Gradients f32, row-major as the nn.Linear parameters; enc_grad = self_w 56x7 | self_b 56 |
 * obj_w 40x5 | obj_b 40. work: asvrl_actor_grads_workspace(B) floats; counters:
 * asvrl_actor_grads_counters() ints, zero before the first launch (each launch leaves them zero). */
typedef struct AsvActorGradIO {
  const void* xb;
  const void* h0;
  const void* h1;
  const void* h2;
  const float* dout;
  const void* dz2;
  const void* dz1;
  const void* dz0;
  int32_t B, n_loss;
  const float* tile_loss;   /* optional (with loss_out) */
  float* loss_out;
  float* w1_grad;           /* hidden_layer [128][256], [128] */
  float* b1_grad;
  float* w2_grad;           /* hidden_layer_2 [128][128], [128] */
  float* b2_grad;
  float* wo_grad;           /* output_layer [2][128], [2] */
  float* bo_grad;
  float* enc_grad;          /* [688] */
  double* norm_parts;       /* optional: asvrl_actor_grads_norm_parts() slots */
  float* step;              /* optional */
  float* work;
  int64_t work_floats;
  int32_t* counters;
} AsvActorGradIO;
int64_t asvrl_actor_grads_workspace(int32_t B);
int32_t asvrl_actor_grads_counters(void);
int32_t asvrl_actor_grads_norm_parts(void);
int asvrl_actor_grads(const AsvActorGradIO* io, void* stream);

/* One output unit's version: dw[k] = sum_r dq[r*ldq] x[r][k], db = sum_r dq[r*ldq] with dq f32 and
 * x bf16 (R x K, ldx); K in {64, 128, 256}; work >= 256 * (K + 1) floats. */
int asvrl_linear_wgrad_vec(const float* dq, int64_t ldq, const void* x, int64_t ldx, int32_t R, int32_t K, float* dw,
                           float* db, int32_t accumulate, float* work, int64_t work_floats, void* stream);

int32_t asvrl_linear_wgrad_vec_groups(int32_t R);
int asvrl_linear_wgrad_vec_partial(const float* dq, int64_t ldq, const void* x, int64_t ldx, int32_t R,
                                   int32_t K, float* partial, int64_t partial_floats, int32_t* groups_out,
                                   void* stream);

/* One pending reduction: dw[i] (+)= sum_g partial[g][i] for i < nw, db likewise for the
 * trailing nb values of each group's (nw + nb)-float partial (db optional). A segment with
 * nw + nb == 1 (a scalar over many groups) is reduced by a whole workgroup. */
#define ASVRL_MAX_SUM_SEGS 24
#define ASVRL_SUM_PLAIN 0
/* The 256 x 32 encoder-image partials (asvrl_mlp_pack's block-structured image) folded straight
 * into the contiguous gradients [self_w 56x7 | self_b 56 | obj_w 40x5 | obj_b 40] at dw (688
 * floats, nw = 688, nb = 0): the object encoder's five copies are summed, in object order, after
 * each copy's own fixed-order group sum (bit-identical to asvrl_encoder_fold after a plain sum). */
#define ASVRL_SUM_FOLD_ENCODERS 1
typedef struct AsvPartialSum {
  const float* partial;
  float* dw;
  float* db;
  int32_t groups, nw, nb, accumulate;
  int32_t stride;   /* floats per group in partial; 0 = nw + nb */
  int32_t boff;     /* offset of the bias partials within a group; 0 = nw. With stride / boff a
                       32-row MFMA reduction can fill a layer of fewer rows (IQN's 25 actions) */
  int32_t mode;     /* ASVRL_SUM_PLAIN or ASVRL_SUM_FOLD_ENCODERS */
  int32_t norm;     /* 1: the outputs count towards the gradient norm (asvrl_partial_sums_norm) */
} AsvPartialSum;
/* Reduce up to ASVRL_MAX_SUM_SEGS pending partial sets in one launch (fixed order per output). */
int asvrl_partial_sums(const AsvPartialSum* segs, int32_t nseg, void* stream);

/* asvrl_partial_sums that also prepares the global gradient norm of the segments with norm = 1
 * for an asvrl_adam_step right after (replaces asvrl_adam_clip's norm pass when every gradient is
 * produced by this launch and no all-reduce follows): each working workgroup writes the f64 sum of
 * the squares of the outputs it wrote to its own slot of norm_parts (asvrl_partial_sums_norm_parts
 * slots), and *step is incremented. */
int asvrl_partial_sums_norm(const AsvPartialSum* segs, int32_t nseg, double* norm_parts, float* step,
                            void* stream);
int32_t asvrl_partial_sums_norm_parts(const AsvPartialSum* segs, int32_t nseg);

/* ---------------------------------------------------------------- per-row MLPs (actor, encoders) */

/* f32 parameters of one AC-IQN network's per-row layers (AC_IQN_model.py:254-262, 389-404):
 * self_encoder (56 x 7), object_encoder (40 x 5); for an Actor also hidden_layer (128 x 256) and
 * hidden_layer_2 (128 x 128); for a Critic also action_encoder (128 x 2). Unused entries NULL. */
typedef struct AsvMlpSrc {
  const float* self_w;
  const float* self_b;
  const float* obj_w;
  const float* obj_b;
  const float* w1;
  const float* w2;
  const float* ae_w;
} AsvMlpSrc;

/* Packed images the kernels read (filled by asvrl_mlp_pack, which writes through these
 * pointers) plus direct pointers to the remaining f32 parameters. */
typedef struct AsvMlpWeights {
  const void* enc_frag;   /* both encoders as one block-structured 256 x 32 bf16 image (16 KB) */
  const float* b_enc;     /* [256] their biases (written by the pack) */
  const void* w1_frag;    /* hidden_layer, chained order (64 KB)          (Actor) */
  const void* w2_frag;    /* hidden_layer_2 (32 KB)                        (Actor) */
  const void* w2t_frag;   /* hidden_layer_2^T (32 KB, backward)            (Actor) */
  const void* w1t_frag;   /* hidden_layer^T (64 KB, backward)              (Actor) */
  const float* b1;        /* hidden_layer.bias [128]                       (Actor) */
  const float* b2;        /* hidden_layer_2.bias [128]                     (Actor) */
  const float* wout;      /* output_layer.weight [2][128]                  (Actor) */
  const float* bout;      /* output_layer.bias [2]                         (Actor) */
  const void* ae_frag;    /* action_encoder as a 128 x 16 image (cols 2.. zero) (Critic) */
  const float* b_ae;      /* action_encoder.bias [128]                     (Critic) */
  float out_scale;        /* Actor.atan_scale = float32(2 / pi) */
} AsvMlpWeights;

/* Rows in / out of the MLP kernels. Observation rows are the packed ASVRL_OBS_DIM layout at
 * row stride ldx floats (40 for env observations, 88 for replay rows), 16-byte aligned. */
typedef struct AsvMlpIO {
  const float* x;
  int64_t ldx;
  const float* act;       /* ENCODE: actions [n] at stride lda (G = relu(W_ae a + b_ae)) */
  int64_t lda;
  int32_t n;
  float* F;               /* ENCODE out [n][256] */
  float* G;               /* ENCODE out [n][128] (optional) */
  void* xb;               /* ENCODE (optional) / TRAIN out: bf16 copy of obs columns 0..31 [n][32] */
  float* a_out;           /* FWD / TRAIN out: actions, stride ld_aout */
  int64_t ld_aout;
  double* a_out64;        /* ACT out: [n][2] f64 */
  float* pre;             /* TRAIN out / backward in: pre-atan outputs [n][2] */
  void* h0;               /* TRAIN out: bf16 [n][256] encoder output (hidden_layer input) */
  void* h1;               /* TRAIN out: bf16 [n][128] */
  void* h2;               /* TRAIN out: bf16 [n][128] */
  const float* dA;        /* backward in: dL/d(action) [n][2] */
  float* dout;            /* backward out: dL/d(output_layer pre-activation) [n][2] */
  void* dz2;              /* backward out: bf16 [n][128] hidden_layer_2 pre-activation grad */
  void* dz1;              /* backward out: bf16 [n][128] hidden_layer pre-activation grad */
  void* dz0;              /* backward out: bf16 [n][256] encoder pre-activation grad */
  const int64_t* step_dev;      /* ACT: device step counter (epsilon schedule, trainer.py:257-264) */
  double eps_steps_per_count;   /* timesteps per counter tick (= n_envs) */
  double eps_total, eps_fraction, eps_initial, eps_final;
  uint64_t seed;                /* ACT: Philox key of the exploration draws */
} AsvMlpIO;

/* Pack the bf16 images of `w` from the f32 parameters in `src` (one launch). */
int asvrl_mlp_pack(const AsvMlpSrc* src, const AsvMlpWeights* w, void* stream);
/* observation_processor (AC_IQN_model.py:284-308) -> F, and action_encoder -> G, per row. */
int asvrl_mlp_encode(const AsvMlpWeights* w, const AsvMlpIO* io, void* stream);
/* Actor.forward (AC_IQN_model.py:310-321). mode 1 = ACT (epsilon-greedy f64 actions,
 * agent.py:207-225), 2 = FWD (f32 actions), 3 = TRAIN (f32 actions + saved activations). */
int asvrl_actor_forward(const AsvMlpWeights* w, const AsvMlpIO* io, int32_t mode, void* stream);
/* The AC-IQN learn step's prologue in ONE launch (ABI 18): asvrl_replay_sample's draw of B rows and
 * their quantile fractions (uniform ring, replay_buffer.py:26-45; taus of AC_IQN_model.py:419), the local
 * Actor's TRAIN forward on s (agent.py:419-421; outputs in train_io, n = B) and the target Actor's FWD
 * on s' into na [B][2] (agent.py:397-398) -- bit-identical to the three separate launches. B must be a
 * multiple of 32. */
typedef struct AsvSampleArgs {
  const float* ring;            /* [capacity][ASVRL_TR_DIM] */
  int64_t capacity;
  const int64_t* ring_state;    /* {head, size} to sample against */
  uint64_t seed, counter;
  const uint64_t* counter_dev;  /* optional, added to counter */
  int64_t guard;                /* skip the oldest rows a concurrent push of <= guard rows may overwrite */
  int32_t B, tau_sets, tau_n, _pad0;
  float* out;                   /* [B][ASVRL_TR_DIM] sampled rows */
  float* taus;                  /* optional [tau_sets][B][tau_n] */
} AsvSampleArgs;
int asvrl_learn_prologue(const AsvSampleArgs* s, const AsvMlpWeights* actor, const AsvMlpIO* train_io,
                         const AsvMlpWeights* target_actor, float* na, void* stream);
/* Backward of the Actor from dA to every layer's pre-activation gradient (agent.py:425). */
int asvrl_actor_backward(const AsvMlpWeights* w, const AsvMlpIO* io, void* stream);
/* Fold the 256 x 32 encoder-image gradient (dw, db from asvrl_linear_wgrad) back onto
 * self_encoder / object_encoder weight and bias gradients (object rows summed over objects). */
int asvrl_encoder_fold(const float* dw, const float* db, float* self_w, float* self_b, float* obj_w,
                       float* obj_b, int32_t accumulate, void* stream);
/* dw[m][k] = sum_r dz[r][m] x[r][k], db[m] = sum_r dz[r][m] for f32 inputs with K <= 4 and
 * M | 256 (the critic action_encoder). work >= ceil(R / 32) * (M*K + M) floats. */
int asvrl_small_wgrad(const float* dz, int64_t ldz, const float* x, int64_t ldx, int32_t R, int32_t M,
                      int32_t K, float* dw, float* db, int32_t accumulate, float* work,
                      int64_t work_floats, void* stream);
int asvrl_small_wgrad_partial(const float* dz, int64_t ldz, const float* x, int64_t ldx, int32_t R,
                              int32_t M, int32_t K, float* partial, int64_t partial_floats,
                              int32_t* groups_out, void* stream);

/* ---------------------------------------------------------------- misc */
const char* asvrl_last_error(void);
int asvrl_abi_version(void);
/* Bytes per learner-kernel operand element: 2 in libasvrl.so (bf16 MFMA operands, weight images
 * and saved activations, f32 accumulation), 4 in libasvrl_f32.so -- the same sources built with
 * ASVRL_OPERAND_F32=1, every operand f32 (v_mfma_f32_32x32x2_f32), the parity build of the
 * hand-written learner. Every other entry point is identical in both libraries. */
int32_t asvrl_operand_bytes(void);
/* sizeof(AsvParams, AsvEnvState, AsvStepCtl, AsvStepOut, AsvResetCfg) as compiled, for
 * binding checks (host pointer to 5 int64). */
void asvrl_struct_sizes(int64_t* out5);

#ifdef __cplusplus
}
#endif
#endif /* ASVRL_H */
