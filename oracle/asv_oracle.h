/* asv_oracle.h -- CPU restatement of the rfarl env step (TEST INFRASTRUCTURE ONLY).
 *
 * This is the checker, never the product: only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it. Parity is pinned against the reference's own
 * outputs captured in tests/golden/ by tools/capture_oracle.py.
 *
 * Every function mirrors one reference function, per robot, in the reference's loop
 * order and arithmetic order (citations are /root/reference/rfarl/rfarl/... file:line).
 */
#ifndef ASV_ORACLE_H
#define ASV_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Vehicle + perception + reward parameters (wamv.py:45-125, env.py:33-54). */
typedef struct OrParams {
  double dt;        /* wamv.py:46 */
  int32_t N;        /* wamv.py:47 substeps per action */
  double length, width, r, goal_dis, min_thrust, max_thrust;
  double m, Izz;
  double xDotU, yDotV, yDotR, nDotR, nDotV, xU, xUU, yV, yVV, yR, yRV, yVR, yRR, nR, nRR, nV,
      nVV, nRV, nVR;
  double P[9];      /* inv(A^T A) A^T, A = M_RB + M_A, row-major (wamv.py:267-271) */
  double thrust_change[5]; /* left == right table (wamv.py:86-88) */
  double range, angle, r_mean_ratio; /* Perception (wamv.py:12-25) */
  int32_t max_obj_num;
  double timestep_penalty, COLREGs_penalty, collision_penalty, goal_reward; /* env.py:47-50 */
  double core_r;    /* env.py:35 vortex core radius */
  int32_t episode_limit; /* env.py:312 (1000) */
} OrParams;

/* One robot's mutable state (wamv.py:92-101,130-132) plus goal. */
typedef struct OrRobot {
  double x, y, theta, vr[3], v[3], tl, tr, lp, rp, goal[2];
  uint8_t deactivated, collision, reach_goal, apply_colregs;
  double phi;
} OrRobot;

void or_default_params(OrParams* p);

/* env.py:458-501 current at (x, y); cores: [n][4] = x, y, clockwise, Gamma */
void or_current(const double* cores, int n_cores, double core_r, double x, double y,
                double out[3]);

/* env.py:254-277 for one robot: N substeps of wamv.py:204-279; returns reward base
 * -0.1 + (d_before - d_after). */
double or_robot_act(const OrParams* p, OrRobot* rb, const double action[2], int continuous,
                    const double* cores, int n_cores);

/* wamv.py:436-529 for robot i. noise: [(O + R)][5] draws for this robot (slot o = obstacle
 * o, slot O + j = robot j). Writes self_obs[7], objs[5][5]; returns object count, or -1
 * when the robot is deactivated ((None, None)). */
int or_perceive(const OrParams* p, OrRobot* robots, int n_robots, int i, const double* obstacles,
                int n_obs, int O, const double* noise, double* self_obs, double* objs);

/* env.py:240-333: one full MarineNavEnv3.step for one env.
 * actions [R][2] (discrete: actions[i][0] = index), noise [R][(O + R)][5].
 * Outputs: rewards[R], dones[R], infos[R] (codes: 0 normal, 1 too long, 2 collision,
 * 3 reach goal, 4 deactivated after collision, 5 deactivated after reaching goal),
 * self_obs [R][7], objs [R][5][5], cnt [R]. Returns 0, or -1 for the RuntimeError of
 * env.py:303. ep_ts is episode_timesteps before the step (incremented on return). */
int or_env_step(const OrParams* p, OrRobot* robots, int n_robots, int R, const double* obstacles,
                int n_obs, int O, const double* cores, int n_cores, const double* actions,
                int continuous, const double* noise, int32_t* ep_ts, double* rewards,
                uint8_t* dones, uint8_t* infos, double* self_obs, double* objs, int32_t* cnt);

/* Batched CPU baseline: E independent envs with R robots each, noise from a counter-based
 * generator (Philox-4x32-10, Box-Muller normals, Best-Fisher von Mises), trainer-side
 * deactivation applied. Threads via OpenMP. Returns env-steps executed. */
int64_t or_batch_rollout(const OrParams* p, int E, int R, int O, int steps, uint64_t seed,
                         int threads, double* checksum);

/* The fast path's device reset (asvrl_env_reset) restated one candidate at a time: MarineNavEnv3.reset's
 * rejection sampling (robots env.py:106-120 with check_start_and_goal :360-376, cores :123-136 with
 * check_core :378-418, obstacles :151-162 with check_obstacle :420-456), each phase drawing candidates
 * c = 0, 1, ... in order, accepting the ones valid against everything accepted before them, at most 500
 * candidates per phase. Candidate c's values come from Philox-4x32-10 at counter (4c + j/2, env, phase,
 * counter) under the key seed ^ (counter >> 32) * 0x9E3779B97F4A7C15 (the device streams; the reference
 * draws them from np.random instead, so this pins the kernel's sequential semantics, not the
 * reference's numbers). Outputs for env e: robots [R][5] = x, y, gx, gy, theta; n_robots; cores
 * [n][4] = x, y, clockwise, Gamma; obstacles [n][3] = x, y, r. cfg: AsvResetCfg's fields in order. */
typedef struct OrResetCfg {
  int32_t num_robots, num_obs, num_cores, _pad0;
  double min_start_goal_dis, width, height, clear_r, obs_r_lo, obs_r_hi, v_lo, v_hi, v_rel_max, p_rel;
} OrResetCfg;
void or_device_reset(const OrResetCfg* cfg, double core_r, int R, int O, int C, uint64_t seed, uint64_t counter,
                     int e, double* robots, int* n_robots, double* cores, int* n_cores, double* obstacles,
                     int* n_obs);

/* C51 projection restated from agent.py:616-631 in f32 with the CPU index_add_ order. */
void or_c51_project(const float* pns_a, const float* returns, const float* nonterminal,
                    const float* support, int B, int atoms, float vmin, float vmax,
                    float gamma_n, float* m);

#ifdef __cplusplus
}
#endif
#endif
