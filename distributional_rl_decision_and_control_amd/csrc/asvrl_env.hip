// asvrl_env.hip -- the vectorised ASV marine-env step and reset on gfx950.
//
// Replaces MarineNavEnv3.step / reset (rfarl/rfarl/envs/marinenav/env.py:72-164,240-333)
// and the per-robot Robot methods they call (rfarl/rfarl/envs/marinenav/vehicles/wamv.py).
//
// Layout: robot state is field-major SoA in HBM (rs[field][e * R + i]). A 256-lane workgroup
// owns about 40 robots' worth of whole envs, lane = (env_in_block, robot) in its first wave.
// Phase 1 runs the N Fossen substeps of each robot entirely in registers (f64, one sincos per
// substep). The post-move positions/velocities of the block's robots, their frames and the envs'
// buoys are then staged in LDS; phase 2a gives every (robot, candidate) pair of the block one lane
// across all four waves (noisy observation, detection, collision, sort key into LDS), and phase 2b
// merges each robot's candidates in the reference's order (stable top-5 insertion), then COLREGs,
// reward, done/info and -- in the fused training loop -- trainer.py's deactivation and the
// episode-end test, reduced per env through LDS. (AsvEnvLaunch layout 2: the per-robot sweep, phase 2
// as one serial loop per lane, 64-lane groups.)
//
// Arithmetic follows the reference's operation order (np.matrix products as explicit row
// sums, no FMA contraction: built with -ffp-contract=off) so f64 state agrees with the
// reference to ~1e-14 and collision/goal/done masks bit-exactly.
#include <type_traits>

#include "asvrl_common.h"
#include "asvrl_vonmises_k1.h"

namespace asvrl {
namespace {

constexpr int kBlock = 256;
// env-step workgroup: one wave of whole envs when they fit (R <= 64), spreading a 4096-env batch
// over every CU instead of packing 51 envs per 256-lane group onto a third of them
__host__ __device__ constexpr int step_block(int R) { return R <= 64 ? 64 : 256; }
constexpr int kMaxCores = 16;        // the device reset sampler's LDS table (env_reset_kernel)
constexpr int kMaxCoresStep = 4096;  // the step and the current field read the cores from HBM

struct Regs {
  double x, y, th, vr0, vr1, vr2, v0, v1, v2, tl, tr, lp, rp;
};

// The pair kernels' arguments, read through the kernarg segment pointer (KArg) rather than as by-value
// parameters: a by-value struct parameter is loaded whole at kernel entry and held to its last use, which
// spilled 122 SGPRs to VGPR lanes (a v_readlane at every later use). A field loaded after kfresh() is not
// merged with the same field's earlier load, so each phase below re-reads what it uses from the kernarg
// segment (scalar loads) and holds it for that phase only.
struct PairsArgs {
  AsvParams p;
  AsvEnvState s;
  AsvStepCtl ctl;
  AsvStepOut out;
  const double* actions;
  const double* noise;
  int epb, group0;
};

__device__ inline double clampd(double v, double lo, double hi) {  // np.clip
  return v < lo ? lo : (v > hi ? hi : v);
}

// env.py:458-501. Cores contribute in ascending-distance order (KDTree query with k = all).
__device__ inline void current_at(const double* __restrict__ cores, int nc, double core_r, double x,
                                  double y, double& cx, double& cy) {
  cx = 0.0;
  cy = 0.0;
  if (nc <= 0) return;
  double prev_d = -1.0;
  int prev_k = -1;
  for (int t = 0; t < nc; ++t) {
    double best_d = 0.0;
    int best_k = -1;
    for (int k = 0; k < nc; ++k) {
      const double dx = cores[4 * k] - x, dy = cores[4 * k + 1] - y;
      const double d = sqrt(dx * dx + dy * dy);
      const bool after = (d > prev_d) || (d == prev_d && k > prev_k);
      if (after && (best_k < 0 || d < best_d)) {
        best_d = d;
        best_k = k;
      }
    }
    prev_d = best_d;
    prev_k = best_k;
    const double* c = cores + 4 * best_k;
    double rx = c[0] - x, ry = c[1] - y;
    const double dis = sqrt(rx * rx + ry * ry);
    rx /= dis;
    ry /= dis;
    double tx, ty;
    if (c[2] != 0.0) { tx = -ry; ty = rx; } else { tx = ry; ty = -rx; }
    const double sp = dis <= core_r ? c[3] / (2 * kPi * core_r * core_r) * dis : c[3] / (2 * kPi * dis);
    cx += tx * sp;
    cy += ty * sp;
  }
}

// One robot's action: N substeps of Robot.update_state (wamv.py:204-231) + compute_motion
// (wamv.py:233-279) with the current sampled at the pre-move position (env.py:257-260).
// The parameters as a plain reference (the sweep kernel) or re-read from the kernarg segment at every substep
// (the pair kernel: the substep loop then holds no parameter in SGPRs across iterations)
struct ParamsRef {
  const AsvParams* q;
  __device__ void fresh() {}
  __device__ const AsvParams& get() const { return *q; }
};
struct ParamsKArg {
  KArg<AsvParams> q;
  __device__ void fresh() { q = kfresh(q); }
  __device__ const AsvParams& get() const { return kref(q); }
};
template <class PR>
__device__ inline void robot_act(PR P, Regs& r, double a0, double a1, int continuous, const double* cores, int nc) {
  // propulsion (wamv.py:251-264) depends only on the thrusts, which change on substep 0
  double fx = 0, fy = 0, mn = 0;
  const double clp = cos(r.lp), slp = sin(r.lp), crp = cos(r.rp), srp = sin(r.rp);
  const int n_sub = P.get().N;
  for (int idx = 0; idx < n_sub; ++idx) {
    P.fresh();
    const AsvParams& p = P.get();
    double cx = 0.0, cy = 0.0;
    if (nc > 0) current_at(cores, nc, p.core_r, r.x, r.y, cx, cy);
    r.v0 = r.vr0 + cx;  // update_velocity (wamv.py:201-202)
    r.v1 = r.vr1 + cy;
    r.v2 = r.vr2 + 0.0;
    r.x += r.v0 * p.dt;
    r.y += r.v1 * p.dt;
    r.th += r.v2 * p.dt;
    while (r.th < 0.0) r.th += kTwoPi;
    while (r.th >= kTwoPi) r.th -= kTwoPi;
    if (idx == 0) {
      double l, rr;
      if (continuous) {
        l = a0 * 1000.0;
        rr = a1 * 1000.0;
      } else {
        const int a = static_cast<int>(a0);
        l = p.left_thrust_change[a / 5];
        rr = p.right_thrust_change[a % 5];
      }
      r.tl = clampd(r.tl + l * p.dt * p.N, p.min_thrust, p.max_thrust);
      r.tr = clampd(r.tr + rr * p.dt * p.N, p.min_thrust, p.max_thrust);
      const double fxl = r.tl * clp, fyl = r.tl * slp;
      const double fxr = r.tr * crp, fyr = r.tr * srp;
      const double mxl = fxl * p.width / 2, myl = -fyl * p.length / 2;
      const double mxr = -fxr * p.width / 2, myr = -fyr * p.length / 2;
      fx = fxl + fxr;
      fy = fyl + fyr;
      mn = mxl + myl + mxr + myr;
    }
    // compute_motion
    double s, c;
    sincos(r.th, &s, &c);
    const double u_r = c * r.vr0 + s * r.vr1;
    const double v_r = -s * r.vr0 + c * r.vr1;
    const double u = c * r.v0 + s * r.v1;
    const double v = -s * r.v0 + c * r.v1;
    const double w = r.v2;
    const double mr = p.m * w;
    const double cv0 = -(-mr * v), cv1 = -(mr * u), cv2 = 0.0;
    const double ca02 = p.yDotV * v_r + p.yDotR * w;
    const double ca12 = -p.xDotU * u_r;
    const double ca20 = -p.yDotV * v_r - p.yDotR * w;
    const double ca21 = p.xDotU * u_r;
    const double au = fabs(u_r), av = fabs(v_r), ar = fabs(w);
    const double n00 = (0.0 + -p.xU) + -(p.xUU * au);
    const double n02 = (ca02 + -0.0) + -0.0;
    const double n11 = (0.0 + -p.yV) + -(p.yVV * av + p.yRV * ar);
    const double n12 = (ca12 + -p.yR) + -(p.yVR * av + p.yRR * ar);
    const double n20 = (ca20 + -0.0) + -0.0;
    const double n21 = (ca21 + -p.nV) + -(p.nVV * av + p.nRV * ar);
    const double n22 = (0.0 + -p.nR) + -(p.nVR * av + p.nRR * ar);
    const double nv0 = n00 * u_r + 0.0 * v_r + n02 * w;
    const double nv1 = 0.0 * u_r + n11 * v_r + n12 * w;
    const double nv2 = n20 * u_r + n21 * v_r + n22 * w;
    const double b0 = cv0 - nv0 + fx, b1 = cv1 - nv1 + fy, b2 = cv2 - nv2 + mn;
    const double acc0 = p.P[0] * b0 + p.P[1] * b1 + p.P[2] * b2;
    const double acc1 = p.P[3] * b0 + p.P[4] * b1 + p.P[5] * b2;
    const double acc2 = p.P[6] * b0 + p.P[7] * b1 + p.P[8] * b2;
    const double w0 = u_r + acc0 * p.dt, w1 = v_r + acc1 * p.dt, w2 = w + acc2 * p.dt;
    r.vr0 = c * w0 + -s * w1;
    r.vr1 = s * w0 + c * w1;
    r.vr2 = w2;
  }
}

__device__ inline double wrap_to_pi(double a) {  // wamv.py:425-434
  while (a < -kPi) a += kTwoPi;
  while (a >= kPi) a -= kTwoPi;
  return a;
}

// reward / done / info (env.py:290-331) and the trainer's bookkeeping (trainer.py:157-172): the
// discounted return gamma^ep_ts * r and deactivation on collision or goal
struct StepResult {
  double reward, ret;
  uint8_t done, info, nfl;
};

__device__ inline StepResult step_result(const AsvParams& p, const AsvStepCtl& ctl, bool exists, bool deact,
                                         bool active, int ep_ts, uint8_t fl, bool coll, bool reach, bool apply,
                                         double phi, double reward, double ret) {
  uint8_t done = 1, info = ASVRL_INFO_ABSENT;
  if (exists) {
    if (deact) {
      reward = 0.0;
      done = 1;
      info = coll ? ASVRL_INFO_DEACT_COLLISION : (reach ? ASVRL_INFO_DEACT_GOAL : ASVRL_INFO_ABSENT);
    } else if (ctl.do_dynamics) {
      double pen = 0.0;
      if (apply) pen += p.COLREGs_penalty * phi;
      reward += pen;
      if (ep_ts >= p.episode_limit) {
        done = 1;
        info = ASVRL_INFO_TOO_LONG;
      } else if (coll) {
        reward += p.collision_penalty;
        done = 1;
        info = ASVRL_INFO_COLLISION;
      } else if (reach) {
        reward += p.goal_reward;
        done = 1;
        info = ASVRL_INFO_REACH_GOAL;
      } else {
        done = 0;
        info = ASVRL_INFO_NORMAL;
      }
    } else {
      done = 0;
      info = ASVRL_INFO_NORMAL;
    }
  }
  uint8_t nfl = static_cast<uint8_t>((fl & ASVRL_FLAG_DEACTIVATED) | (coll ? ASVRL_FLAG_COLLISION : 0) |
                                     (reach ? ASVRL_FLAG_REACH_GOAL : 0) | (apply ? ASVRL_FLAG_COLREGS : 0));
  if (active && ctl.do_dynamics && ctl.trainer_deactivate) {
    if (ctl.gamma > 0) ret += pow(ctl.gamma, static_cast<double>(ep_ts)) * reward;
    if (coll || reach) nfl |= ASVRL_FLAG_DEACTIVATED;
  }
  return StepResult{reward, ret, done, info, nfl};
}

// per-env end of the step (env.py:330, trainer.py:172): episode counter, episode end when the limit is
// hit or no robot is left active, and the finished episode's totals
__device__ inline void env_end(const AsvParams& p, const AsvEnvState& s, const AsvStepCtl& ctl,
                               const AsvStepOut& out, int e, int ep_ts, int nrob, int alive, size_t NT) {
  s.ep_ts[e] = ep_ts + 1;
  if (ctl.trainer_deactivate && out.env_done != nullptr) {
    const bool end = (ep_ts >= p.episode_limit) || alive == 0;
    out.env_done[e] = end ? 1 : 0;
    if (end && out.stats != nullptr) {
      double sr = 0, sc = 0, sg = 0, sk = 0, st = 0;
      for (int j = 0; j < nrob; ++j) {
        const size_t jd = static_cast<size_t>(e) * s.max_robots + j;
        const uint8_t fj = s.rflags[jd];
        sr += s.rs[ASVRL_F_RET * NT + jd];
        sc += 1;
        sg += (fj & ASVRL_FLAG_REACH_GOAL) ? 1 : 0;
        sk += (fj & ASVRL_FLAG_COLLISION) ? 1 : 0;
        st += (fj & ASVRL_FLAG_DEACTIVATED) ? 0 : 1;
      }
      atomicAdd(out.stats + 0, sr);
      atomicAdd(out.stats + 1, sc);
      atomicAdd(out.stats + 2, sg);
      atomicAdd(out.stats + 3, sk);
      atomicAdd(out.stats + 4, st);
      atomicAdd(out.stats + 5, 1.0);
    }
  }
}

// check_apply_COLREGs (wamv.py:398-423) for one kept object. `ev` says whether the test got as far as
// the turn angle (the reference assigns phi exactly then); returns phi > 0.
__device__ __forceinline__ bool colregs_body(double rself, double c, double s, double v0, double v1, double ox,
                                             double oy, double ovx, double ovy, double orad, double& phi, bool& ev) {
  ev = false;
  if (sqrt(ovx * ovx + ovy * ovy) < 0.5) return false;
  const double ev0 = c * v0 + s * v1;
  const double ev1 = -s * v0 + c * v1;
  if (sqrt(ev0 * ev0 + ev1 * ev1) < 0.5) return false;
  const double al = atan2(ovy, ovx);  // project_ego_to_vehicle_frame (wamv.py:324-342)
  double sa, ca;
  sincos(al, &sa, &ca);
  const double px = -ca * ox + -sa * oy;
  const double py = sa * ox + -ca * oy;
  const double qx = ca * ev0 + sa * ev1;
  const double qy = -sa * ev0 + ca * ev1;
  const bool x_in = (px >= -9.0) && (px <= 12.0);  // wamv.py:344-362
  const bool y_in = (py >= -17.0) && (py <= 0.0);
  const bool in_tri = (py - (-7.0)) > (-7.0 / 12.0) * (px - 12.0);
  const bool left_pos = x_in && y_in && !in_tri;
  const bool head_pos = (px >= 0.0) && (px <= 17.0) && (py >= -0.5 * 9.0) && (py <= 0.5 * 9.0);  // :364-377
  if (!(left_pos || head_pos)) return false;   // the heading test below cannot rescue either zone
  const double ang = atan2(qy, qx);
  const bool left = left_pos && (ang >= kPi / 4) && (ang <= 3 * kPi / 4);
  const bool head = head_pos && (fabs(ang) > 3 * kPi / 4);
  if (!(left || head)) return false;
  const double ego_ang = atan2(ev1, ev0);  // compute_COLREGs_turn_angle (wamv.py:379-396)
  const double obj_ang = atan2(oy, ox);
  const double base1 = orad + 1.0;
  const double dist = sqrt(ox * ox + oy * oy);
  const double add1 = asin(base1 / dist);
  const double tang = sqrt(dist * dist - base1 * base1);
  const double add2 = atan2(rself, tang);
  const double desired = wrap_to_pi(obj_ang + add1 + add2);
  phi = wrap_to_pi(desired - ego_ang);
  ev = true;
  return phi > 0;
}

// called out of line: its f64 atan2 / asin / sincos inlined at a call site would set the whole kernel's
// register budget (the pair kernel: 162 -> 133 VGPRs)
__device__ __attribute__((noinline)) bool colregs_ev(double rself, double c, double s, double v0, double v1,
                                                     double ox, double oy, double ovx, double ovy, double orad,
                                                     double& phi, bool& ev) {
  return colregs_body(rself, c, s, v0, v1, ox, oy, ovx, ovy, orad, phi, ev);
}

// the per-robot sweep's serial chain (phi written when evaluated)
__device__ __attribute__((noinline)) bool colregs(double rself, double c, double s, double v0, double v1,
                               double ox, double oy, double ovx, double ovy, double orad,
                               double& phi) {
  bool ev;
  return colregs_body(rself, c, s, v0, v1, ox, oy, ovx, ovy, orad, phi, ev);
}

struct Cand {
  double key, a, b, c, d, e;
};

__device__ inline void cswap(bool cond, Cand& x, Cand& y) {
  if (cond) {
    const Cand t = x;
    x = y;
    y = t;
  }
}

// vonmises(0, 1) by its inverse CDF (asvrl_vonmises_k1.h, 1025 f32 knots) at the uniform u, linearly
// interpolated: no rejection loop (Best-Fisher's one or two extra Philox calls per draw, and a wave runs
// the second whenever one of its 64 lanes rejects twice)
__device__ __forceinline__ float vonmises_k1_icdf(float u) {
  const float x = u * static_cast<float>(kVmIcdfN);
  const int i = min(static_cast<int>(x), kVmIcdfN - 1);
  const float lo = kVmIcdfK1[i], hi = kVmIcdfK1[i + 1];
  return lo + (x - static_cast<float>(i)) * (hi - lo);
}

// perception noise of (robot qidx, candidate slot): injected (noise_mode 0, [robot][O + R][5]), f64
// Philox (1) or f32 Philox (2), the substream keyed by (robot, slot) so every launch shape draws the same
// NM: the mode fixed at compile time (the pair kernel's instances), -1: read from ctl. VM = false skips the
// von Mises radius draw n4 (a rejection loop, the costly part; it comes after the four Gaussians in the
// substream, so the Gaussians are the same either way)
template <int NM, bool VM = true>
__device__ __forceinline__ void draw_noise(const AsvParams& p, const AsvStepCtl& ctl, uint64_t ctr,
                                          const double* __restrict__ noise, size_t qidx, int slot, int S,
                                          double& n0, double& n1, double& n2, double& n3, double& n4) {
  const int mode = NM >= 0 ? NM : ctl.noise_mode;
  if (mode == 0) {
    const double* nz = noise + (qidx * static_cast<size_t>(S) + slot) * 5;
    n0 = nz[0]; n1 = nz[1]; n2 = nz[2]; n3 = nz[3];
    if (VM) n4 = nz[4];
  } else if (mode == 1) {
    Stream rng(ctl.seed ^ (ctr >> 32) * 0x9E3779B97F4A7C15ull, static_cast<uint32_t>(qidx),
               (static_cast<uint32_t>(qidx >> 32) ^ 0x5EEDu) + (static_cast<uint32_t>(slot) << 20),
               static_cast<uint32_t>(ctr));
    rng.normal2(n0, n1);
    rng.normal2(n2, n3);
    n0 *= p.pos_std; n1 *= p.pos_std; n2 *= p.vel_std; n3 *= p.vel_std;
    if (VM) n4 = rng.vonmises(p.r_kappa);
  } else {
    StreamF rngf(ctl.seed ^ (ctr >> 32) * 0x9E3779B97F4A7C15ull, static_cast<uint32_t>(qidx),
                 (static_cast<uint32_t>(qidx >> 32) ^ 0xF32Au) + (static_cast<uint32_t>(slot) << 20),
                 static_cast<uint32_t>(ctr));
    float f0, f1, f2, f3, u;
    rngf.normal4u(f0, f1, f2, f3, u);
    n0 = f0 * p.pos_std; n1 = f1 * p.pos_std; n2 = f2 * p.vel_std; n3 = f3 * p.vel_std;
    // the default radius noise (r_kappa = 1, wamv.py:24) from the table; other kappas by rejection
    if (VM) n4 = p.r_kappa == 1.0 ? vonmises_k1_icdf(u) : rngf.vonmises(static_cast<float>(p.r_kappa));
  }
}

// Per-robot sweep (AsvEnvLaunch layout 2): one lane per robot, BLOCK / R whole envs per workgroup;
// perception is one serial loop over the robot's candidates (wamv.py:478-511), top-5 kept in registers.
// PR: every robot's own vehicle / perception parameters from s.robot_params (reset_with_eval_config,
// env.py:553-607); the env-level members (rewards, episode limit, core radius) stay p's.
template <int BLOCK, bool PR>
__global__ __launch_bounds__(BLOCK) void env_sweep_kernel(AsvParams p, AsvEnvState s,
                                                          const double* __restrict__ actions,
                                                          const double* __restrict__ noise,
                                                          AsvStepCtl ctl, AsvStepOut out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int R = s.max_robots;
  const int O = s.max_obs;
  const int epb = BLOCK / R;
  const int tid = threadIdx.x;
  const int le = tid / R;
  const int i = tid - le * R;
  const int e = blockIdx.x * epb + le;
  const bool lane_env = (le < epb) && (e < s.n_envs);
  const bool env_on = lane_env && (ctl.env_mask == nullptr || ctl.env_mask[e] != 0);
  if (ctl.env_mask != nullptr && !__syncthreads_or(env_on ? 1 : 0)) return;   // no env of the workgroup is on
  const int nrob = lane_env ? s.n_robots[e] : 0;
  const bool exists = env_on && i < nrob;
  const size_t NT = static_cast<size_t>(s.n_envs) * R;
  const size_t idx = static_cast<size_t>(e) * R + i;
  const AsvParams& P = PR ? s.robot_params[exists ? idx : 0] : p;   // this robot's parameters

  // LDS carve: positions/velocities of the block's robots after the move, their pre-step
  // deactivated flags, the envs' obstacles and per-env reductions.
  double* sx = reinterpret_cast<double*>(smem);
  double* sy = sx + BLOCK;
  double* sv0 = sy + BLOCK;
  double* sv1 = sv0 + BLOCK;
  double* sob = sv1 + BLOCK;                 // [epb][O][3]
  int* salive = reinterpret_cast<int*>(sob + static_cast<size_t>(epb) * O * 3);  // [epb]
  unsigned char* soff = reinterpret_cast<unsigned char*>(salive + epb);         // [BLOCK]

  Regs r{};
  uint8_t fl = 0;
  if (exists) {
    const double* rs = s.rs;
    r.x = rs[ASVRL_F_X * NT + idx];
    r.y = rs[ASVRL_F_Y * NT + idx];
    r.th = rs[ASVRL_F_THETA * NT + idx];
    r.vr0 = rs[ASVRL_F_VR0 * NT + idx];
    r.vr1 = rs[ASVRL_F_VR1 * NT + idx];
    r.vr2 = rs[ASVRL_F_VR2 * NT + idx];
    r.v0 = rs[ASVRL_F_V0 * NT + idx];
    r.v1 = rs[ASVRL_F_V1 * NT + idx];
    r.v2 = rs[ASVRL_F_V2 * NT + idx];
    r.tl = rs[ASVRL_F_TL * NT + idx];
    r.tr = rs[ASVRL_F_TR * NT + idx];
    r.lp = rs[ASVRL_F_LP * NT + idx];
    r.rp = rs[ASVRL_F_RP * NT + idx];
    fl = s.rflags[idx];
  }
  const bool deact = (fl & ASVRL_FLAG_DEACTIVATED) != 0;
  const bool active = exists && !deact;
  const int ep_ts = env_on ? s.ep_ts[e] : 0;
  double gx = 0, gy = 0;
  if (exists) {
    gx = s.rs[ASVRL_F_GX * NT + idx];
    gy = s.rs[ASVRL_F_GY * NT + idx];
  }

  // ---------------- phase 1: dynamics (env.py:247-277)
  double reward = 0.0;
  if (active && ctl.do_dynamics) {
    const double d_before = sqrt((gx - r.x) * (gx - r.x) + (gy - r.y) * (gy - r.y));
    const int nc = s.n_cores[e];
    const double* cores = s.cores + static_cast<size_t>(e) * s.max_cores * 4;
    robot_act(ParamsRef{&P}, r, actions[2 * idx], actions[2 * idx + 1], ctl.is_continuous, cores,
              nc < s.max_cores ? nc : s.max_cores);
    const double d_after = sqrt((gx - r.x) * (gx - r.x) + (gy - r.y) * (gy - r.y));
    reward = 0.0;
    reward += p.timestep_penalty;
    reward += d_before - d_after;
  }

  // ---------------- stage for perception
  sx[tid] = r.x;
  sy[tid] = r.y;
  sv0[tid] = r.v0;
  sv1[tid] = r.v1;
  soff[tid] = exists ? (deact ? 1 : 0) : 1;
  if (env_on) {
    const int no = s.n_obs[e];
    for (int k = i; k < O; k += R) {
      const double* ob = s.obstacles + (static_cast<size_t>(e) * O + k) * 3;
      double* dst = sob + (static_cast<size_t>(le) * O + k) * 3;
      if (k < no) {
        dst[0] = ob[0];
        dst[1] = ob[1];
        dst[2] = ob[2];
      }
    }
    if (i == 0) salive[le] = 0;
  }
  __syncthreads();

  // ---------------- phase 2: perception_output (wamv.py:436-529)
  bool coll = (fl & ASVRL_FLAG_COLLISION) != 0;
  bool reach = (fl & ASVRL_FLAG_REACH_GOAL) != 0;
  bool apply = false;
  double phi = exists ? s.rs[ASVRL_F_PHI * NT + idx] : 0.0;
  int cnt = -1;
  Cand t0{INFINITY, 0, 0, 0, 0, 0}, t1 = t0, t2 = t0, t3 = t0, t4 = t0;
  double so0 = 0, so1 = 0, so2 = 0, so3 = 0, so4 = 0;
  if (active) {
    double sn, cs;
    sincos(r.th, &sn, &cs);
    const double tx = -(cs * r.x + sn * r.y);
    const double ty = -(-sn * r.x + cs * r.y);
    so0 = (cs * gx + sn * gy) + tx;
    so1 = (-sn * gx + cs * gy) + ty;
    so2 = cs * r.v0 + sn * r.v1;
    so3 = -sn * r.v0 + cs * r.v1;
    so4 = r.v2;
    if (sqrt((gx - r.x) * (gx - r.x) + (gy - r.y) * (gy - r.y)) <= P.goal_dis) reach = true;

    int nkept = 0;
    const int no = s.n_obs[e];
    const int base = le * R;
    const uint64_t ctr = ctl.counter + (ctl.counter_dev != nullptr ? *ctl.counter_dev : 0ull);
    const int ncand = no + nrob;
    const bool full_circle = 0.5 * P.angle >= kPi;
    for (int k = 0; k < ncand; ++k) {
      double ox, oy, orad, vx0, vy0;
      int slot;
      if (k < no) {
        const double* ob = sob + (static_cast<size_t>(le) * O + k) * 3;
        ox = ob[0];
        oy = ob[1];
        orad = ob[2];
        vx0 = 0.0;
        vy0 = 0.0;
        slot = k;
      } else {
        const int j = k - no;
        if (j == i || soff[base + j]) continue;  // self / deactivated (wamv.py:487-491)
        ox = sx[base + j];
        oy = sy[base + j];
        orad = PR ? s.robot_params[static_cast<size_t>(e) * R + j].r : p.r;   // the other robot's r
        vx0 = sv0[base + j];
        vy0 = sv1[base + j];
        slot = O + j;
      }
      double n0, n1, n2, n3, n4;
      draw_noise<-1>(P, ctl, ctr, noise, idx, slot, O + R, n0, n1, n2, n3, n4);
      const double pxn = ox + n0, pyn = oy + n1;  // Perception (wamv.py:27-40)
      const double vxn = vx0 + n2, vyn = vy0 + n3;
      const double rn = P.r_mean_ratio * orad + (1 - P.r_mean_ratio) * n4 / kPi * orad;
      const double qx = (cs * pxn + sn * pyn) + tx, qy = (-sn * pxn + cs * pyn) + ty;
      const double qn = sqrt(qx * qx + qy * qy);
      if (qn > P.range + rn) continue;  // check_detection (wamv.py:293-303)
      if (!full_circle) {              // atan2 lies in [-pi, pi]: the test only bites when angle < 2 pi
        const double ang = atan2(qy, qx);
        if (ang < -0.5 * P.angle || ang > 0.5 * P.angle) continue;
      }
      if (!coll) {  // check_collision (wamv.py:281-291), true positions
        const double d = sqrt((r.x - ox) * (r.x - ox) + (r.y - oy) * (r.y - oy)) - orad - P.r;
        if (d <= 0.0) coll = true;
      }
      Cand cd{qn - rn - P.r, qx, qy, cs * vxn + sn * vyn, -sn * vxn + cs * vyn, rn};
      // heapq.nsmallest == stable ascending order: a new candidate passes equal keys
      cswap(cd.key < t0.key, cd, t0);
      cswap(cd.key < t1.key, cd, t1);
      cswap(cd.key < t2.key, cd, t2);
      cswap(cd.key < t3.key, cd, t3);
      cswap(cd.key < t4.key, cd, t4);
      ++nkept;
    }
    cnt = nkept < P.max_obj_num ? nkept : P.max_obj_num;
    // COLREGs over the kept objects in order, stop at the first hit (wamv.py:517-521)
    if (cnt > 0) apply = colregs(P.r, cs, sn, r.v0, r.v1, t0.a, t0.b, t0.c, t0.d, t0.e, phi);
    if (!apply && cnt > 1) apply = colregs(P.r, cs, sn, r.v0, r.v1, t1.a, t1.b, t1.c, t1.d, t1.e, phi);
    if (!apply && cnt > 2) apply = colregs(P.r, cs, sn, r.v0, r.v1, t2.a, t2.b, t2.c, t2.d, t2.e, phi);
    if (!apply && cnt > 3) apply = colregs(P.r, cs, sn, r.v0, r.v1, t3.a, t3.b, t3.c, t3.d, t3.e, phi);
    if (!apply && cnt > 4) apply = colregs(P.r, cs, sn, r.v0, r.v1, t4.a, t4.b, t4.c, t4.d, t4.e, phi);
  }

  const StepResult res = step_result(p, ctl, exists, deact, active, ep_ts, fl, coll, reach, apply, phi, reward,
                                     exists ? s.rs[ASVRL_F_RET * NT + idx] : 0.0);
  if (ctl.trainer_deactivate && ctl.do_dynamics && exists && !(res.nfl & ASVRL_FLAG_DEACTIVATED))
    atomicAdd(&salive[le], 1);

  // ---------------- write back
  if (exists) {
    double* rs = s.rs;
    if (ctl.do_dynamics) {
      rs[ASVRL_F_X * NT + idx] = r.x;
      rs[ASVRL_F_Y * NT + idx] = r.y;
      rs[ASVRL_F_THETA * NT + idx] = r.th;
      rs[ASVRL_F_VR0 * NT + idx] = r.vr0;
      rs[ASVRL_F_VR1 * NT + idx] = r.vr1;
      rs[ASVRL_F_VR2 * NT + idx] = r.vr2;
      rs[ASVRL_F_V0 * NT + idx] = r.v0;
      rs[ASVRL_F_V1 * NT + idx] = r.v1;
      rs[ASVRL_F_V2 * NT + idx] = r.v2;
      rs[ASVRL_F_TL * NT + idx] = r.tl;
      rs[ASVRL_F_TR * NT + idx] = r.tr;
      rs[ASVRL_F_RET * NT + idx] = res.ret;
    }
    rs[ASVRL_F_PHI * NT + idx] = phi;
    s.rflags[idx] = res.nfl;
  }
  if (env_on && i < R) {
    // packed f32 obs row (replay_buffer.py:51-69 + the .float() of agent.py:363-366)
    float4* o4 = reinterpret_cast<float4*>(out.obs + idx * ASVRL_OBS_DIM);
    const bool a = active;
    const float m0 = (a && cnt > 0) ? 1.f : 0.f, m1 = (a && cnt > 1) ? 1.f : 0.f,
                m2 = (a && cnt > 2) ? 1.f : 0.f, m3 = (a && cnt > 3) ? 1.f : 0.f,
                m4 = (a && cnt > 4) ? 1.f : 0.f;
    auto f = [](double v, float m) { return m != 0.f ? static_cast<float>(v) : 0.f; };
    const float sf = a ? 1.f : 0.f;
    o4[0] = make_float4(f(so0, sf), f(so1, sf), f(so2, sf), f(so3, sf));
    o4[1] = make_float4(f(so4, sf), f(r.tl, sf), f(r.tr, sf), f(t0.a, m0));
    o4[2] = make_float4(f(t0.b, m0), f(t0.c, m0), f(t0.d, m0), f(t0.e, m0));
    o4[3] = make_float4(f(t1.a, m1), f(t1.b, m1), f(t1.c, m1), f(t1.d, m1));
    o4[4] = make_float4(f(t1.e, m1), f(t2.a, m2), f(t2.b, m2), f(t2.c, m2));
    o4[5] = make_float4(f(t2.d, m2), f(t2.e, m2), f(t3.a, m3), f(t3.b, m3));
    o4[6] = make_float4(f(t3.c, m3), f(t3.d, m3), f(t3.e, m3), f(t4.a, m4));
    o4[7] = make_float4(f(t4.b, m4), f(t4.c, m4), f(t4.d, m4), f(t4.e, m4));
    o4[8] = make_float4(m0, m1, m2, m3);
    o4[9] = make_float4(m4, 0.f, 0.f, 0.f);
    if (out.obs64 != nullptr) {
      double* o = out.obs64 + idx * 32;
      const double v[32] = {so0, so1, so2, so3, so4, r.tl, r.tr,
                            t0.a, t0.b, t0.c, t0.d, t0.e, t1.a, t1.b, t1.c, t1.d, t1.e,
                            t2.a, t2.b, t2.c, t2.d, t2.e, t3.a, t3.b, t3.c, t3.d, t3.e,
                            t4.a, t4.b, t4.c, t4.d, t4.e};
#pragma unroll
      for (int k = 0; k < 32; ++k) {
        const bool keep = a && (k < 7 || (k - 7) / 5 < cnt);
        o[k] = keep ? v[k] : 0.0;
      }
    }
    out.obj_cnt[idx] = static_cast<int8_t>(exists ? cnt : -1);
    out.reward[idx] = res.reward;
    out.done[idx] = res.done;
    out.info[idx] = res.info;
  }
  __syncthreads();
  if (env_on && i == 0 && ctl.do_dynamics) env_end(p, s, ctl, out, e, ep_ts, nrob, salive[le], NT);
}

// Pair-parallel env step (AsvEnvLaunch layout 1). A workgroup owns `epb` whole envs; their robots
// occupy its first nrb = epb * R lanes. Phases, each over all lanes, separated by workgroup barriers:
//   1  robot lanes: N Fossen substeps in registers, state written back, the observation's self part,
//      the robot's frame, position and velocity into LDS
//   2  one lane per (robot, candidate slot) pair: noise, detection, collision, sort key -- 13 B per
//      pair in LDS (key, von Mises draw, flag; 17 B with f64 draws)
//   3  robot lanes: the stable top-5 of the keys in the reference's order (slot indices only), collision
//      as an OR
//   4  one lane per kept object (a work list built by a scan of the counts): the object's row
//      recomputed from the same noise draw and arithmetic as in phase 2 (bit-identical; the von Mises
//      radius draw kept from phase 2, the Gaussians redrawn), written into the observation; its
//      COLREGs test
//   5  robot lanes: the first COLREGs hit in order and the phi the reference's serial chain leaves,
//      reward / done / info, trainer bookkeeping; then the per-env episode end
// No phase keeps another's values in registers and LDS holds ~15 KB per 12-env workgroup, so several
// workgroups share a CU (the round-1 form kept 40-B rows per pair and the top-5 rows in registers:
// 239 VGPRs, 35 KB, two waves per SIMD).
#ifndef ASVRL_ENV_PAIRS_WPE
#define ASVRL_ENV_PAIRS_WPE 4
#endif
// one workgroup's envs [bid * epb, (bid + 1) * epb) of the step (env_pairs_kernel loops over them)
template <int BLOCK, int NM, bool DYN = true>   // DYN false: an observation pass only (do_dynamics = 0)
__device__ __forceinline__ void env_pairs_block(KArg<PairsArgs> A, int epb, int bid, unsigned char* smem) {
  const int R = A->s.max_robots;
  const int O = A->s.max_obs;
  const int S = O + R;               // candidate slots per robot (obstacles, then robots)
  const int nrb = epb * R;
  const int npairs = nrb * S;
  const int nslot = npairs > 5 * nrb ? npairs : 5 * nrb;
  const int tid = threadIdx.x;

  double* sx = reinterpret_cast<double*>(smem);   // [nrb] robots after the move
  double* sy = sx + nrb;
  double* sv0 = sy + nrb;
  double* sv1 = sv0 + nrb;
  double* scs = sv1 + nrb;           // robot frame: cos, sin, translation
  double* ssn = scs + nrb;
  double* stx = ssn + nrb;
  double* sty = stx + nrb;
  double* pk = sty + nrb;            // [nslot] phase 2 sort keys; phase 4 phi of (robot, k)
  double* sob = pk + nslot;          // [epb][O][3]
  using VmT = typename std::conditional<NM == 2, float, double>::type;   // the f32 stream's draw is a float
  VmT* pvm = reinterpret_cast<VmT*>(sob + static_cast<size_t>(epb) * O * 3);  // [npairs] von Mises radius draws
  int* salive = reinterpret_cast<int*>(pvm + npairs);  // [epb]
  int* sno = salive + epb;           // [epb] obstacles, robots of each env
  int* snr = sno + epb;
  int* swt = snr + epb;              // [BLOCK / 64] kept objects per wave (phase 3 scan)
  unsigned short* skept = reinterpret_cast<unsigned short*>(swt + BLOCK / kWave);  // [nrb][5] kept slots in order
  unsigned short* sitem = skept + 5 * nrb;   // [5 * nrb] phase 4 work list: robot * 5 + k of every kept object
  unsigned char* pfl = reinterpret_cast<unsigned char*>(sitem + 5 * nrb);  // [nslot] 1 detected | 2 collision; phase 4: 1 evaluated | 2 hit
  unsigned char* soff = pfl + nslot;   // [nrb] not a candidate (absent / deactivated before the step)
  unsigned char* sact = soff + nrb;    // [nrb] active
  signed char* scnt = reinterpret_cast<signed char*>(sact + nrb);  // [nrb] kept count, -1 inactive

  const bool rlane = tid < nrb;
  const int le = tid / R;
  const int i = tid - le * R;
  const int e = bid * epb + le;
  const bool lane_env = rlane && e < A->s.n_envs;
  const bool env_on = lane_env && (A->ctl.env_mask == nullptr || A->ctl.env_mask[e] != 0);
  // a masked pass (the observation pass after a reset) touches few envs: workgroups with none leave
  if (A->ctl.env_mask != nullptr && !__syncthreads_or(env_on ? 1 : 0)) return;
  const int nrob = lane_env ? A->s.n_robots[e] : 0;
  const bool exists = env_on && i < nrob;
  const size_t NT = static_cast<size_t>(A->s.n_envs) * R;
  const size_t idx = static_cast<size_t>(e) * R + i;
  const uint8_t fl = exists ? A->s.rflags[idx] : 0;
  const bool deact = (fl & ASVRL_FLAG_DEACTIVATED) != 0;
  const bool active = exists && !deact;
  const int ep_ts = env_on ? A->s.ep_ts[e] : 0;
  bool coll = (fl & ASVRL_FLAG_COLLISION) != 0;
  bool reach = (fl & ASVRL_FLAG_REACH_GOAL) != 0;
  double reward = 0.0;

  // ---------------- phase 1: dynamics (env.py:247-277), the observation's self part
  {
    Regs r{};
    double gx = 0, gy = 0;
    if (exists) {
      const double* rs = A->s.rs;
      r.x = rs[ASVRL_F_X * NT + idx];
      r.y = rs[ASVRL_F_Y * NT + idx];
      r.th = rs[ASVRL_F_THETA * NT + idx];
      r.vr0 = rs[ASVRL_F_VR0 * NT + idx];
      r.vr1 = rs[ASVRL_F_VR1 * NT + idx];
      r.vr2 = rs[ASVRL_F_VR2 * NT + idx];
      r.v0 = rs[ASVRL_F_V0 * NT + idx];
      r.v1 = rs[ASVRL_F_V1 * NT + idx];
      r.v2 = rs[ASVRL_F_V2 * NT + idx];
      r.tl = rs[ASVRL_F_TL * NT + idx];
      r.tr = rs[ASVRL_F_TR * NT + idx];
      r.lp = rs[ASVRL_F_LP * NT + idx];
      r.rp = rs[ASVRL_F_RP * NT + idx];
      gx = rs[ASVRL_F_GX * NT + idx];
      gy = rs[ASVRL_F_GY * NT + idx];
    }
    if (active && (DYN && A->ctl.do_dynamics)) {
      const double d_before = sqrt((gx - r.x) * (gx - r.x) + (gy - r.y) * (gy - r.y));
      const int nc = A->s.n_cores[e];
      const double* cores = A->s.cores + static_cast<size_t>(e) * A->s.max_cores * 4;
      robot_act(ParamsKArg{&A->p}, r, A->actions[2 * idx], A->actions[2 * idx + 1], A->ctl.is_continuous, cores,
                nc < A->s.max_cores ? nc : A->s.max_cores);
      const double d_after = sqrt((gx - r.x) * (gx - r.x) + (gy - r.y) * (gy - r.y));
      reward = 0.0;
      reward += A->p.timestep_penalty;
      reward += d_before - d_after;
    }
    if (exists && (DYN && A->ctl.do_dynamics)) {
      double* rs = A->s.rs;
      rs[ASVRL_F_X * NT + idx] = r.x;
      rs[ASVRL_F_Y * NT + idx] = r.y;
      rs[ASVRL_F_THETA * NT + idx] = r.th;
      rs[ASVRL_F_VR0 * NT + idx] = r.vr0;
      rs[ASVRL_F_VR1 * NT + idx] = r.vr1;
      rs[ASVRL_F_VR2 * NT + idx] = r.vr2;
      rs[ASVRL_F_V0 * NT + idx] = r.v0;
      rs[ASVRL_F_V1 * NT + idx] = r.v1;
      rs[ASVRL_F_V2 * NT + idx] = r.v2;
      rs[ASVRL_F_TL * NT + idx] = r.tl;
      rs[ASVRL_F_TR * NT + idx] = r.tr;
    }
    double so0 = 0, so1 = 0, so2 = 0, so3 = 0, so4 = 0;
    if (rlane) {
      sx[tid] = r.x;
      sy[tid] = r.y;
      sv0[tid] = r.v0;
      sv1[tid] = r.v1;
      soff[tid] = exists ? (deact ? 1 : 0) : 1;
      sact[tid] = active ? 1 : 0;
    }
    if (active) {
      double sn, cs;
      sincos(r.th, &sn, &cs);
      const double tx = -(cs * r.x + sn * r.y);
      const double ty = -(-sn * r.x + cs * r.y);
      scs[tid] = cs;
      ssn[tid] = sn;
      stx[tid] = tx;
      sty[tid] = ty;
      so0 = (cs * gx + sn * gy) + tx;
      so1 = (-sn * gx + cs * gy) + ty;
      so2 = cs * r.v0 + sn * r.v1;
      so3 = -sn * r.v0 + cs * r.v1;
      so4 = r.v2;
      if (sqrt((gx - r.x) * (gx - r.x) + (gy - r.y) * (gy - r.y)) <= A->p.goal_dis) reach = true;
    }
    if (env_on) {   // packed f32 obs row, self part (replay_buffer.py:51-69 + the .float() of agent.py:363-366)
      float* of = A->out.obs + idx * ASVRL_OBS_DIM;
      const bool a = active;
      *reinterpret_cast<float4*>(of) = a ? make_float4(static_cast<float>(so0), static_cast<float>(so1),
                                                        static_cast<float>(so2), static_cast<float>(so3))
                                         : make_float4(0.f, 0.f, 0.f, 0.f);
      of[4] = a ? static_cast<float>(so4) : 0.f;
      of[5] = a ? static_cast<float>(r.tl) : 0.f;
      of[6] = a ? static_cast<float>(r.tr) : 0.f;
      if (A->out.obs64 != nullptr) {
        double* o = A->out.obs64 + idx * 32;
        o[0] = a ? so0 : 0.0;
        o[1] = a ? so1 : 0.0;
        o[2] = a ? so2 : 0.0;
        o[3] = a ? so3 : 0.0;
        o[4] = a ? so4 : 0.0;
        o[5] = a ? r.tl : 0.0;
        o[6] = a ? r.tr : 0.0;
      }
    }
  }
  if (env_on) {
    const int no = A->s.n_obs[e];
    for (int k = i; k < O; k += R) {
      const double* ob = A->s.obstacles + (static_cast<size_t>(e) * O + k) * 3;
      double* dst = sob + (static_cast<size_t>(le) * O + k) * 3;
      if (k < no) {
        dst[0] = ob[0];
        dst[1] = ob[1];
        dst[2] = ob[2];
      }
    }
    if (i == 0) {
      salive[le] = 0;
      sno[le] = no;
      snr[le] = nrob;
    }
  }
  __syncthreads();
  A = kfresh(A);

  // candidate slot c of robot qi in local env qe: obstacles first, then robots (self, deactivated and
  // absent ones are not candidates, wamv.py:487-491)
  auto candidate = [&](int qe, int qi, int c, double& ox, double& oy, double& orad, double& vx0, double& vy0) {
    if (c < O) {
      if (c >= sno[qe]) return false;
      const double* ob = sob + (static_cast<size_t>(qe) * O + c) * 3;
      ox = ob[0];
      oy = ob[1];
      orad = ob[2];
      vx0 = 0.0;
      vy0 = 0.0;
      return true;
    }
    const int j = c - O;
    if (!(j < snr[qe] && j != qi && !soff[qe * R + j])) return false;
    ox = sx[qe * R + j];
    oy = sy[qe * R + j];
    orad = A->p.r;
    vx0 = sv0[qe * R + j];
    vy0 = sv1[qe * R + j];
    return true;
  };
  const uint64_t ctr = A->ctl.counter + (A->ctl.counter_dev != nullptr ? *A->ctl.counter_dev : 0ull);
  const bool full_circle = 0.5 * A->p.angle >= kPi;

  // ---------------- phase 2: one (robot, candidate) pair per lane (wamv.py:478-511)
  const KArg<PairsArgs> A_loop = A;
  for (int q = tid; q < npairs; q += BLOCK) {
    const KArg<PairsArgs> A = kfresh(A_loop);   // this iteration's parameters, not held across iterations
    const int qr = q / S;
    const int c = q - qr * S;
    const int qe = qr / R;
    const int qi = qr - qe * R;
    unsigned char flag = 0;
    double key = INFINITY;
    double ox = 0, oy = 0, orad = 0, vx0 = 0, vy0 = 0;
    if (sact[qr] && candidate(qe, qi, c, ox, oy, orad, vx0, vy0)) {
      const size_t qidx = static_cast<size_t>(bid * epb + qe) * R + qi;
      double n0, n1, n2, n3, n4;
      draw_noise<NM>(kref(A).p, kref(A).ctl, ctr, A->noise, qidx, c, S, n0, n1, n2, n3, n4);
      pvm[q] = static_cast<VmT>(n4);
      const double cs = scs[qr], sn = ssn[qr], tx = stx[qr], ty = sty[qr];
      const double pxn = ox + n0, pyn = oy + n1;  // Perception (wamv.py:27-40)
      const double rn = A->p.r_mean_ratio * orad + (1 - A->p.r_mean_ratio) * n4 / kPi * orad;
      const double qx = (cs * pxn + sn * pyn) + tx, qy = (-sn * pxn + cs * pyn) + ty;
      const double qn = sqrt(qx * qx + qy * qy);
      bool det = qn <= A->p.range + rn;  // check_detection (wamv.py:293-303)
      if (det && !full_circle) {
        const double ang = atan2(qy, qx);
        det = !(ang < -0.5 * A->p.angle || ang > 0.5 * A->p.angle);
      }
      if (det) {
        flag = 1;
        const double rx = sx[qr], ry = sy[qr];   // check_collision (wamv.py:281-291), true positions
        const double d = sqrt((rx - ox) * (rx - ox) + (ry - oy) * (ry - oy)) - orad - A->p.r;
        if (d <= 0.0) flag |= 2;
        key = qn - rn - A->p.r;
      }
    }
    pk[q] = key;
    pfl[q] = flag;
  }
  __syncthreads();
  A = kfresh(A);

  // ---------------- phase 3: the robot's candidates in the reference's order (wamv.py:512-516)
  int cnt = -1;
  if (active) {
    double k0 = INFINITY, k1 = INFINITY, k2 = INFINITY, k3 = INFINITY, k4 = INFINITY;
    int c0 = 0, c1 = 0, c2 = 0, c3 = 0, c4 = 0;
    int nkept = 0;
    const int q0 = tid * S;
    for (int c = 0; c < S; ++c) {
      const unsigned char f = pfl[q0 + c];
      if (!(f & 1)) continue;
      if (f & 2) coll = true;
      double kc = pk[q0 + c];
      int cc = c;
      // heapq.nsmallest == stable ascending order: a new candidate passes equal keys
      auto ins = [&](double& kk, int& ck) {
        if (kc < kk) {
          const double tk = kk;
          const int tc = ck;
          kk = kc;
          ck = cc;
          kc = tk;
          cc = tc;
        }
      };
      ins(k0, c0);
      ins(k1, c1);
      ins(k2, c2);
      ins(k3, c3);
      ins(k4, c4);
      ++nkept;
    }
    cnt = nkept < A->p.max_obj_num ? nkept : A->p.max_obj_num;
    unsigned short* kp = skept + 5 * tid;
    kp[0] = static_cast<unsigned short>(c0);
    kp[1] = static_cast<unsigned short>(c1);
    kp[2] = static_cast<unsigned short>(c2);
    kp[3] = static_cast<unsigned short>(c3);
    kp[4] = static_cast<unsigned short>(c4);
  }
  if (rlane) scnt[tid] = static_cast<signed char>(cnt);
  // phase 4's work list: the kept objects only (about half of the 5 * nrb (robot, k) slots), placed by
  // a workgroup scan of the counts in robot order
  const int lane = tid & (kWave - 1);
  int kin = cnt > 0 ? cnt : 0;
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const int t = __shfl_up(kin, d);
    if (lane >= d) kin += t;
  }
  if (lane == kWave - 1) swt[tid / kWave] = kin;
  __syncthreads();
  A = kfresh(A);
  int nitem = 0, ibase = 0;
#pragma unroll
  for (int w = 0; w < BLOCK / kWave; ++w) {
    ibase += w < tid / kWave ? swt[w] : 0;
    nitem += swt[w];
  }
  if (cnt > 0) {
    const int off = ibase + kin - cnt;
    for (int k = 0; k < cnt; ++k) sitem[off + k] = static_cast<unsigned short>(5 * tid + k);
  }
  __syncthreads();
  A = kfresh(A);

  // ---------------- phase 4: one lane per kept object: its observation row and COLREGs test
  const KArg<PairsArgs> A_loop4 = A;
  for (int it = tid; it < nitem; it += BLOCK) {
    const KArg<PairsArgs> A = kfresh(A_loop4);   // this iteration's parameters, not held across iterations
    const int kq = sitem[it];
    const int qr = kq / 5;
    const int k = kq - 5 * qr;
    const int qe = qr / R;
    const int qi = qr - qe * R;
    const int e2 = bid * epb + qe;
    unsigned char cf = 0;
    double ph = 0.0;
    {
      const size_t qidx = static_cast<size_t>(e2) * R + qi;
      double ra, rb, rc, rd, re;
      {
        const int c = skept[kq];
        double ox = 0, oy = 0, orad = 0, vx0 = 0, vy0 = 0;
        candidate(qe, qi, c, ox, oy, orad, vx0, vy0);
        double n0, n1, n2, n3, n4 = static_cast<double>(pvm[qr * S + c]);
        draw_noise<NM, false>(kref(A).p, kref(A).ctl, ctr, A->noise, qidx, c, S, n0, n1, n2, n3, n4);
        const double cs = scs[qr], sn = ssn[qr], tx = stx[qr], ty = sty[qr];
        const double pxn = ox + n0, pyn = oy + n1;  // as phase 2
        const double vxn = vx0 + n2, vyn = vy0 + n3;
        const double rn = A->p.r_mean_ratio * orad + (1 - A->p.r_mean_ratio) * n4 / kPi * orad;
        ra = (cs * pxn + sn * pyn) + tx;
        rb = (-sn * pxn + cs * pyn) + ty;
        rc = cs * vxn + sn * vyn;
        rd = -sn * vxn + cs * vyn;
        re = rn;
        if (!(sqrt(rc * rc + rd * rd) < 0.5)) {   // colregs_body's first test, ahead of the call
          bool ev;
          const bool hit = colregs_ev(A->p.r, cs, sn, sv0[qr], sv1[qr], ra, rb, rc, rd, re, ph, ev);
          cf = static_cast<unsigned char>((ev ? 1 : 0) | (hit ? 2 : 0));
        }
      }
      float* of = A->out.obs + qidx * ASVRL_OBS_DIM + 7 + 5 * k;
      of[0] = static_cast<float>(ra);
      of[1] = static_cast<float>(rb);
      of[2] = static_cast<float>(rc);
      of[3] = static_cast<float>(rd);
      of[4] = static_cast<float>(re);
      if (A->out.obs64 != nullptr) {
        double* o = A->out.obs64 + qidx * 32 + 7 + 5 * k;
        o[0] = ra;
        o[1] = rb;
        o[2] = rc;
        o[3] = rd;
        o[4] = re;
      }
    }
    pfl[kq] = cf;
    pk[kq] = ph;
  }
  __syncthreads();
  A = kfresh(A);

  // ---------------- phase 5: COLREGs in order (wamv.py:517-521), reward / done / info, bookkeeping
  bool apply = false;
  double phi = exists ? A->s.rs[ASVRL_F_PHI * NT + idx] : 0.0;
  for (int k = 0; k < cnt; ++k) {   // the serial chain: phi of every evaluated object up to the first hit
    const unsigned char f = pfl[5 * tid + k];
    if (f & 1) phi = pk[5 * tid + k];
    if (f & 2) {
      apply = true;
      break;
    }
  }
  const StepResult res = step_result(kref(A).p, kref(A).ctl, exists, deact, active, ep_ts, fl, coll, reach, apply, phi, reward,
                                     exists ? A->s.rs[ASVRL_F_RET * NT + idx] : 0.0);
  if (A->ctl.trainer_deactivate && (DYN && A->ctl.do_dynamics) && exists && !(res.nfl & ASVRL_FLAG_DEACTIVATED))
    atomicAdd(&salive[le], 1);
  if (exists) {
    if ((DYN && A->ctl.do_dynamics)) A->s.rs[ASVRL_F_RET * NT + idx] = res.ret;
    A->s.rs[ASVRL_F_PHI * NT + idx] = phi;
    A->s.rflags[idx] = res.nfl;
  }
  if (env_on) {
    float4* o4 = reinterpret_cast<float4*>(A->out.obs + idx * ASVRL_OBS_DIM);
    const bool a = active;
    for (int k = cnt > 0 ? cnt : 0; k < 5; ++k) {   // the object rows phase 4 did not write
      float* of = A->out.obs + idx * ASVRL_OBS_DIM + 7 + 5 * k;
      of[0] = 0.f;
      of[1] = 0.f;
      of[2] = 0.f;
      of[3] = 0.f;
      of[4] = 0.f;
      if (A->out.obs64 != nullptr) {
        double* o = A->out.obs64 + idx * 32 + 7 + 5 * k;
        o[0] = 0.0;
        o[1] = 0.0;
        o[2] = 0.0;
        o[3] = 0.0;
        o[4] = 0.0;
      }
    }
    o4[8] = make_float4((a && cnt > 0) ? 1.f : 0.f, (a && cnt > 1) ? 1.f : 0.f, (a && cnt > 2) ? 1.f : 0.f,
                        (a && cnt > 3) ? 1.f : 0.f);
    o4[9] = make_float4((a && cnt > 4) ? 1.f : 0.f, 0.f, 0.f, 0.f);
    A->out.obj_cnt[idx] = static_cast<int8_t>(exists ? cnt : -1);
    A->out.reward[idx] = res.reward;
    A->out.done[idx] = res.done;
    A->out.info[idx] = res.info;
  }
  __syncthreads();
  A = kfresh(A);
  if (env_on && i == 0 && (DYN && A->ctl.do_dynamics)) env_end(kref(A).p, kref(A).s, kref(A).ctl, kref(A).out, e, ep_ts, nrob, salive[le], NT);
}


// The step kernel: workgroup b takes env group group0 + b (a step may be split into launches of at most
// AsvEnvLaunch.max_groups workgroups, one after another: the rollout's share of the chip beside the learner).
// XCD-aware (1): the dispatcher deals workgroups to the eight XCDs round-robin, so consecutive env groups --
// whose state / observation rows share cache lines at their edges -- would sit in different L2s and each
// write back its part of the shared lines; the bijection below gives each XCD a contiguous run of groups.
#ifndef ASVRL_ENV_XCD_SWIZZLE
#define ASVRL_ENV_XCD_SWIZZLE 1
#endif
__device__ __forceinline__ int xcd_group(int x, int n) {
#if ASVRL_ENV_XCD_SWIZZLE
  constexpr int kXcd = 8;
  const int q = n / kXcd, rr = n % kXcd, xcd = x % kXcd, k = x / kXcd;
  return (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + k;
#else
  (void)n;
  return x;
#endif
}
template <int BLOCK, int NM>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(NM == 1 ? 1 : ASVRL_ENV_PAIRS_WPE))) void env_pairs_kernel(PairsArgs) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const KArg<PairsArgs> A = kargs<PairsArgs>();
  env_pairs_block<BLOCK, NM>(A, A->epb,
                             A->group0 + xcd_group(static_cast<int>(blockIdx.x), static_cast<int>(gridDim.x)), smem);
}

// ------------------------------------------------------------------ reset (env.py:72-164)
__device__ inline bool far_enough(double ax, double ay, double bx, double by, double lim, bool strict) {
  const double dx = ax - bx, dy = ay - by;
  const double d = sqrt(dx * dx + dy * dy);
  return strict ? !(d <= lim) : !(d < lim);
}

// One wave per env being reset. Every phase is rejection sampling with at most 500 draws in
// the reference's order (robots env.py:106-120, cores :123-136 with check_core :378-418,
// obstacles :151-162 with check_obstacle :420-456). The wave draws 64 consecutive candidates at
// once (candidate c's values come from its own Philox counter (c, env, phase, step), not from a
// shared stream) and tests each against everything accepted so far; then, while the batch holds a
// valid one, it accepts the lowest-numbered (ballot), broadcasts its values (v_readlane) and drops the
// candidates before it and those conflicting with it -- the same accepted sequence as testing the
// candidates one by one (a rejected candidate stays rejected as the accepted set grows; a later one is
// valid iff it is valid against the old set and the new member). Each batch's draws and tests against
// the set are made once (round 4's kernel restarted the batch after every acceptance, redrawing and
// retesting up to 63 candidates each time). The accepted set of the phase lives in LDS for the phases
// after it. Restated one candidate at a time by oracle/asv_oracle.c or_device_reset (bit-identical:
// tests/test_env_kernel_gpu.py).
constexpr int kResetWaves = 4;
constexpr int kResetMaxR = 32;
constexpr int kResetMaxO = 32;

struct CandDraw {
  uint32_t k0, k1, e, ctr;
  __device__ double u(int phase, int cand, int j) const {   // j-th double of candidate cand
    const U4 r = philox4x32_10(U4{static_cast<uint32_t>(cand) * 4u + static_cast<uint32_t>(j >> 1), e,
                                  static_cast<uint32_t>(phase), ctr}, k0, k1);
    const uint64_t hi = (j & 1) ? r.z : r.x, lo = (j & 1) ? r.w : r.y;
    const uint64_t bits = ((hi << 32) | lo) >> 11;
    return (static_cast<double>(bits) + 1.0) * (1.0 / 9007199254740992.0);
  }
  // both doubles of one Philox call (j = 2 p, 2 p + 1)
  __device__ void u2(int phase, int cand, int p, double& a, double& b) const {
    const U4 r = philox4x32_10(U4{static_cast<uint32_t>(cand) * 4u + static_cast<uint32_t>(p), e,
                                  static_cast<uint32_t>(phase), ctr}, k0, k1);
    a = (static_cast<double>(((static_cast<uint64_t>(r.x) << 32) | r.y) >> 11) + 1.0) * (1.0 / 9007199254740992.0);
    b = (static_cast<double>(((static_cast<uint64_t>(r.z) << 32) | r.w) >> 11) + 1.0) * (1.0 / 9007199254740992.0);
  }
};

// lane f's value (f wave-uniform, from a ballot) in every lane
__device__ __forceinline__ double bcast(double v, int f) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(u), f);
  const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(u >> 32), f);
  return __builtin_bit_cast(double, (static_cast<uint64_t>(hi) << 32) | lo);
}

// check_core (env.py:378-418) of candidate (cx, cy, cw, Gamma) against accepted core (qx, qy, qw, qG):
// true when they conflict
__device__ __forceinline__ bool core_conflict(const AsvResetCfg& cfg, double core_r, double qx, double qy, double qw,
                                              double qG, double cx, double cy, double cw, double Gamma) {
  const double dx = qx - cx, dy = qy - cy;
  const double dis = sqrt(dx * dx + dy * dy);
  if (qw == cw) {
    const double bi = qG / (2 * kPi * cfg.v_rel_max);
    const double bj = Gamma / (2 * kPi * cfg.v_rel_max);
    return dis < bi + bj;
  }
  const double gl = fmax(qG, Gamma), gs = fmin(qG, Gamma);
  const double v1 = gl / (2 * kPi * (dis - 2 * core_r));
  const double v2 = gs / (2 * kPi * core_r);
  return v1 > cfg.p_rel * v2;
}

// The accepted sets of one env's reset, in the resetting wave's LDS
struct ResetLds {
  double rob[4][kResetMaxR];      // x, y, gx, gy of accepted robots
  double core[kMaxCores][4];      // x, y, clockwise, Gamma
  double obs[kResetMaxO][3];      // x, y, r
};

// env e's reset by one wave (lane = its lane index)
__device__ __forceinline__ void reset_env(const AsvParams& p, const AsvEnvState& s, const AsvResetCfg& cfg, int e,
                                          uint64_t seed, uint64_t ctr, int lane, ResetLds& W) {
  double (*srob)[kResetMaxR] = W.rob;
  double (*score)[4] = W.core;
  double (*sobs)[3] = W.obs;
  const int R = s.max_robots, O = s.max_obs, Cmax = s.max_cores;
  const size_t NT = static_cast<size_t>(s.n_envs) * R;
  double* rs = s.rs;
  const uint64_t key = seed ^ (ctr >> 32) * 0x9E3779B97F4A7C15ull;
  const CandDraw g{static_cast<uint32_t>(key), static_cast<uint32_t>(key >> 32), static_cast<uint32_t>(e),
                   static_cast<uint32_t>(ctr)};
  constexpr int kDraws = 500;

  // ---- robots
  const int want_r = cfg.num_robots < R ? cfg.num_robots : R;
  int nr = 0;
  for (int base = 0; nr < want_r && base < kDraws; base += kWave) {
    const int c = base + lane;
    double u0, u1, u2, u3;
    g.u2(0, c, 0, u0, u1);
    g.u2(0, c, 1, u2, u3);
    const double sxv = 2.0 + (cfg.width - 4.0) * (1.0 - u0);
    const double syv = 2.0 + (cfg.height - 4.0) * (1.0 - u1);
    const double gxv = 2.0 + (cfg.width - 4.0) * (1.0 - u2);
    const double gyv = 2.0 + (cfg.height - 4.0) * (1.0 - u3);
    bool ok = c < kDraws && far_enough(gxv, gyv, sxv, syv, cfg.min_start_goal_dis, false);  // env.py:361
    for (int k = 0; k < nr && ok; ++k)
      ok = far_enough(srob[0][k], srob[1][k], sxv, syv, cfg.clear_r, true) &&
           far_enough(srob[2][k], srob[3][k], gxv, gyv, cfg.clear_r, true);
    while (nr < want_r) {
      const uint64_t bal = __ballot(ok);
      if (bal == 0) break;
      const int f = __builtin_amdgcn_readfirstlane(__ffsll(static_cast<unsigned long long>(bal)) - 1);
      const double fx = bcast(sxv, f), fy = bcast(syv, f), fgx = bcast(gxv, f), fgy = bcast(gyv, f);
      if (lane == f) {
        srob[0][nr] = sxv;
        srob[1][nr] = syv;
        srob[2][nr] = gxv;
        srob[3][nr] = gyv;
        const size_t id = static_cast<size_t>(e) * R + nr;
        rs[ASVRL_F_X * NT + id] = sxv;  // reset_robot / reset_state (env.py:166-176, wamv.py:177-193)
        rs[ASVRL_F_Y * NT + id] = syv;
        rs[ASVRL_F_GX * NT + id] = gxv;
        rs[ASVRL_F_GY * NT + id] = gyv;
        rs[ASVRL_F_THETA * NT + id] = kTwoPi * (1.0 - g.u(0, c, 4));
        for (int fld = ASVRL_F_VR0; fld <= ASVRL_F_RP; ++fld) rs[fld * NT + id] = 0.0;
        rs[ASVRL_F_PHI * NT + id] = 0.0;
        rs[ASVRL_F_RET * NT + id] = 0.0;
        s.rflags[id] = 0;
      }
      ok = ok && lane > f && far_enough(fx, fy, sxv, syv, cfg.clear_r, true) &&
           far_enough(fgx, fgy, gxv, gyv, cfg.clear_r, true);
      ++nr;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");   // the batch's LDS rows before the next batch's reads
    __builtin_amdgcn_wave_barrier();
  }
  for (int k = nr + lane; k < R; k += kWave) s.rflags[static_cast<size_t>(e) * R + k] = ASVRL_FLAG_DEACTIVATED;

  // ---- vortex cores (env.py:123-136, check_core :378-418)
  double* cores = s.cores + static_cast<size_t>(e) * Cmax * 4;
  const int want_c = cfg.num_cores < Cmax ? cfg.num_cores : Cmax;
  int nc = 0;
  for (int base = 0; nc < want_c && base < kDraws; base += kWave) {
    const int c = base + lane;
    double u0, u1, u2, u3;
    g.u2(1, c, 0, u0, u1);
    g.u2(1, c, 1, u2, u3);
    const double cx = cfg.width * (1.0 - u0);
    const double cy = cfg.height * (1.0 - u1);
    const double cw = u2 <= 0.5 ? 1.0 : 0.0;
    const double ve = cfg.v_lo + (cfg.v_hi - cfg.v_lo) * (1.0 - u3);
    const double Gamma = 2 * kPi * p.core_r * ve;
    bool ok = c < kDraws && !(cx - p.core_r < 0.0 || cx + p.core_r > cfg.width) &&
              !(cy - p.core_r < 0.0 || cy + p.core_r > cfg.width);  // (sic) env.py:383
    for (int k = 0; k < nr && ok; ++k)
      ok = far_enough(cx, cy, srob[0][k], srob[1][k], p.core_r + cfg.clear_r, false) &&
           far_enough(cx, cy, srob[2][k], srob[3][k], p.core_r + cfg.clear_r, false);
    for (int k = 0; k < nc && ok; ++k)
      ok = !core_conflict(cfg, p.core_r, score[k][0], score[k][1], score[k][2], score[k][3], cx, cy,
                          cw, Gamma);
    while (nc < want_c) {
      const uint64_t bal = __ballot(ok);
      if (bal == 0) break;
      const int f = __builtin_amdgcn_readfirstlane(__ffsll(static_cast<unsigned long long>(bal)) - 1);
      const double fx = bcast(cx, f), fy = bcast(cy, f), fw = bcast(cw, f), fG = bcast(Gamma, f);
      if (lane == f) {
        score[nc][0] = cores[4 * nc] = cx;
        score[nc][1] = cores[4 * nc + 1] = cy;
        score[nc][2] = cores[4 * nc + 2] = cw;
        score[nc][3] = cores[4 * nc + 3] = Gamma;
      }
      ok = ok && lane > f && !core_conflict(cfg, p.core_r, fx, fy, fw, fG, cx, cy, cw, Gamma);
      ++nc;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
  }

  // ---- static obstacles (env.py:151-162, check_obstacle :420-456)
  double* obs = s.obstacles + static_cast<size_t>(e) * O * 3;
  const int want_o = cfg.num_obs < O ? cfg.num_obs : O;
  int no = 0;
  for (int base = 0; no < want_o && base < kDraws; base += kWave) {
    const int c = base + lane;
    double u0, u1, u2, u3;
    g.u2(2, c, 0, u0, u1);
    g.u2(2, c, 1, u2, u3);
    const double ox = 5.0 + (cfg.width - 10.0) * (1.0 - u0);
    const double oy = 5.0 + (cfg.height - 10.0) * (1.0 - u1);
    const double orad = cfg.obs_r_lo + (cfg.obs_r_hi - cfg.obs_r_lo) * (1.0 - u2);
    bool ok = c < kDraws && !(ox - orad < 0.0 || ox + orad > cfg.width) && !(oy - orad < 0.0 || oy + orad > cfg.height);
    for (int k = 0; k < nr && ok; ++k)
      ok = far_enough(ox, oy, srob[0][k], srob[1][k], orad + cfg.clear_r, false) &&
           far_enough(ox, oy, srob[2][k], srob[3][k], orad + cfg.clear_r, false);
    for (int k = 0; k < nc && ok; ++k) ok = far_enough(score[k][0], score[k][1], ox, oy, p.core_r + orad, true);
    for (int k = 0; k < no && ok; ++k) ok = far_enough(sobs[k][0], sobs[k][1], ox, oy, sobs[k][2] + orad, true);
    while (no < want_o) {
      const uint64_t bal = __ballot(ok);
      if (bal == 0) break;
      const int f = __builtin_amdgcn_readfirstlane(__ffsll(static_cast<unsigned long long>(bal)) - 1);
      const double fx = bcast(ox, f), fy = bcast(oy, f), fr = bcast(orad, f);
      if (lane == f) {
        sobs[no][0] = obs[3 * no] = ox;
        sobs[no][1] = obs[3 * no + 1] = oy;
        sobs[no][2] = obs[3 * no + 2] = orad;
      }
      ok = ok && lane > f && far_enough(fx, fy, ox, oy, fr + orad, true);
      ++no;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
  }
  if (lane == 0) {
    s.n_robots[e] = nr;
    s.n_cores[e] = nc;
    s.n_obs[e] = no;
    s.ep_ts[e] = 0;
  }
}

__global__ __launch_bounds__(kResetWaves * kWave) void env_reset_kernel(AsvParams p, AsvEnvState s, AsvResetCfg cfg,
                                                                        const uint8_t* __restrict__ mask,
                                                                        uint64_t seed, uint64_t counter,
                                                                        const uint64_t* __restrict__ counter_dev) {
  __shared__ ResetLds W[kResetWaves];
  const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
  const int e = blockIdx.x * kResetWaves + wv;
  if (e >= s.n_envs) return;                     // wave-uniform exits
  if (mask != nullptr && mask[e] == 0) return;
  reset_env(p, s, cfg, e, seed, counter + (counter_dev != nullptr ? *counter_dev : 0ull), lane, W[wv]);
}

// The training loop's auto-reset in ONE launch (asvrl_env_reset_observe): workgroup e is one wave; if env e
// ended its episode (mask), the wave resets it (reset_env) and then computes its reset observation with the
// step kernel's own phases (env_pairs_block, one env per workgroup, do_dynamics = 0): the same values as
// asvrl_env_reset followed by the masked asvrl_env_step pass, without the second launch over every env.
struct ResetObsArgs {
  PairsArgs k;   // actions / noise null, epb 1
  AsvResetCfg cfg;
  const uint8_t* mask;
  uint64_t seed, counter;
  const uint64_t* counter_dev;
};
template <int NM>
__global__ __launch_bounds__(kWave) void env_reset_observe_kernel(ResetObsArgs) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];   // env_pairs_block's carve
  __shared__ ResetLds W;
  const KArg<ResetObsArgs> RA = kargs<ResetObsArgs>();
  const ResetObsArgs& a = kref(RA);
  const int e = blockIdx.x;
  if (a.mask[e] == 0) return;                      // workgroup-uniform
  reset_env(a.k.p, a.k.s, a.cfg, e, a.seed, a.counter + (a.counter_dev != nullptr ? *a.counter_dev : 0ull),
            threadIdx.x, W);
  __syncthreads();   // the reset's global writes (workgroup-scope release / acquire) before the observation reads
  env_pairs_block<kWave, NM, false>(kfresh<PairsArgs>(&RA->k), 1, e, smem);
}

__global__ __launch_bounds__(kBlock) void current_kernel(const double* __restrict__ cores, int nc, double core_r,
                                                        const double* __restrict__ xy, int n, double* __restrict__ out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  double cx, cy;
  current_at(cores, nc, core_r, xy[2 * k], xy[2 * k + 1], cx, cy);
  out[3 * k] = cx;
  out[3 * k + 1] = cy;
  out[3 * k + 2] = 0.0;
}

}  // namespace

size_t env_sweep_smem(int R, int O) {
  const int blk = step_block(R);
  const int epb = blk / R;
  return sizeof(double) * (4 * blk + static_cast<size_t>(epb) * O * 3) + sizeof(int) * epb + blk;
}

// the pair-parallel launch: workgroup size from the pair count, envs per workgroup so that the
// pairs fill it (at least one env); AsvEnvLaunch may set the block and the envs per workgroup
struct PairLaunch {
  int blk, epb;
  size_t smem;
};
PairLaunch pair_launch(int R, int O, int n_envs, int blk_req, int epb_req, int vm_bytes) {
  const int np1 = R * (O + R);
  PairLaunch L;
  // Launch-shape rule (tools/env_try.sh, profiles/r02_env_pairs_v2_sweep*.jsonl; the kernel holds 4
  // waves per SIMD by registers, so the shape sets LDS use, tail waste and per-workgroup overheads):
  //  - up to 8 robots per env, below 16384 envs: 256-lane workgroups of about 40 robots (R = 5: 8 envs,
  //    27 us at 4096 envs vs 31-42 us for the other shapes)
  //  - up to 8 robots, from 16384 envs: one-wave workgroups of about 40 robots (R = 5: 8 envs; 416-422 us
  //    at 2^18 envs vs 428-440 us for 128/256 lanes)
  //  - more robots: 256-lane workgroups of about 120 robots (R = 17: 7 envs, 61 us at 4096 envs vs 70 us
  //    for 3 envs and 74-124 us for the other shapes)
  const bool large = n_envs >= 16384 && R <= 8;
  L.blk = (blk_req == 64 || blk_req == 128 || blk_req == 256) ? blk_req : (large ? 64 : 256);
  if (R > L.blk) L.blk = 256;
  if (R <= 8)
    L.epb = large ? 40 / R : ((40 + R - 1) / R < 64 / R ? (40 + R - 1) / R : 64 / R);
  else
    L.epb = 120 / R > 1 ? 120 / R : 1;
  if (epb_req > 0) L.epb = epb_req;
  if (L.epb * R > L.blk) L.epb = L.blk / R;
  // env_pairs_kernel's carve: 8 per-robot f64 arrays, the per-pair keys (reused as phase 4's phi),
  // obstacles, the per-pair radius draws (f32 for noise mode 2), 3 ints per env and one per wave, 5 kept
  // slots and 5 work-list entries (u16) per robot, then bytes (pair / COLREGs flags, 2 per-robot flags,
  // kept count)
  const size_t nrb = static_cast<size_t>(L.epb) * R;
  const size_t np = static_cast<size_t>(L.epb) * np1;
  const size_t nslot = np > 5 * nrb ? np : 5 * nrb;
  L.smem = sizeof(double) * (8 * nrb + nslot + static_cast<size_t>(L.epb) * O * 3) + vm_bytes * np +
           sizeof(int) * (3 * L.epb + L.blk / 64) + sizeof(unsigned short) * 10 * nrb + nslot + 3 * nrb;
  return L;
}

}  // namespace asvrl

using namespace asvrl;

extern "C" int asvrl_env_step_ex(const AsvParams* params, const AsvEnvState* state, const double* actions,
                                 const double* noise, const AsvStepCtl* ctl, const AsvStepOut* out,
                                 const AsvEnvLaunch* launch, void* stream) {
  ASVRL_REQUIRE(params && state && ctl && out, "asvrl_env_step: null argument");
  ASVRL_REQUIRE(state->max_robots >= 1 && state->max_robots <= kBlock, "asvrl_env_step: max_robots must be in [1, 256]");
  ASVRL_REQUIRE(state->max_obs >= 0 && state->max_cores >= 0 && state->max_cores <= kMaxCoresStep,
                "asvrl_env_step: bad max_obs/max_cores");
  ASVRL_REQUIRE(params->max_obj_num >= 0 && params->max_obj_num <= ASVRL_MAX_OBJ, "asvrl_env_step: max_obj_num > 5");
  ASVRL_REQUIRE(params->N >= 1, "asvrl_env_step: N < 1");
  ASVRL_REQUIRE(out->obs && out->obj_cnt && out->reward && out->done && out->info, "asvrl_env_step: null output");
  ASVRL_REQUIRE(ctl->noise_mode != 0 || noise != nullptr, "asvrl_env_step: noise_mode 0 needs injected noise");
  ASVRL_REQUIRE(!ctl->do_dynamics || actions != nullptr, "asvrl_env_step: actions required");
  ASVRL_REQUIRE(state->rs && state->rflags && state->n_robots && state->n_obs && state->n_cores && state->ep_ts,
                "asvrl_env_step: null state array");
  if (state->n_envs == 0) return 0;
  const AsvEnvLaunch lz{};
  const AsvEnvLaunch& lc = launch != nullptr ? *launch : lz;
  ASVRL_REQUIRE(lc.layout >= 0 && lc.layout <= 2, "asvrl_env_step: layout must be 0 (auto), 1 (pairs) or 2 (sweep)");
  ASVRL_REQUIRE(lc.block == 0 || lc.block == 64 || lc.block == 128 || lc.block == 256,
                "asvrl_env_step: block must be 0, 64, 128 or 256");
  ASVRL_REQUIRE(lc.envs_per_block >= 0 && lc.max_groups >= 0, "asvrl_env_step: negative envs_per_block / max_groups");
  const int nm = ctl->noise_mode == 0 ? 0 : (ctl->noise_mode == 1 ? 1 : 2);
  const PairLaunch pl = pair_launch(state->max_robots, state->max_obs, state->n_envs, lc.block, lc.envs_per_block,
                                    nm == 2 ? 4 : 8);
  const bool per_robot = state->robot_params != nullptr;
  ASVRL_REQUIRE(lc.layout != 1 || pl.smem <= 150 * 1024, "asvrl_env_step: the pair layout's LDS does not fit");
  ASVRL_REQUIRE(lc.layout != 1 || !per_robot, "asvrl_env_step: per-robot parameters take the sweep layout (2)");
  if (lc.layout != 2 && !per_robot && pl.smem <= 150 * 1024) {
    const int groups = (state->n_envs + pl.epb - 1) / pl.epb;
    const int chunk = lc.max_groups > 0 && lc.max_groups < groups ? lc.max_groups : groups;
    auto go = [&](auto kern) {
      PairsArgs a{*params, *state, *ctl, *out, actions, noise, pl.epb, 0};
      for (int g0 = 0; g0 < groups; g0 += chunk) {
        a.group0 = g0;
        hipLaunchKernelGGL(kern, dim3(groups - g0 < chunk ? groups - g0 : chunk), dim3(pl.blk), pl.smem,
                           as_stream(stream), a);
      }
    };
    if (pl.blk == 64)
      nm == 0 ? go(env_pairs_kernel<64, 0>) : nm == 1 ? go(env_pairs_kernel<64, 1>) : go(env_pairs_kernel<64, 2>);
    else if (pl.blk == 128)
      nm == 0 ? go(env_pairs_kernel<128, 0>) : nm == 1 ? go(env_pairs_kernel<128, 1>) : go(env_pairs_kernel<128, 2>);
    else
      nm == 0 ? go(env_pairs_kernel<256, 0>) : nm == 1 ? go(env_pairs_kernel<256, 1>) : go(env_pairs_kernel<256, 2>);
    return check_launch("asvrl_env_step");
  }
  const int blk = step_block(state->max_robots);
  const int epb = blk / state->max_robots;
  const int grid = (state->n_envs + epb - 1) / epb;
  const size_t smem = env_sweep_smem(state->max_robots, state->max_obs);
  ASVRL_REQUIRE(smem <= 160 * 1024, "asvrl_env_step: max_obs too large for LDS");
  auto sweep = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(blk), smem, as_stream(stream), *params, *state, actions, noise, *ctl,
                       *out);
  };
  if (blk == 64)
    per_robot ? sweep(env_sweep_kernel<64, true>) : sweep(env_sweep_kernel<64, false>);
  else
    per_robot ? sweep(env_sweep_kernel<256, true>) : sweep(env_sweep_kernel<256, false>);
  return check_launch("asvrl_env_step");
}

extern "C" int asvrl_env_step(const AsvParams* params, const AsvEnvState* state, const double* actions,
                              const double* noise, const AsvStepCtl* ctl, const AsvStepOut* out, void* stream) {
  return asvrl_env_step_ex(params, state, actions, noise, ctl, out, nullptr, stream);
}

extern "C" int asvrl_env_reset(const AsvParams* params, const AsvEnvState* state, const AsvResetCfg* cfg,
                               const uint8_t* env_mask, uint64_t seed, uint64_t counter,
                               const uint64_t* counter_dev, void* stream) {
  ASVRL_REQUIRE(params && state && cfg, "asvrl_env_reset: null argument");
  ASVRL_REQUIRE(state->max_cores <= kMaxCores, "asvrl_env_reset: max_cores > 16");
  ASVRL_REQUIRE(state->max_robots <= kResetMaxR && state->max_obs <= kResetMaxO,
                "asvrl_env_reset: max_robots and max_obs must be <= 32");
  ASVRL_REQUIRE(cfg->width > 4.0 && cfg->height > 4.0, "asvrl_env_reset: map too small");
  if (state->n_envs == 0) return 0;
  const int grid = (state->n_envs + kResetWaves - 1) / kResetWaves;
  hipLaunchKernelGGL(env_reset_kernel, dim3(grid), dim3(kResetWaves * kWave), 0, as_stream(stream), *params, *state,
                     *cfg, env_mask, seed, counter, counter_dev);
  return check_launch("asvrl_env_reset");
}

extern "C" int asvrl_env_reset_observe(const AsvParams* params, const AsvEnvState* state, const AsvResetCfg* cfg,
                                       const uint8_t* env_mask, uint64_t seed, uint64_t counter,
                                       const uint64_t* counter_dev, const AsvStepCtl* ctl, const AsvStepOut* out,
                                       void* stream) {
  ASVRL_REQUIRE(params && state && cfg && ctl && out && env_mask, "asvrl_env_reset_observe: null argument");
  ASVRL_REQUIRE(state->max_cores <= kMaxCores, "asvrl_env_reset_observe: max_cores > 16");
  ASVRL_REQUIRE(state->max_robots <= kResetMaxR && state->max_obs <= kResetMaxO,
                "asvrl_env_reset_observe: max_robots and max_obs must be <= 32");
  ASVRL_REQUIRE(cfg->width > 4.0 && cfg->height > 4.0, "asvrl_env_reset_observe: map too small");
  ASVRL_REQUIRE(state->robot_params == nullptr, "asvrl_env_reset_observe: per-robot parameters take the two-launch path");
  ASVRL_REQUIRE(!ctl->do_dynamics && ctl->env_mask == env_mask, "asvrl_env_reset_observe: ctl must be the masked "
                "observation pass (do_dynamics = 0, env_mask = the reset mask)");
  ASVRL_REQUIRE(ctl->noise_mode == 1 || ctl->noise_mode == 2, "asvrl_env_reset_observe: Philox noise only (mode 1 or 2)");
  ASVRL_REQUIRE(out->obs && out->obj_cnt && out->reward && out->done && out->info,
                "asvrl_env_reset_observe: null output");
  if (state->n_envs == 0) return 0;
  const PairLaunch pl = pair_launch(state->max_robots, state->max_obs, state->n_envs, kWave, 1,
                                    ctl->noise_mode == 2 ? 4 : 8);
  ASVRL_REQUIRE(pl.blk == kWave && pl.epb == 1 && pl.smem <= 60 * 1024, "asvrl_env_reset_observe: env too large");
  auto go = [&](auto kern) {
    const ResetObsArgs a{PairsArgs{*params, *state, *ctl, *out, nullptr, nullptr, 1, 0}, *cfg, env_mask, seed, counter,
                         counter_dev};
    hipLaunchKernelGGL(kern, dim3(state->n_envs), dim3(kWave), pl.smem, as_stream(stream), a);
  };
  ctl->noise_mode == 2 ? go(env_reset_observe_kernel<2>) : go(env_reset_observe_kernel<1>);
  return check_launch("asvrl_env_reset_observe");
}

extern "C" int asvrl_current_field(const double* cores, int32_t n_cores, double core_r, const double* xy,
                                   int32_t n, double* out, void* stream) {
  ASVRL_REQUIRE(xy && out && (n_cores == 0 || cores), "asvrl_current_field: null argument");
  ASVRL_REQUIRE(n_cores >= 0 && n_cores <= kMaxCoresStep, "asvrl_current_field: n_cores > 4096");
  if (n <= 0) return 0;
  hipLaunchKernelGGL(current_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, as_stream(stream), cores,
                     n_cores, core_r, xy, n, out);
  return check_launch("asvrl_current_field");
}
