#!/usr/bin/env python3
"""Capture golden vectors from the reference rfarl package (test infrastructure).

Runs ONLY in the build container, where the read-only reference is mounted at
/root/reference. It imports the reference's own Python code and writes small
.npz fixtures under tests/golden/. Nothing in the product, the GPU tests,
smoke() or bench.py reads /root/reference; they read these fixtures.

    PYTHONDONTWRITEBYTECODE=1 python3 -W ignore tools/capture_oracle.py

Fixture families:
  env_dynamics.npz  F1  Robot.update_state x N substeps on random states
                        (rfarl/rfarl/envs/marinenav/vehicles/wamv.py:204-279,
                         env.py:257-260 loop, env.py:458-501 current field)
  env_traces.npz    F2/F3  MarineNavEnv3.step traces with every perception noise
                        draw recorded (env.py:240-333, wamv.py:436-529)
  env_evalcfg.npz   F2c reset_with_eval_config with per-robot vehicle / perception parameters, and a
                        20-core scene (env.py:503-614)
  env_reset.npz     F7  MarineNavEnv3.reset rejection sampler (env.py:72-164)
  learn_ac_iqn.npz  F4  Agent.train_AC_IQN (agent.py:386-432), N=8 and N=32
  learn_iqn.npz     F5  Agent.train_IQN (agent.py:434-476)
  learn_rainbow.npz F6  Agent.train_Rainbow incl. the C51 projection target m
                        (agent.py:597-641)
  learn_rainbow_full.npz F6b  the same at the default network size (the size the kernels take),
                        networks from a numpy-seeded generator (oracle/learn_ref.py)
  learn_dqn.npz     F8  Agent.train_DQN / act_dqn (agent.py:518-545, 271-287)
  eval_ref.npz      F9  Trainer.evaluation (trainer.py:266-392), AC-IQN and Rainbow
  eval_iqn_ref.npz  F9b the same for IQN with every act_iqn call's K = 32 taus recorded (capture_eval_iqn)
  eval60_ref.npz    F10 Trainer.evaluation on config/ac_iqn.json's 60-episode eval_schedule, the seeded
                        AC-IQN agent and the same agent after 200 train_AC_IQN steps (capture_eval60)
  eval60_tf.npz     F10b the same two evaluations re-run from F10's own configs and actor weights, with every
                        robot's per-step action and its perception-noise draws (count and checksums) recorded,
                        for the teacher-forced env replay (capture_eval60_tf)
"""
import os
import sys
import types

import numpy as np

REF = "/root/reference/rfarl"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")

sys.path.insert(0, REF)
sys.dont_write_bytecode = True

import torch  # noqa: E402
import rfarl.agent as ref_agent_mod  # noqa: E402
from rfarl.envs.marinenav.env import MarineNavEnv3, Core, Obstacle  # noqa: E402
import rfarl.envs.marinenav.vehicles.wamv as wamv  # noqa: E402
from rfarl.policy.AC_IQN_model import Critic  # noqa: E402
from rfarl.policy.IQN_model import IQN_Policy  # noqa: E402
import scipy.spatial  # noqa: E402

STATE_FIELDS = ["x", "y", "theta", "vr0", "vr1", "vr2", "v0", "v1", "v2",
                "TL", "TR", "lp", "rp"]
INFO_CODES = {"normal": 0, "too long episode": 1, "collision": 2, "reach goal": 3,
              "deactivated after collision": 4, "deactivated after reaching goal": 5}


# ----------------------------------------------------------------------------------
# helpers
# ----------------------------------------------------------------------------------
class RecRD:
    """Proxy over a robot's Perception.rd that records every draw in order."""

    def __init__(self, rd):
        self.rd = rd
        self.log = []

    def normal(self, loc, scale):
        v = self.rd.normal(loc, scale)
        self.log.append(float(v))
        return v

    def vonmises(self, mu, kappa):
        v = self.rd.vonmises(mu, kappa)
        self.log.append(float(v))
        return v


def robot_state(r):
    return [float(r.x), float(r.y), float(r.theta),
            float(r.velocity_r[0]), float(r.velocity_r[1]), float(r.velocity_r[2]),
            float(r.velocity[0]), float(r.velocity[1]), float(r.velocity[2]),
            float(r.left_thrust), float(r.right_thrust),
            float(r.left_pos), float(r.right_pos)]


def set_robot_state(r, s):
    r.x, r.y, r.theta = float(s[0]), float(s[1]), float(s[2])
    r.velocity_r = np.array(s[3:6], dtype=np.float64)
    r.velocity = np.array(s[6:9], dtype=np.float64)
    r.left_thrust, r.right_thrust = float(s[9]), float(s[10])
    r.left_pos, r.right_pos = float(s[11]), float(s[12])


def install_recorders(env):
    for rob in env.robots:
        if not isinstance(rob.perception.rd, RecRD):
            rob.perception.rd = RecRD(rob.perception.rd)


def clear_recorders(env):
    for rob in env.robots:
        rob.perception.rd.log = []


def noise_slots(env, deact_before, R, O):
    """Map each robot's recorded draws into per-candidate slots.

    Slot k < O is obstacle k; slot O + j is other robot j. Each slot holds the 5 draws
    [n_px, n_py, n_vx, n_vy, vonmises] in the order wamv.py:466-468,493-495 makes them.
    Unused slots are NaN.
    """
    slots = np.full((R, O + R, 5), np.nan)
    n = len(env.robots)
    for i, rob in enumerate(env.robots):
        if deact_before[i]:
            assert len(rob.perception.rd.log) == 0
            continue
        log = rob.perception.rd.log
        k = 0
        for o in range(len(env.obstacles)):
            slots[i, o] = log[k:k + 5]
            k += 5
        for j in range(n):
            if j == i or deact_before[j]:
                continue
            slots[i, O + j] = log[k:k + 5]
            k += 5
        assert k == len(log), (k, len(log))
    return slots


def pack_obs(obs, R):
    self_obs = np.zeros((R, 7))
    objs = np.zeros((R, 5, 5))
    cnt = np.zeros(R, np.int32)
    valid = np.zeros(R, np.uint8)
    for i, (s, o) in enumerate(obs):
        if s is None:
            continue
        valid[i] = 1
        self_obs[i] = np.array(s, dtype=np.float64)
        cnt[i] = len(o)
        for k, ob in enumerate(o):
            objs[i, k] = np.array(ob, dtype=np.float64)
    return self_obs, objs, cnt, valid


# ----------------------------------------------------------------------------------
# F2/F3: env.step traces
# ----------------------------------------------------------------------------------
def run_trace(env, n_steps, action_fn, continuous, R, O, ep_ts_override=None,
              post_reset=None, reset=None):
    """Reset (env.reset(), or `reset(env)`) + run n_steps of env.step the way Trainer.learn drives it
    (trainer.py:110-172: None actions for deactivated robots, deactivate on flags)."""
    if reset is None:
        env.reset()
    else:
        reset(env)
    if post_reset is not None:
        post_reset(env)
    # re-observe so recorded observation matches a post_reset edit is not needed; the
    # trace starts from the state after reset/post_reset.
    install_recorders(env)
    if ep_ts_override is not None:
        env.episode_timesteps = ep_ts_override
    n = len(env.robots)
    rec = {k: [] for k in ["state_before", "state_after", "deact_before", "actions", "noise",
                           "self_obs", "obj_obs", "obj_cnt", "obs_valid", "collision", "reach",
                           "apply_colregs", "phi", "reward", "done", "info", "ep_ts",
                           "ep_return", "deact_after", "end_episode"]}
    # Trainer.learn's per-episode bookkeeping (trainer.py:96-98,157-172), GAMMA = Agent.GAMMA
    # default (agent.py:23). ep_length is the env's episode_timesteps before the step (equal to the
    # trainer's counter from a reset; the timeout trace starts it at ep_ts_override)
    GAMMA = 0.99
    ep_rewards = np.zeros(R)
    static = dict(
        obstacles=np.array([[o.x, o.y, o.r] for o in env.obstacles] + [[0, 0, 0]] * (O - len(env.obstacles)), dtype=np.float64).reshape(O, 3),
        n_obs=len(env.obstacles),
        goals=np.array([list(r.goal) for r in env.robots] + [[0, 0]] * (R - n)),
        n_robots=n,
        cores=np.array([[c.x, c.y, float(c.clockwise), c.Gamma] for c in env.cores] + [[0, 0, 0, 0]] * max(0, 8 - len(env.cores))).reshape(max(8, len(env.cores)), 4),
        n_cores=len(env.cores),
        core_r=env.r,
        width=env.width, height=env.height,
    )
    for t in range(n_steps):
        if all(r.deactivated for r in env.robots):
            break
        if env.check_all_reach_goal():
            break
        deact = [bool(r.deactivated) for r in env.robots]
        sb = np.zeros((R, 13))
        for i, r in enumerate(env.robots):
            sb[i] = robot_state(r)
        acts = []
        act_arr = np.zeros((R, 2))
        for i, r in enumerate(env.robots):
            if r.deactivated:
                acts.append(None)
                continue
            a = action_fn(t, i)
            acts.append(a)
            if continuous:
                act_arr[i] = a
            else:
                act_arr[i, 0] = a
        ep_ts = env.episode_timesteps
        clear_recorders(env)
        obs, rew, done, info = env.step(acts, continuous)
        slots = noise_slots(env, deact, R, O)
        sa = np.zeros((R, 13))
        for i, r in enumerate(env.robots):
            sa[i] = robot_state(r)
        so, oo, oc, ov = pack_obs(obs, R)
        coll = np.zeros(R, np.uint8)
        reach = np.zeros(R, np.uint8)
        app = np.zeros(R, np.uint8)
        phi = np.full(R, np.nan)
        rw = np.zeros(R)
        dn = np.zeros(R, np.uint8)
        inf = np.zeros(R, np.uint8)
        for i, r in enumerate(env.robots):
            coll[i] = r.collision
            reach[i] = r.reach_goal
            if not deact[i]:
                app[i] = r.apply_COLREGs
                if r.apply_COLREGs:
                    phi[i] = r.phi
            rw[i] = rew[i]
            dn[i] = done[i]
            inf[i] = INFO_CODES[info[i]["state"]]
        db = np.zeros(R, np.uint8)
        db[:n] = deact
        for k, v in [("state_before", sb), ("state_after", sa), ("deact_before", db), ("actions", act_arr),
                     ("noise", slots), ("self_obs", so), ("obj_obs", oo), ("obj_cnt", oc), ("obs_valid", ov),
                     ("collision", coll), ("reach", reach), ("apply_colregs", app), ("phi", phi),
                     ("reward", rw), ("done", dn), ("info", inf), ("ep_ts", ep_ts)]:
            rec[k].append(v)
        # trainer.py:157-172: discounted return of every robot active this step, then the
        # deactivation on collision / goal, then the episode-end test
        ep_length = ep_ts
        for i, r in enumerate(env.robots):
            if r.deactivated:
                continue
            ep_rewards[i] += GAMMA ** ep_length * rew[i]
            if r.collision or r.reach_goal:
                r.deactivated = True
        end_episode = (ep_length >= 1000) or env.check_all_deactivated()
        da = np.zeros(R, np.uint8)
        da[:n] = [bool(r.deactivated) for r in env.robots]
        rec["ep_return"].append(ep_rewards.copy())
        rec["deact_after"].append(da)
        rec["end_episode"].append(np.uint8(end_episode))
    out = {k: np.array(v) for k, v in rec.items()}
    out.update({k: np.array(v) for k, v in static.items()})
    return out


def crowd_post_reset(seed, speed=2.0):
    """Pack robots into a small area with fast headings so collisions and COLREGs
    encounters happen inside a short trace. Only robot state is edited."""

    def f(env):
        rs = np.random.RandomState(1000 + seed)
        cx, cy = env.width / 2, env.height / 2
        for r in env.robots:
            r.x = float(cx + rs.uniform(-12, 12))
            r.y = float(cy + rs.uniform(-12, 12))
            r.theta = float(rs.uniform(0, 2 * np.pi))
            sp = rs.uniform(0.3, speed)
            vr = np.array([np.cos(r.theta) * sp, np.sin(r.theta) * sp, rs.uniform(-0.2, 0.2)])
            r.velocity_r = vr
            r.velocity = vr + np.array([rs.normal(0, 0.05), rs.normal(0, 0.05), 0.0])
            r.left_thrust = float(rs.uniform(0, 1000))
            r.right_thrust = float(rs.uniform(0, 1000))
        # move obstacles into the crowd too
        for o in env.obstacles:
            o.x = float(cx + rs.uniform(-10, 10))
            o.y = float(cy + rs.uniform(-10, 10))
    return f


def goal_post_reset(seed):
    """Start every robot 2-6 m from its goal, pointed at it, so reach-goal (+10) fires."""

    def f(env):
        rs = np.random.RandomState(2000 + seed)
        for r in env.robots:
            ang = rs.uniform(0, 2 * np.pi)
            d = rs.uniform(2.0, 6.0)
            r.x = float(r.goal[0] - d * np.cos(ang))
            r.y = float(r.goal[1] - d * np.sin(ang))
            r.theta = float(ang)
            sp = rs.uniform(0.5, 2.0)
            vr = np.array([np.cos(ang) * sp, np.sin(ang) * sp, 0.0])
            r.velocity_r = vr
            r.velocity = vr.copy()
            r.left_thrust = r.right_thrust = 300.0
    return f


def capture_traces():
    traces = {}

    def cont_fn(seed):
        rs = np.random.RandomState(77 + seed)
        return lambda t, i: [float(rs.uniform(-1, 1)), float(rs.uniform(-1, 1))]

    def fwd_fn(seed):
        rs = np.random.RandomState(99 + seed)
        return lambda t, i: [float(rs.uniform(0.2, 1.0)), float(rs.uniform(0.2, 1.0))]

    def disc_fn(seed):
        rs = np.random.RandomState(55 + seed)
        return lambda t, i: int(rs.randint(0, 25))

    def env_for(seed, R, O, msgd, width=55, cores=0):
        e = MarineNavEnv3(seed=seed)
        e.num_robots, e.num_cores, e.num_obs, e.min_start_goal_dis = R, cores, O, msgd
        e.width = e.height = width
        return e

    # T0-T1: config-2 scene (R=5, O=4), continuous random actions
    for s in (0, 1):
        traces[f"cont_r5o4_s{s}"] = (run_trace(env_for(s, 5, 4, 40.0), 120, cont_fn(s), True, 5, 4), 5, 4)
    # T2: discrete actions (IQN / Rainbow action grid, wamv.py:86-88,146-147)
    traces["disc_r5o4_s2"] = (run_trace(env_for(2, 5, 4, 40.0), 120, disc_fn(2), False, 5, 4), 5, 4)
    # T3: crowded scene -> collisions + COLREGs
    for s in (3, 4, 5):
        traces[f"crowd_r8o4_s{s}"] = (run_trace(env_for(s, 8, 4, 30.0, width=80), 150, fwd_fn(s), True, 8, 4,
                                                post_reset=crowd_post_reset(s)), 8, 4)
    # T4: big scene, 12 robots on a 110 m map
    traces["cont_r12o8_s6"] = (run_trace(env_for(6, 12, 8, 40.0, width=110), 60, cont_fn(6), True, 12, 8), 12, 8)
    # T5: timeout branch (env.py:312-315, checked before collision)
    traces["timeout_r5o4_s7"] = (run_trace(env_for(7, 5, 4, 40.0), 4, cont_fn(7), True, 5, 4,
                                           ep_ts_override=998, post_reset=crowd_post_reset(7, 3.0)), 5, 4)
    # T7: goal reaching (+10, deactivated-after-goal info, env.py:321-325)
    traces["goal_r5o4_s9"] = (run_trace(env_for(9, 5, 4, 40.0), 40, fwd_fn(9), True, 5, 4,
                                        post_reset=goal_post_reset(9)), 5, 4)
    # T6: vortex current field on (env.py:458-501), 4 cores
    traces["cores_r5o4_s8"] = (run_trace(env_for(8, 5, 4, 30.0, cores=4), 60, cont_fn(8), True, 5, 4), 5, 4)
    out = {}
    for name, (tr, R, O) in traces.items():
        for k, v in tr.items():
            out[f"{name}/{k}"] = v
        out[f"{name}/R"] = np.int32(R)
        out[f"{name}/O"] = np.int32(O)
        print(f"trace {name}: steps={len(tr['reward'])} robots={tr['n_robots']} "
              f"collisions={int(tr['collision'].sum())} reach={int(tr['reach'].sum())} "
              f"colregs={int(tr['apply_colregs'].sum())} timeouts={int((tr['info'] == 1).sum())}")
    out["names"] = np.array(list(traces.keys()))
    np.savez_compressed(os.path.join(OUT, "env_traces.npz"), **out)


# ----------------------------------------------------------------------------------
# F1: dynamics on random states
# ----------------------------------------------------------------------------------
def capture_dynamics():
    rs = np.random.RandomState(2024)
    n = 384
    out = {}
    # env with 4 vortex cores for the current-field case
    env = MarineNavEnv3(seed=11)
    env.cores.clear()
    cores = []
    for k in range(4):
        cx, cy = rs.uniform(5, 50, size=2)
        cw = bool(rs.randint(0, 2))
        Gamma = 2 * np.pi * env.r * rs.uniform(1, 3)
        env.cores.append(Core(cx, cy, cw, Gamma))
        cores.append([cx, cy, float(cw), Gamma])
    env.core_centers = scipy.spatial.KDTree(np.array([[c.x, c.y] for c in env.cores]))
    out["cores"] = np.array(cores)
    out["core_r"] = np.float64(env.r)
    env_nocore = MarineNavEnv3(seed=12)
    env_nocore.cores.clear()
    for case, (e, continuous) in {"cont": (env_nocore, True), "disc": (env_nocore, False),
                                  "cont_cores": (env, True)}.items():
        sb = np.zeros((n, 13))
        sa = np.zeros((n, 13))
        acts = np.zeros((n, 2))
        for k in range(n):
            rob = wamv.Robot(seed=k)
            x, y = rs.uniform(0, 55, size=2)
            th = rs.uniform(0, 2 * np.pi)
            if k % 16 == 0:
                th = 2 * np.pi - 1e-4
            if k % 16 == 1:
                th = 1e-4
            vr = np.array([rs.uniform(-3, 3), rs.uniform(-3, 3), rs.uniform(-1.5, 1.5)])
            if k % 16 == 0:
                vr[2] = 1.2
            if k % 16 == 1:
                vr[2] = -1.2
            v = vr + np.array([rs.normal(0, 0.1), rs.normal(0, 0.1), 0.0])
            TL, TR = rs.uniform(-500, 1000, size=2)
            if k % 8 == 2:
                TL, TR = 1000.0, -500.0
            s = [x, y, th, *vr, *v, TL, TR, 0.0, 0.0]
            set_robot_state(rob, s)
            if continuous:
                a = [float(rs.uniform(-1, 1)), float(rs.uniform(-1, 1))]
                if k % 8 == 3:
                    a = [1.0, -1.0]
                acts[k] = a
            else:
                a = int(rs.randint(0, 25))
                acts[k, 0] = a
            sb[k] = robot_state(rob)
            for idx in range(rob.N):  # env.py:257-260
                c = e.get_velocity(rob.x, rob.y)
                rob.update_state(a, c, idx == 0, continuous)
            sa[k] = robot_state(rob)
        out[f"{case}/state_before"] = sb
        out[f"{case}/state_after"] = sa
        out[f"{case}/actions"] = acts
    # current field samples (env.py:458-491)
    q = rs.uniform(0, 55, size=(256, 2))
    q[:4] = np.array([[c[0] + 0.2, c[1] - 0.1] for c in cores])  # inside core radius
    out["current_query"] = q
    out["current_value"] = np.array([env.get_velocity(float(a), float(b)) for a, b in q])
    # A = M_RB + M_A projection matrix inv(A^T A) A^T (wamv.py:267-271)
    r0 = wamv.Robot(0)
    A = r0.M_RB + r0.M_A
    out["P"] = np.array(np.linalg.inv(A.transpose() * A) * A.transpose())
    np.savez_compressed(os.path.join(OUT, "env_dynamics.npz"), **out)
    print("dynamics: ", {k: v.shape for k, v in out.items()})


# ----------------------------------------------------------------------------------
# F7: reset
# ----------------------------------------------------------------------------------
def capture_reset():
    out = {}
    schedule = {"timesteps": [0, 1000000, 2000000, 3000000, 4000000, 5000000],
                "num_robots": [3, 4, 5, 5, 5, 5], "num_cores": [0, 0, 0, 0, 0, 0],
                "num_obstacles": [0, 0, 0, 2, 3, 4], "min_start_goal_dis": [30.0, 35.0, 40.0, 40.0, 40.0, 40.0]}
    cases = []
    for seed in range(12):
        cases.append(("sched", seed, 0))
    for seed in range(4):
        cases.append(("sched", seed, 5_000_000))
    for seed in range(4):
        cases.append(("cores", seed, 0))
    for seed in range(3):
        cases.append(("r17", seed, 0))
    import contextlib
    import io
    for ci, (kind, seed, ts) in enumerate(cases):
        if kind == "sched":
            env = MarineNavEnv3(seed=seed, schedule=schedule)
            env.total_timesteps = ts
        elif kind == "cores":
            env = MarineNavEnv3(seed=seed)
            env.num_robots, env.num_cores, env.num_obs, env.min_start_goal_dis = 4, 4, 3, 30.0
        else:
            env = MarineNavEnv3(seed=seed)
            env.num_robots, env.num_cores, env.num_obs, env.min_start_goal_dis = 17, 0, 4, 40.0
            env.width = env.height = 110
        with contextlib.redirect_stdout(io.StringIO()):
            obs, coll, reach = env.reset()
        ep = env.episode_data()
        n = len(env.robots)
        p = f"c{ci}/"
        out[p + "kind"] = np.array(kind)
        out[p + "seed"] = np.int64(seed)
        out[p + "total_timesteps"] = np.int64(ts)
        out[p + "n_robots"] = np.int32(n)
        out[p + "start"] = np.array(ep["robots"]["start"]).reshape(n, 2)
        out[p + "goal"] = np.array(ep["robots"]["goal"]).reshape(n, 2)
        out[p + "init_theta"] = np.array(ep["robots"]["init_theta"])
        out[p + "perception_seed"] = np.array([r.perception.seed for r in env.robots])
        out[p + "obstacles"] = np.array([[o.x, o.y, o.r] for o in env.obstacles]).reshape(-1, 3)
        out[p + "cores"] = np.array([[c.x, c.y, float(c.clockwise), c.Gamma] for c in env.cores]).reshape(-1, 4)
        so, oo, oc, ov = pack_obs(obs, n)
        out[p + "self_obs"] = so
        out[p + "obj_obs"] = oo
        out[p + "obj_cnt"] = oc
        out[p + "rng_after"] = np.array(env.rd.get_state()[1][:8])  # RandomState key words after reset
        out[p + "rng_pos_after"] = np.int64(env.rd.get_state()[2])
    out["n_cases"] = np.int32(len(cases))
    np.savez_compressed(os.path.join(OUT, "env_reset.npz"), **out)
    print("reset cases:", len(cases))


# ----------------------------------------------------------------------------------
# learn fixtures
# ----------------------------------------------------------------------------------
def collect_transitions(n_needed, seed=0, discrete=False):
    """Transitions (s, a, r, s', d) from reference env rollouts, in the Trainer's format."""
    import contextlib
    import io
    env = MarineNavEnv3(seed=seed)
    env.num_robots, env.num_cores, env.num_obs, env.min_start_goal_dis = 5, 0, 4, 40.0
    rs = np.random.RandomState(seed + 5)
    trans = []
    with contextlib.redirect_stdout(io.StringIO()):
        states, _, _ = env.reset()
        steps = 0
        while len(trans) < n_needed:
            acts = []
            for i, r in enumerate(env.robots):
                if r.deactivated:
                    acts.append(None)
                elif discrete:
                    acts.append(int(rs.randint(0, 25)))
                else:
                    acts.append([float(rs.uniform(-1, 1)), float(rs.uniform(-1, 1))])
            nxt, rew, done, info = env.step(acts, not discrete)
            for i, r in enumerate(env.robots):
                if r.deactivated:
                    continue
                trans.append((states[i], acts[i], rew[i], nxt[i], done[i]))
                if r.collision or r.reach_goal:
                    r.deactivated = True
            steps += 1
            if steps >= 60 or env.check_all_deactivated():
                states, _, _ = env.reset()
                steps = 0
            else:
                states = nxt
    return trans


def make_batch(agent, trans, idx):
    samples = [trans[i] for i in idx]
    s = agent.memory.state_batch([t[0] for t in samples])
    ns = agent.memory.state_batch([t[3] for t in samples])
    a = [t[1] for t in samples]
    r = [t[2] for t in samples]
    d = [t[4] for t in samples]
    return s, a, r, ns, d


def batch_arrays(prefix, s, a, r, ns, d, B):
    out = {}
    for name, st in (("s", s), ("ns", ns)):
        out[prefix + name + "_self"] = np.array(st[0], dtype=np.float64).reshape(B, 7)
        if len(st[1]) == 0:
            out[prefix + name + "_obj"] = np.zeros((B, 5, 5))
            out[prefix + name + "_mask"] = np.zeros((B, 5))
        else:
            out[prefix + name + "_obj"] = np.array(st[1], dtype=np.float64)
            out[prefix + name + "_mask"] = np.array(st[2], dtype=np.float64)
    out[prefix + "a"] = np.array(a, dtype=np.float64)
    out[prefix + "r"] = np.array(r, dtype=np.float64)
    out[prefix + "d"] = np.array(d, dtype=np.float64)
    return out


def sd_arrays(prefix, module):
    return {prefix + k: v.detach().cpu().numpy().copy() for k, v in module.state_dict().items()}


class ClipRecorder:
    def __init__(self):
        self.norms = []
        self.orig = torch.nn.utils.clip_grad_norm_

    def __enter__(self):
        orig = self.orig
        rec = self

        def f(params, max_norm, *a, **k):
            n = orig(params, max_norm, *a, **k)
            rec.norms.append(float(n))
            return n
        torch.nn.utils.clip_grad_norm_ = f
        return self

    def __exit__(self, *a):
        torch.nn.utils.clip_grad_norm_ = self.orig


def capture_ac_iqn():
    out = {}
    trans = collect_transitions(600, seed=3)
    rs = np.random.RandomState(31)
    # N = 8: the reference's own train_AC_IQN
    agent = ref_agent_mod.Agent(device="cpu", seed=100, agent_type="AC-IQN")
    out.update(sd_arrays("init/actor/", agent.policy_local.actor))
    out.update(sd_arrays("init/critic/", agent.policy_local.critic))
    for k, v in agent.policy_target.critic.state_dict().items():
        assert torch.equal(v, agent.policy_local.critic.state_dict()[k])
    taus_rec = []
    orig_calc = Critic.calc_cos

    def rec_calc(self, batch_size, num_tau=8, cvar=1.0):
        cos, taus = orig_calc(self, batch_size, num_tau, cvar)
        taus_rec.append(taus.detach().numpy().copy())
        return cos, taus
    Critic.calc_cos = rec_calc
    try:
        for step in range(3):
            idx = rs.choice(len(trans), 64, replace=False)
            batch = make_batch(agent, trans, idx)
            out.update(batch_arrays(f"step{step}/", *batch, 64))
            agent.memory.sample = (lambda b=batch: b)
            taus_rec.clear()
            with ClipRecorder() as cr:
                closs, aloss = agent.train_AC_IQN()
            out[f"step{step}/taus"] = np.stack(taus_rec)  # (3, B, 8, 1): target, local, actor-step
            out[f"step{step}/critic_loss"] = np.float64(closs)
            out[f"step{step}/actor_loss"] = np.float64(aloss)
            out[f"step{step}/grad_norms"] = np.array(cr.norms)  # critic, actor (pre-clip)
            if step in (0, 2):
                out.update(sd_arrays(f"after{step}/actor/", agent.policy_local.actor))
                out.update(sd_arrays(f"after{step}/critic/", agent.policy_local.critic))
    finally:
        Critic.calc_cos = orig_calc

    # N = N' = 32: the same 20 lines (agent.py:386-427) with num_tau=32, the shape assert
    # (agent.py:407) being the only thing that pins 8. Reference modules, reference math.
    agent = ref_agent_mod.Agent(device="cpu", seed=100, agent_type="AC-IQN")
    taus_rec = []
    Critic.calc_cos = rec_calc
    try:
        idx = rs.choice(len(trans), 64, replace=False)
        batch = make_batch(agent, trans, idx)
        out.update(batch_arrays("n32/", *batch, 64))
        states, actions, rewards, next_states, dones = batch
        states = agent.state_to_tensor(states)
        actions = torch.tensor(actions).float()
        rewards = torch.tensor(rewards).unsqueeze(-1).float()
        next_states = agent.state_to_tensor(next_states)
        dones = torch.tensor(dones).unsqueeze(-1).float()
        NT = 32
        with ClipRecorder() as cr:
            agent.critic_optimizer.zero_grad()
            next_actions = agent.policy_target.actor(next_states).detach()
            qn, _ = agent.policy_target.critic(next_states, next_actions, num_tau=NT)
            qn = qn.detach().unsqueeze(1)
            qt = rewards.unsqueeze(-1) + (agent.GAMMA * qn * (1. - dones.unsqueeze(-1)))
            qe, taus = agent.policy_local.critic(states, actions, num_tau=NT)
            qe = qe.unsqueeze(-1)
            td = qt - qe
            hub = torch.where(td.abs() <= 1.0, 0.5 * td.pow(2), 1.0 * (td.abs() - 0.5 * 1.0))
            ql = abs(taus - (td.detach() < 0).float()) * hub / 1.0
            closs = ql.sum(dim=1).mean(dim=1).mean()
            closs.backward()
            torch.nn.utils.clip_grad_norm_(agent.policy_local.critic.parameters(), 0.5)
            agent.critic_optimizer.step()
            agent.actor_optimizer.zero_grad()
            ao = agent.policy_local.actor(states)
            al, _ = agent.policy_local.critic(states, ao, num_tau=NT)
            al = -al.mean()
            al.backward()
            torch.nn.utils.clip_grad_norm_(agent.policy_local.actor.parameters(), 0.5)
            agent.actor_optimizer.step()
        out["n32/taus"] = np.stack(taus_rec)
        out["n32/critic_loss"] = np.float64(closs.item())
        out["n32/actor_loss"] = np.float64(al.item())
        out["n32/grad_norms"] = np.array(cr.norms)
        out.update(sd_arrays("n32after/actor/", agent.policy_local.actor))
        out.update(sd_arrays("n32after/critic/", agent.policy_local.critic))
    finally:
        Critic.calc_cos = orig_calc

    # actor forward on a batch with no objects at all (x_2 is None path,
    # AC_IQN_model.py:293-294) and on a full batch
    agent = ref_agent_mod.Agent(device="cpu", seed=100, agent_type="AC-IQN")
    noobj = [t for t in trans if len(t[0][1]) == 0][:8]
    st = agent.memory.state_batch([t[0] for t in noobj])
    assert len(st[1]) == 0
    with torch.no_grad():
        out["fwd/noobj_self"] = np.array(st[0], dtype=np.float64)
        out["fwd/noobj_actions"] = agent.policy_local.actor(agent.state_to_tensor(st)).numpy()
    np.savez_compressed(os.path.join(OUT, "learn_ac_iqn.npz"), **out)
    print("ac_iqn keys:", len(out))


def capture_iqn():
    out = {}
    trans = collect_transitions(600, seed=4, discrete=True)
    rs = np.random.RandomState(41)
    agent = ref_agent_mod.Agent(device="cpu", seed=100, agent_type="IQN")
    out.update(sd_arrays("init/", agent.policy_local))
    taus_rec = []
    orig_calc = IQN_Policy.calc_cos

    def rec_calc(self, batch_size, num_tau=8, cvar=1.0):
        cos, taus = orig_calc(self, batch_size, num_tau, cvar)
        taus_rec.append(taus.detach().numpy().copy())
        return cos, taus
    IQN_Policy.calc_cos = rec_calc
    try:
        for step in range(3):
            idx = rs.choice(len(trans), 64, replace=False)
            batch = make_batch(agent, trans, idx)
            out.update(batch_arrays(f"step{step}/", *batch, 64))
            agent.memory.sample = (lambda b=batch: b)
            taus_rec.clear()
            with ClipRecorder() as cr:
                loss = agent.train_IQN()
            out[f"step{step}/taus"] = np.stack(taus_rec)  # (2, B, 8, 1): target, local
            out[f"step{step}/loss"] = np.float64(loss)
            out[f"step{step}/grad_norms"] = np.array(cr.norms)
            if step in (0, 2):
                out.update(sd_arrays(f"after{step}/", agent.policy_local))
        # act_iqn (agent.py:227-250): K=32 quantiles, argmax of the mean
        taus_rec.clear()
        st = trans[5][0]
        import random as pyrandom
        pyrandom.seed(5)
        a, q, tq = agent.act_iqn(st, eps=0.0)
        out["act/state_self"] = np.array(st[0], dtype=np.float64)
        out["act/state_obj"] = np.array(st[1], dtype=np.float64).reshape(-1, 5)
        out["act/action"] = np.int64(a)
        out["act/quantiles"] = q
        out["act/taus"] = tq
    finally:
        IQN_Policy.calc_cos = orig_calc
    np.savez_compressed(os.path.join(OUT, "learn_iqn.npz"), **out)
    print("iqn keys:", len(out))


class TorchZerosProxy(types.ModuleType):
    """Stand-in for the `torch` name inside rfarl.agent that records torch.zeros outputs
    (the C51 target m, agent.py:628) while passing everything else through."""

    def __init__(self, real):
        super().__init__("torch_proxy")
        self._real = real
        self.captured = []

    def __getattr__(self, name):
        return getattr(self._real, name)

    def zeros(self, *a, **k):
        z = self._real.zeros(*a, **k)
        self.captured.append(z)
        return z


def capture_rainbow():
    out = {}
    trans = collect_transitions(400, seed=5, discrete=True)
    rs = np.random.RandomState(51)
    dims = dict(self_feature_dimension=8, object_feature_dimension=8, concat_feature_dimension=48,
                hidden_dimension=16)
    out["dims"] = np.array([8, 8, 48, 16])
    for bsz, tag in ((64, "b64"), (1024, "b1024")):
        agent = ref_agent_mod.Agent(device="cpu", seed=100, agent_type="Rainbow", BATCH_SIZE=bsz, **dims)
        if tag == "b64":
            out.update(sd_arrays("init/", agent.policy_local))
            out.update({"init_target/" + k: v for k, v in sd_arrays("", agent.policy_target).items()})
        idx = rs.choice(len(trans), bsz, replace=len(trans) < bsz)
        samples = [trans[i] for i in idx]
        s = agent.memory.state_batch([t[0] for t in samples])
        ns = agent.memory.state_batch([t[3] for t in samples])
        st = (torch.tensor(s[0]).float(), torch.tensor(s[1]).float(), torch.tensor(s[2]).float())
        nst = (torch.tensor(ns[0]).float(), torch.tensor(ns[1]).float(), torch.tensor(ns[2]).float())
        actions = torch.tensor([t[1] for t in samples], dtype=torch.int64)
        # n-step returns across the projection's edge cases: exact-integer b (l == u fix,
        # agent.py:622-624), clamping at Vmin/Vmax, terminal and non-terminal
        R = torch.tensor(rs.uniform(-1.5, 1.5, size=bsz), dtype=torch.float32)
        nonterm = torch.tensor(rs.randint(0, 2, size=(bsz, 1)), dtype=torch.float32)
        R[0], nonterm[0] = 0.0, 0.0      # b = 25 exactly
        R[1], nonterm[1] = -1.0, 0.0     # b = 0 exactly
        R[2], nonterm[2] = 1.0, 0.0      # b = 50 exactly
        R[3], nonterm[3] = 5.0, 1.0      # clamp high
        R[4], nonterm[4] = -5.0, 1.0     # clamp low
        R[5], nonterm[5] = 0.0, 1.0      # b integer for every atom when gamma^n z is on-grid? (not exactly)
        R[6], nonterm[6] = 0.4, 0.0      # b = 35 exactly in f32?
        weights = torch.tensor(rs.uniform(0.2, 1.0, size=bsz), dtype=torch.float32)
        weights = weights / weights.max()
        batch = (np.arange(bsz), st, actions, R, nst, nonterm, weights)
        agent.memory.sample = (lambda b, batch=batch: batch)
        prio = []
        agent.memory.update_priorities = lambda i, p: prio.append(np.array(p))
        with torch.no_grad():
            pns_online = agent.policy_local(nst)
            argmax_ns = (agent.support.expand_as(pns_online) * pns_online).sum(2).argmax(1)
        proxy = TorchZerosProxy(torch)
        ref_agent_mod.torch = proxy
        try:
            with ClipRecorder() as cr:
                loss = agent.train_Rainbow()
        finally:
            ref_agent_mod.torch = torch
        m = [z for z in proxy.captured if tuple(z.shape) == (bsz, 51)]
        assert len(m) == 1
        with torch.no_grad():
            pns_t = agent.policy_target(nst)
            pns_a = pns_t[range(bsz), argmax_ns]
        p = tag + "/"
        out[p + "s_self"], out[p + "s_obj"], out[p + "s_mask"] = [x.numpy() for x in st]
        out[p + "ns_self"], out[p + "ns_obj"], out[p + "ns_mask"] = [x.numpy() for x in nst]
        out[p + "actions"] = actions.numpy()
        out[p + "returns"] = R.numpy()
        out[p + "nonterminal"] = nonterm.numpy()
        out[p + "weights"] = weights.numpy()
        out[p + "argmax_ns"] = argmax_ns.numpy()
        out[p + "pns_a"] = pns_a.numpy()
        out[p + "m"] = m[0].numpy()
        out[p + "loss"] = np.array(loss)
        out[p + "priorities"] = prio[0]
        out[p + "grad_norm"] = np.array(cr.norms)
        out[p + "support"] = agent.support.numpy()
        # target noise buffers drawn by reset_noise() inside train (agent.py:612)
        out.update({p + "target_after/" + k: v for k, v in sd_arrays("", agent.policy_target).items()
                    if "epsilon" in k})
        if tag == "b64":
            out.update(sd_arrays("after/", agent.policy_local))
    np.savez_compressed(os.path.join(OUT, "learn_rainbow.npz"), **out)
    print("rainbow keys:", len(out))


def capture_rainbow_full():
    """F6b: Agent.train_Rainbow (agent.py:597-641) at the default network size (the size the Rainbow
    kernels take), compact: the networks come from oracle.learn_ref.synthetic_rainbow_state(seed) (numpy,
    reproducible bit for bit), so the fixture holds the seed, the batch, the target noise reset_noise drew
    inside train (its eps_in / eps_out vectors, recorded per layer), and the outputs: per-sample loss,
    m, the online argmax over s_{t+n}, p(s_{t+n}, a*), the pre-clip gradient norm, and per parameter the
    post-clip gradient and the parameter after the Adam step (full for tensors of <= 4096 elements, else
    at 2048 fixed sampled positions plus f64 sum / sum of squares of the whole tensor)."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from oracle import learn_ref as lr
    out = {}
    seed, bsz = 7, 64
    out["seed"] = np.array([seed])
    sd = lr.synthetic_rainbow_state(seed)
    agent = ref_agent_mod.Agent(device="cpu", seed=100, agent_type="Rainbow", BATCH_SIZE=bsz)
    with torch.no_grad():
        for net in (agent.policy_local, agent.policy_target):
            for k, v in net.state_dict().items():
                v.copy_(torch.from_numpy(sd[k]))
    # record the target's reset_noise draws (eps_in, eps_out per layer, in the reference's call order)
    rec = {}
    for name, layer in agent.policy_target.named_children():
        if "hidden_layer" in name or "output_layer" in name:
            orig = layer._scale_noise

            def wrapped(size, orig=orig, name=name):
                x = orig(size)
                rec.setdefault(name, []).append(x.detach().numpy().copy())
                return x
            layer._scale_noise = wrapped
    trans = collect_transitions(400, seed=9, discrete=True)
    rs = np.random.RandomState(61)
    idx = rs.choice(len(trans), bsz, replace=False)
    samples = [trans[i] for i in idx]
    s = agent.memory.state_batch([t[0] for t in samples])
    ns = agent.memory.state_batch([t[3] for t in samples])
    st = tuple(torch.tensor(x).float() for x in s)
    nst = tuple(torch.tensor(x).float() for x in ns)
    actions = torch.tensor([t[1] for t in samples], dtype=torch.int64)
    R = torch.tensor(rs.uniform(-1.5, 1.5, size=bsz), dtype=torch.float32)
    nonterm = torch.tensor(rs.randint(0, 2, size=(bsz, 1)), dtype=torch.float32)
    R[0], nonterm[0] = 0.0, 0.0      # b = 25 exactly (the l == u fix)
    R[1], nonterm[1] = -1.0, 0.0     # b = 0
    R[2], nonterm[2] = 1.0, 0.0      # b = 50
    R[3], nonterm[3] = 5.0, 1.0      # clamped high
    R[4], nonterm[4] = -5.0, 1.0     # clamped low
    weights = torch.tensor(rs.uniform(0.2, 1.0, size=bsz), dtype=torch.float32)
    weights = weights / weights.max()
    batch = (np.arange(bsz), st, actions, R, nst, nonterm, weights)
    agent.memory.sample = (lambda b, batch=batch: batch)
    prio = []
    agent.memory.update_priorities = lambda i, p: prio.append(np.array(p))
    with torch.no_grad():
        pns_online = agent.policy_local(nst)
        argmax_ns = (agent.support.expand_as(pns_online) * pns_online).sum(2).argmax(1)
    grads = {}
    opt_step = agent.optimizer.step

    def step_rec(*a, **k):   # the clipped gradient the optimizer applies
        for n, p in agent.policy_local.named_parameters():
            grads[n] = p.grad.detach().numpy().astype(np.float32).copy()
        return opt_step(*a, **k)
    agent.optimizer.step = step_rec
    proxy = TorchZerosProxy(torch)
    ref_agent_mod.torch = proxy
    try:
        with ClipRecorder() as cr:
            loss = agent.train_Rainbow()
    finally:
        ref_agent_mod.torch = torch
    m = [z for z in proxy.captured if tuple(z.shape) == (bsz, 51)]
    assert len(m) == 1
    with torch.no_grad():
        pns_a = agent.policy_target(nst)[range(bsz), argmax_ns]
    for name, xs in rec.items():
        assert len(xs) == 2, (name, len(xs))
        out["target_eps_in/" + name], out["target_eps_out/" + name] = xs[0], xs[1]
    out["s_self"], out["s_obj"], out["s_mask"] = [x.numpy() for x in st]
    out["ns_self"], out["ns_obj"], out["ns_mask"] = [x.numpy() for x in nst]
    out["actions"], out["returns"], out["nonterminal"] = actions.numpy(), R.numpy(), nonterm.numpy()
    out["weights"], out["argmax_ns"], out["pns_a"] = weights.numpy(), argmax_ns.numpy(), pns_a.numpy()
    out["m"], out["loss"], out["priorities"] = m[0].numpy(), np.array(loss), prio[0]
    out["grad_norm"] = np.array(cr.norms)
    pick = np.random.RandomState(5)
    for n, p in agent.policy_local.named_parameters():
        g, a = grads[n].reshape(-1), p.detach().numpy().reshape(-1)
        if g.size <= 4096:
            out["grad/" + n], out["after/" + n] = g, a.copy()
        else:
            ix = np.sort(pick.choice(g.size, 2048, replace=False))
            out["idx/" + n] = ix.astype(np.int32)
            out["grad/" + n], out["after/" + n] = g[ix], a[ix].copy()
            out["gsum/" + n] = np.array([g.astype(np.float64).sum(), (g.astype(np.float64) ** 2).sum()])
            out["asum/" + n] = np.array([a.astype(np.float64).sum(), (a.astype(np.float64) ** 2).sum()])
    np.savez_compressed(os.path.join(OUT, "learn_rainbow_full.npz"), **out)
    print("rainbow_full keys:", len(out), "loss mean", float(np.mean(loss)), "grad norm", cr.norms)


def capture_evalcfg():
    """F2c: MarineNavEnv3.reset_with_eval_config (env.py:503-614) with every robot's own vehicle and
    perception parameters (dt, N, size, goal distance, thrust limits and grid, m, Izz, the hydrodynamic
    coefficients, perception range / angle / max_obj_num / sigma / kappa), and a scene with 20 vortex
    cores; then env.step traces as capture_traces records them (every perception draw). The eval config
    is stored as its JSON text (env_evalcfg.npz, key <name>/config)."""
    import contextlib
    import io
    import json

    def cont_fn(seed):
        rs = np.random.RandomState(177 + seed)
        return lambda t, i: [float(rs.uniform(-1, 1)), float(rs.uniform(-1, 1))]

    def base_config(seed, R, O, cores, msgd, width):
        e = MarineNavEnv3(seed=seed)
        e.num_robots, e.num_cores, e.num_obs, e.min_start_goal_dis = R, cores, O, msgd
        e.width = e.height = width
        with contextlib.redirect_stdout(io.StringIO()):
            e.reset()
        return json.loads(json.dumps(e.episode_data()))

    def vary(cfg, seed):
        rs = np.random.RandomState(seed)
        rb = cfg["robots"]
        n = cfg["env"]["num_robots"]
        scale = lambda k, lo, hi: [float(v * rs.uniform(lo, hi)) for v in rb[k]]  # noqa: E731
        for k in ("m", "Izz", "xDotU", "yDotV", "yDotR", "nDotR", "nDotV", "xU", "xUU", "yV", "yVV", "yR", "yRV",
                  "yVR", "yRR", "nR", "nRR", "nV", "nVV", "nRV", "nVR"):
            rb[k] = scale(k, 0.7, 1.3)
        rb["dt"] = [[0.05, 0.04, 0.05, 0.06, 0.05][i % 5] for i in range(n)]
        rb["N"] = [[10, 12, 8, 10, 10][i % 5] for i in range(n)]
        rb["length"] = scale("length", 0.8, 1.2)
        rb["width"] = scale("width", 0.8, 1.2)
        rb["r"] = [float(0.5 * np.sqrt(L * L + W * W)) for L, W in zip(rb["length"], rb["width"])]
        rb["detect_r"] = list(rb["r"])
        rb["goal_dis"] = [[2.0, 2.5, 1.5, 3.0, 2.0][i % 5] for i in range(n)]
        rb["min_thrust"] = [[-500.0, -400.0, -600.0, -500.0, -450.0][i % 5] for i in range(n)]
        rb["max_thrust"] = [[1000.0, 900.0, 1100.0, 800.0, 1000.0][i % 5] for i in range(n)]
        pe = rb["perception"]
        pe["range"] = [[20.0, 15.0, 25.0, 18.0, 22.0][i % 5] for i in range(n)]
        pe["angle"] = [[2 * np.pi, 1.5 * np.pi, 2 * np.pi, np.pi, 2 * np.pi][i % 5] for i in range(n)]
        pe["max_obj_num"] = [[5, 4, 5, 3, 5][i % 5] for i in range(n)]
        pe["pos_std"] = [[0.05, 0.1, 0.02, 0.08, 0.05][i % 5] for i in range(n)]
        pe["vel_std"] = [[0.05, 0.03, 0.1, 0.05, 0.07][i % 5] for i in range(n)]
        pe["r_kappa"] = [[1.0, 2.0, 0.5, 1.0, 3.0][i % 5] for i in range(n)]
        pe["r_mean_ratio"] = [[0.8, 0.7, 0.9, 0.8, 0.75][i % 5] for i in range(n)]
        return cfg

    cases = {   # name -> (base seed, R, O, cores, msgd, width, vary robots, eval env seed, steps)
        "evalcfg_r5o4_s11": (11, 5, 4, 0, 40.0, 55, True, 21, 100),
        "evalcfg_r8o4_s13": (13, 8, 4, 0, 30.0, 80, True, 23, 120),
        "cores20_r5o4_s12": (12, 5, 4, 20, 30.0, 110, False, 22, 60),
    }
    out = {}
    for name, (seed, R, O, nc, msgd, width, var, eseed, steps) in cases.items():
        cfg = base_config(seed, R, O, nc, msgd, width)
        if var:
            cfg = vary(cfg, 500 + seed)
        env = MarineNavEnv3(seed=eseed)   # reset_with_eval_config re-seeds env.rd from the config
        env.num_robots = R                # ... and draws the robots' seeds in [0, 5 * num_robots)
        text = json.dumps(cfg)

        def reset(e, text=text):
            with contextlib.redirect_stdout(io.StringIO()):
                e.reset_with_eval_config(json.loads(text))
        tr = run_trace(env, steps, cont_fn(seed), True, R, O, reset=reset)
        for k, v in tr.items():
            out[f"{name}/{k}"] = v
        out[f"{name}/R"], out[f"{name}/O"] = np.int32(R), np.int32(O)
        out[f"{name}/config"] = np.array(text)
        out[f"{name}/num_robots_attr"] = np.int32(R)
        print(f"evalcfg {name}: steps={len(tr['reward'])} robots={tr['n_robots']} cores={len(env.cores)} "
              f"collisions={int(tr['collision'].sum())} reach={int(tr['reach'].sum())} "
              f"colregs={int(tr['apply_colregs'].sum())}")
    out["names"] = np.array(list(cases.keys()))
    np.savez_compressed(os.path.join(OUT, "env_evalcfg.npz"), **out)


def capture_dqn():
    """F8: Agent.train_DQN (agent.py:518-545) x 2 steps and act_dqn's Q values (agent.py:271-287)."""
    out = {}
    trans = collect_transitions(300, seed=6, discrete=True)
    rs = np.random.RandomState(61)
    agent = ref_agent_mod.Agent(device="cpu", seed=100, agent_type="DQN")
    out.update(sd_arrays("init/", agent.policy_local))
    for step in range(2):
        idx = rs.choice(len(trans), 64, replace=False)
        batch = make_batch(agent, trans, idx)
        out.update(batch_arrays(f"step{step}/", *batch, 64))
        agent.memory.sample = (lambda b=batch: b)
        with ClipRecorder() as cr:
            loss = agent.train_DQN()
        out[f"step{step}/loss"] = np.float64(loss)
        out[f"step{step}/grad_norms"] = np.array(cr.norms)
    out.update(sd_arrays("after1/", agent.policy_local))
    st = trans[7][0]
    a = agent.act_dqn(st, eps=0.0)
    with torch.no_grad():
        q = agent.policy_local(agent.state_to_tensor(agent.memory.state_batch([st]))).numpy()
    out["act/state_self"] = np.array(st[0], dtype=np.float64)
    out["act/state_obj"] = np.array(st[1], dtype=np.float64).reshape(-1, 5)
    out["act/action"] = np.int64(a)
    out["act/q"] = np.asarray(q)
    np.savez_compressed(os.path.join(OUT, "learn_dqn.npz"), **out)
    print("dqn keys:", len(out))


EVAL_SCHEDULE = {"num_episodes": [2, 2], "num_robots": [3, 5], "num_cores": [0, 2], "num_obstacles": [2, 4],
                 "min_start_goal_dis": [30.0, 40.0]}


def capture_eval():
    """F9: Trainer.evaluation (trainer.py:266-392) with the seeded initial AC-IQN and Rainbow agents
    (greedy, batch-1 CPU policy per robot) on the eval configs of EVAL_SCHEDULE: the configs, the
    network weights and every per-config metric, per-robot trajectory and action history."""
    import json
    import random
    from rfarl.policy.trainer import Trainer
    out = {}
    for kind in ("AC-IQN", "Rainbow"):
        torch.manual_seed(0)
        agent = ref_agent_mod.Agent(device="cpu", seed=100, agent_type=kind)
        tr = Trainer(MarineNavEnv3(seed=1), MarineNavEnv3(seed=253, is_eval_env=True), EVAL_SCHEDULE, agent)
        random.seed(77)
        np.random.seed(77)
        tr.evaluation()
        p = kind + "/"
        out[p + "configs"] = np.array(json.dumps(tr.eval_config))
        net = agent.policy_local.actor if kind == "AC-IQN" else agent.policy_local
        out.update(sd_arrays(p + "net/", net))
        out[p + "rewards"] = np.array(tr.eval_rewards[0], dtype=np.float64)
        out[p + "successes"] = np.array(tr.eval_successes[0], dtype=bool)
        out[p + "times"] = np.array(tr.eval_times[0], dtype=np.float64)
        out[p + "energies"] = np.array(tr.eval_energies[0], dtype=np.float64)
        for e, ep in enumerate(tr.eval_trajectories[0]):
            for i, traj in enumerate(ep):
                out[f"{p}traj/{e}/{i}"] = np.array(traj, dtype=np.float64)
                out[f"{p}act/{e}/{i}"] = np.array(tr.eval_actions[0][e][i], dtype=np.float64)
        print(kind, "eval lengths", [[len(t) for t in ep] for ep in tr.eval_trajectories[0]],
              "successes", tr.eval_successes[0])
    np.savez_compressed(os.path.join(OUT, "eval_ref.npz"), **out)
    print("eval keys:", len(out))


def capture_eval_iqn():
    """F9b: Trainer.evaluation (trainer.py:266-392) with the seeded initial IQN agent on the eval configs of
    EVAL_SCHEDULE, recording the K = 32 quantile fractions of EVERY act_iqn call (agent.py:227-250, drawn by
    IQN_Policy.calc_cos, IQN_model.py:56-72) keyed by (config, step, robot), with the action it chose and its
    mean quantiles; plus the per-config metrics, trajectories and action histories. The parity test injects the
    same taus into the batched evaluation (eval_iqn_ref.npz)."""
    import json
    import random
    from rfarl.policy.trainer import Trainer
    out = {}
    torch.manual_seed(0)
    agent = ref_agent_mod.Agent(device="cpu", seed=100, agent_type="IQN")
    eval_env = MarineNavEnv3(seed=253, is_eval_env=True)
    tr = Trainer(MarineNavEnv3(seed=1), eval_env, EVAL_SCHEDULE, agent)
    pos = {"e": -1, "t": 0, "k": 0}
    calls = []   # (config, step, robot, action, taus[32], mean quantiles[25])
    orig_reset, orig_step, orig_act = eval_env.reset_with_eval_config, eval_env.step, agent.act_iqn

    def reset(cfg):
        pos["e"] += 1
        pos["t"] = pos["k"] = 0
        return orig_reset(cfg)

    def step(action, cont):
        r = orig_step(action, cont)
        pos["t"] += 1
        pos["k"] = 0
        return r

    def act(state, *a, **k):
        active = [i for i, rob in enumerate(eval_env.robots) if not rob.deactivated]
        robot = active[pos["k"]]
        pos["k"] += 1
        action, q, taus = orig_act(state, *a, **k)
        calls.append((pos["e"], pos["t"], robot, int(action), np.asarray(taus, np.float32).reshape(-1),
                      np.asarray(q, np.float64).mean(axis=1).reshape(-1)))
        return action, q, taus
    eval_env.reset_with_eval_config, eval_env.step, agent.act_iqn = reset, step, act
    random.seed(77)
    np.random.seed(77)
    tr.evaluation()
    p = "IQN/"
    out[p + "configs"] = np.array(json.dumps(tr.eval_config))
    out.update(sd_arrays(p + "net/", agent.policy_local))
    out[p + "rewards"] = np.array(tr.eval_rewards[0], dtype=np.float64)
    out[p + "successes"] = np.array(tr.eval_successes[0], dtype=bool)
    out[p + "times"] = np.array(tr.eval_times[0], dtype=np.float64)
    out[p + "energies"] = np.array(tr.eval_energies[0], dtype=np.float64)
    out[p + "lengths"] = np.array([max(len(t) for t in ep) for ep in tr.eval_trajectories[0]], dtype=np.int64)
    for e, ep in enumerate(tr.eval_trajectories[0]):
        for i, traj in enumerate(ep):
            out[f"{p}traj/{e}/{i}"] = np.array(traj, dtype=np.float64)
            out[f"{p}act/{e}/{i}"] = np.array(tr.eval_actions[0][e][i], dtype=np.float64)
    out[p + "calls/key"] = np.array([c[:3] for c in calls], dtype=np.int32)
    out[p + "calls/action"] = np.array([c[3] for c in calls], dtype=np.int32)
    out[p + "calls/taus"] = np.stack([c[4] for c in calls]).astype(np.float32)
    out[p + "calls/qmean"] = np.stack([c[5] for c in calls]).astype(np.float32)
    print("IQN eval lengths", [[len(t) for t in ep] for ep in tr.eval_trajectories[0]], "successes",
          tr.eval_successes[0], "act calls", len(calls))
    np.savez_compressed(os.path.join(OUT, "eval_iqn_ref.npz"), **out)


def capture_eval60():
    """F10: Trainer.evaluation (trainer.py:266-392) on the SHIPPED eval schedule (config/ac_iqn.json
    eval_schedule: 60 episodes over six curriculum stages, 3-5 robots, 0-4 buoys) with two AC-IQN agents:
    'init' = the seeded initial agent (its episodes mostly run to the 1000-step limit), 'trained' = the same
    agent after 200 reference train_AC_IQN steps (agent.py:386-432) on a replay filled by 3000 steps of the
    reference env under uniform actions (the trainer's add / deactivation, trainer.py:155-172). Stored: the
    60 configs, each agent's actor weights, the per-config metrics (mean return, success, mean time, mean
    energy) and per robot the trajectory length and final trajectory row (tests/golden/eval60_ref.npz)."""
    import contextlib
    import io
    import json
    import random
    from rfarl.policy.trainer import Trainer
    sched = json.load(open(os.path.join(REF, "rfarl", "config", "ac_iqn.json")))["eval_schedule"]
    out = {}
    for tag in ("init", "trained"):
        torch.manual_seed(0)
        random.seed(5)
        np.random.seed(5)
        agent = ref_agent_mod.Agent(device="cpu", seed=100, agent_type="AC-IQN")
        if tag == "trained":
            env = MarineNavEnv3(seed=3)
            env.num_robots, env.num_cores, env.num_obs, env.min_start_goal_dis = 5, 0, 4, 40.0
            rs = np.random.RandomState(9)
            with contextlib.redirect_stdout(io.StringIO()):
                states, _, _ = env.reset()
            for t in range(3000):
                acts = [None if r.deactivated else [float(rs.uniform(-1, 1)), float(rs.uniform(-1, 1))]
                        for r in env.robots]
                nxt, rew, done, _ = env.step(acts, True)
                for i, r in enumerate(env.robots):
                    if r.deactivated:
                        continue
                    agent.memory.add((states[i], acts[i], rew[i], nxt[i], done[i]))
                    if r.collision or r.reach_goal:
                        r.deactivated = True
                states = nxt
                if env.check_all_deactivated() or env.episode_timesteps >= 1000:
                    with contextlib.redirect_stdout(io.StringIO()):
                        states, _, _ = env.reset()
            for _ in range(200):
                agent.train()
        tr = Trainer(MarineNavEnv3(seed=1), MarineNavEnv3(seed=253, is_eval_env=True), sched, agent)
        random.seed(77)
        np.random.seed(77)
        with contextlib.redirect_stdout(io.StringIO()):
            tr.evaluation()
        p = tag + "/"
        out[p + "configs"] = np.array(json.dumps(tr.eval_config))
        out.update(sd_arrays(p + "net/", agent.policy_local.actor))
        out[p + "rewards"] = np.array(tr.eval_rewards[0], dtype=np.float64)
        out[p + "successes"] = np.array(tr.eval_successes[0], dtype=bool)
        out[p + "times"] = np.array(tr.eval_times[0], dtype=np.float64)
        out[p + "energies"] = np.array(tr.eval_energies[0], dtype=np.float64)
        lens, last = [], []
        for ep in tr.eval_trajectories[0]:
            for traj in ep:
                lens.append(len(traj))
                last.append(np.array(traj[-1], dtype=np.float64))
        out[p + "traj_len"] = np.array(lens, np.int32)
        out[p + "traj_last"] = np.array(last)
        out[p + "robots"] = np.array([len(ep) for ep in tr.eval_trajectories[0]], np.int32)
        print(tag, "successes", int(np.sum(tr.eval_successes[0])), "of", len(tr.eval_successes[0]),
              "lengths", [max(len(t) for t in ep) for ep in tr.eval_trajectories[0]])
    np.savez_compressed(os.path.join(OUT, "eval60_ref.npz"), **out)


def capture_eval60_tf():
    """F10b: the two F10 evaluations (trainer.py:266-392) again, from F10's stored configs and actor weights
    (tests/golden/eval60_ref.npz), recording per robot of every episode the actions the reference applied
    (Robot.action_history, env.py:264: the batch-1 actor's f32 outputs as Python floats) and its perception
    noise stream (every rd.normal / rd.vonmises draw of wamv.py:27-40 through a recording proxy: the count, the
    sum and the sum of squares). The metrics are asserted equal to F10's, so the two fixtures describe the same
    runs. Stored in tests/golden/eval60_tf.npz."""
    import contextlib
    import io
    import json
    import random
    from rfarl.policy.trainer import Trainer
    z = np.load(os.path.join(OUT, "eval60_ref.npz"))
    sched = json.load(open(os.path.join(REF, "rfarl", "config", "ac_iqn.json")))["eval_schedule"]
    out = {}
    for tag in ("init", "trained"):
        p = tag + "/"
        torch.manual_seed(0)
        agent = ref_agent_mod.Agent(device="cpu", seed=100, agent_type="AC-IQN")
        sd = {k[len(p + "net/"):]: torch.from_numpy(z[k]) for k in z.files if k.startswith(p + "net/")}
        agent.policy_local.actor.load_state_dict(sd)
        tr = Trainer(MarineNavEnv3(seed=1), MarineNavEnv3(seed=253, is_eval_env=True), sched, agent)
        tr.eval_config = json.loads(str(z[p + "configs"]))
        ev = tr.eval_env
        logs = []   # per episode: the robots' recorders
        orig = ev.reset_with_eval_config

        def reset(cfg, orig=orig, ev=ev, logs=logs):
            res = orig(cfg)
            install_recorders(ev)
            clear_recorders(ev)
            logs.append([rob.perception.rd for rob in ev.robots])
            return res
        ev.reset_with_eval_config = reset
        random.seed(77)
        np.random.seed(77)
        with contextlib.redirect_stdout(io.StringIO()):
            tr.evaluation()
        for key in ("rewards", "energies", "times"):
            assert np.array_equal(np.array(tr.eval_rewards[0] if key == "rewards" else
                                           (tr.eval_energies[0] if key == "energies" else tr.eval_times[0])),
                                  z[p + key]), f"{tag}: {key} differ from eval60_ref.npz"
        acts, alen = [], []
        for ep in tr.eval_actions[0]:
            for a in ep:
                alen.append(len(a))
                acts.extend(np.asarray(x, dtype=np.float64).reshape(2) for x in a)
        out[p + "act"] = np.array(acts, dtype=np.float64).reshape(-1, 2)
        out[p + "act_len"] = np.array(alen, np.int32)
        dn, ds, dq = [], [], []
        for ep in logs:
            for rd in ep:
                v = np.array(rd.log, dtype=np.float64)
                dn.append(len(v))
                ds.append(float(v.sum()))
                dq.append(float((v * v).sum()))
        out[p + "draws_n"] = np.array(dn, np.int64)
        out[p + "draws_sum"] = np.array(ds)
        out[p + "draws_sq"] = np.array(dq)
        assert len(alen) == len(dn) == int(z[p + "robots"].sum())
        print(tag, "robots", len(alen), "steps", int(np.sum(alen)), "draws", int(np.sum(dn)))
    np.savez_compressed(os.path.join(OUT, "eval60_tf.npz"), **out)


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    what = sys.argv[1:] or ["dynamics", "traces", "reset", "ac_iqn", "iqn", "rainbow", "dqn"]
    torch.set_num_threads(1)
    for w in what:
        globals()["capture_" + w]()
