"""MarineNavEnv3 -- drop-in for rfarl.envs.marinenav.env.MarineNavEnv3 (env.py:24-778).

Same constructor, attributes, RandomState consumption, reset / step / eval-config / episode
I/O behaviour as the reference. The per-step physics, perception, COLREGs and reward run in
the gfx950 env-step kernel (libasvrl.so, asvrl_env_step) on a one-env device batch; the
host keeps the reference's Robot objects (so Trainer can read and write them) and draws the
perception noise from each robot's own numpy RandomState in the reference's order, which the
kernel consumes as injected draws -- results therefore match the reference, not just its
distribution. Episode setup (reset's rejection sampler, env.py:72-164) stays on the host as
in the reference; the vectorised fast path (vec_env.VecMarineNavEnv) resets on the device.
"""
import copy
import json

import numpy as np
import torch

from ... import _abi
from ...device_env import DeviceEnvBatch, current_field
from .vehicles import wamv as robot


class Core:
    def __init__(self, x: float, y: float, clockwise: bool, Gamma: float):
        self.x = x
        self.y = y
        self.clockwise = clockwise
        self.Gamma = Gamma


class Obstacle:
    def __init__(self, x: float, y: float, r: float):
        self.x = x
        self.y = y
        self.r = r


class MarineNavEnv3:

    def __init__(self, seed: int = 0, schedule: dict = None, is_eval_env: bool = False, device=None):
        self.seed = seed
        self.rd = np.random.RandomState(seed)
        self.is_eval_env = is_eval_env
        self.width = 55
        self.height = 55
        self.r = 0.5
        self.v_rel_max = 1.0
        self.p = 0.8
        self.v_range = [3, 3]
        self.obs_r_range = [1, 1]
        self.clear_r = 10.0
        self.angular_speed_max = np.pi / 2
        self.angular_speed_penalty = -1.0
        self.steering_reward_angle_max = np.pi / 3
        self.steering_reward_speed_min = 1.0
        self.steering_reward = 0.5
        self.timestep_penalty = -0.1
        self.COLREGs_penalty = -0.1
        self.collision_penalty = -5.0
        self.goal_reward = 10.0
        self.num_cores = 8
        self.num_obs = 8
        self.min_start_goal_dis = 30.0
        self.num_robots = 6
        self.robots = []
        for _ in range(self.num_robots):  # env.py:56-58 (consumes the same randints)
            self.robots.append(robot.Robot(seed=self.rd.randint(0, 5 * self.num_robots)))
        self.cores = []
        self.obstacles = []
        self.schedule = schedule
        self.episode_timesteps = 0
        self.total_timesteps = 0
        self.observation_in_robot_frame = True
        self._device = torch.device(device) if device is not None else torch.device("cuda")
        self._batch = None
        self._shape = (0, 0, 0)

    def get_action_space_dimension(self):
        return self.robots[0].compute_actions_dimension()

    # ------------------------------------------------------------------ reset (env.py:72-164)
    def reset(self):
        self.reset_layout()
        return self.get_observations()

    def reset_layout(self):
        """The host part of reset(): curriculum lookup and the rejection sampler, consuming
        self.rd exactly as env.py:72-162 does. get_observations() is the device part."""
        if self.schedule is not None:
            steps = self.schedule["timesteps"]
            diffs = np.array(steps) - self.total_timesteps
            idx = len(diffs[diffs <= 0]) - 1
            self.num_robots = self.schedule["num_robots"][idx]
            assert self.num_robots > 0, "Number of robots is 0!"
            self.num_cores = self.schedule["num_cores"][idx]
            self.num_obs = self.schedule["num_obstacles"][idx]
            self.min_start_goal_dis = self.schedule["min_start_goal_dis"][idx]
            print("\n======== training schedule ========")
            print("num of robots: ", self.num_robots)
            print("num of cores: ", self.num_cores)
            print("num of obstacles: ", self.num_obs)
            print("min start goal dis: ", self.min_start_goal_dis)
            print("======== training schedule ========\n")
        self.episode_timesteps = 0
        self.cores.clear()
        self.obstacles.clear()
        self.robots.clear()
        num_cores = self.num_cores
        num_obs = self.num_obs
        num_robots = 0
        iteration = 500
        while True:
            start = self.rd.uniform(low=2.0 * np.ones(2), high=np.array([self.width - 2.0, self.height - 2.0]))
            goal = self.rd.uniform(low=2.0 * np.ones(2), high=np.array([self.width - 2.0, self.height - 2.0]))
            iteration -= 1
            if self.check_start_and_goal(start, goal):
                rob = robot.Robot(seed=self.rd.randint(0, 5 * self.num_robots))
                rob.start = start
                rob.goal = goal
                self.reset_robot(rob)
                self.robots.append(rob)
                num_robots += 1
            if iteration == 0 or num_robots == self.num_robots:
                break
        if num_cores > 0:
            iteration = 500
            while True:
                center = self.rd.uniform(low=np.zeros(2), high=np.array([self.width, self.height]))
                direction = self.rd.binomial(1, 0.5)
                v_edge = self.rd.uniform(low=self.v_range[0], high=self.v_range[1])
                Gamma = 2 * np.pi * self.r * v_edge
                core = Core(center[0], center[1], direction, Gamma)
                iteration -= 1
                if self.check_core(core):
                    self.cores.append(core)
                    num_cores -= 1
                if iteration == 0 or num_cores == 0:
                    break
        if num_obs > 0:
            iteration = 500
            while True:
                center = self.rd.uniform(low=5.0 * np.ones(2), high=np.array([self.width - 5.0, self.height - 5.0]))
                r = self.rd.uniform(low=self.obs_r_range[0], high=self.obs_r_range[1])
                obs = Obstacle(center[0], center[1], r)
                iteration -= 1
                if self.check_obstacle(obs):
                    self.obstacles.append(obs)
                    num_obs -= 1
                if iteration == 0 or num_obs == 0:
                    break

    def reset_robot(self, rob):  # env.py:166-176
        rob.reach_goal = False
        rob.collision = False
        rob.deactivated = False
        rob.init_theta = self.rd.uniform(low=0.0, high=2 * np.pi)
        rob.init_velocity_r = np.array([0.0, 0.0, 0.0])
        rob.init_pos = 0.0
        rob.init_thrust = 0.0
        # cores are cleared at the top of reset(), so the current here is zero (env.py:98,175)
        current_v = np.zeros(3) if len(self.cores) == 0 else self.get_velocity(rob.start[0], rob.start[1])
        rob.reset_state(current_velocity=current_v)

    def check_all_deactivated(self):
        return all(rob.deactivated for rob in self.robots)

    def check_all_reach_goal(self):
        return all(rob.reach_goal for rob in self.robots)

    def check_any_collision(self):
        return any(rob.collision for rob in self.robots)

    def compute_COLREGs_penalty(self, rob):  # env.py:232-238
        penalty = 0.0
        if rob.apply_COLREGs:
            penalty += self.COLREGs_penalty * rob.phi
        return penalty

    def check_start_and_goal(self, start, goal):  # env.py:358-376
        if np.linalg.norm(goal - start) < self.min_start_goal_dis:
            return False
        for rob in self.robots:
            if np.linalg.norm(rob.start - start) <= self.clear_r:
                return False
            if np.linalg.norm(rob.goal - goal) <= self.clear_r:
                return False
        return True

    def check_core(self, core_j):  # env.py:378-418
        if core_j.x - self.r < 0.0 or core_j.x + self.r > self.width:
            return False
        if core_j.y - self.r < 0.0 or core_j.y + self.r > self.width:
            return False
        for rob in self.robots:
            core_pos = np.array([core_j.x, core_j.y])
            if np.linalg.norm(core_pos - rob.start) < self.r + self.clear_r:
                return False
            if np.linalg.norm(core_pos - rob.goal) < self.r + self.clear_r:
                return False
        for core_i in self.cores:
            dx = core_i.x - core_j.x
            dy = core_i.y - core_j.y
            dis = np.sqrt(dx * dx + dy * dy)
            if core_i.clockwise == core_j.clockwise:
                boundary_i = core_i.Gamma / (2 * np.pi * self.v_rel_max)
                boundary_j = core_j.Gamma / (2 * np.pi * self.v_rel_max)
                if dis < boundary_i + boundary_j:
                    return False
            else:
                Gamma_l = max(core_i.Gamma, core_j.Gamma)
                Gamma_s = min(core_i.Gamma, core_j.Gamma)
                v_1 = Gamma_l / (2 * np.pi * (dis - 2 * self.r))
                v_2 = Gamma_s / (2 * np.pi * self.r)
                if v_1 > self.p * v_2:
                    return False
        return True

    def check_obstacle(self, obs):  # env.py:420-456
        if obs.x - obs.r < 0.0 or obs.x + obs.r > self.width:
            return False
        if obs.y - obs.r < 0.0 or obs.y + obs.r > self.height:
            return False
        for rob in self.robots:
            obs_pos = np.array([obs.x, obs.y])
            if np.linalg.norm(obs_pos - rob.start) < obs.r + self.clear_r:
                return False
            if np.linalg.norm(obs_pos - rob.goal) < obs.r + self.clear_r:
                return False
        for core in self.cores:
            dx = core.x - obs.x
            dy = core.y - obs.y
            if np.sqrt(dx * dx + dy * dy) <= self.r + obs.r:
                return False
        for obstacle in self.obstacles:
            dx = obstacle.x - obs.x
            dy = obstacle.y - obs.y
            if np.sqrt(dx * dx + dy * dy) <= obstacle.r + obs.r:
                return False
        return True

    # ------------------------------------------------------------------ current field
    def get_velocity(self, x: float, y: float):
        """env.py:458-491, evaluated by the device kernel (asvrl_current_field)."""
        if len(self.cores) == 0:
            return np.zeros(3)
        cores = torch.tensor([[c.x, c.y, float(c.clockwise), c.Gamma] for c in self.cores], dtype=torch.float64,
                             device=self._device)
        xy = torch.tensor([[float(x), float(y)]], dtype=torch.float64, device=self._device)
        return current_field(cores, self.r, xy).cpu().numpy()[0]

    def compute_speed(self, Gamma: float, d: float):  # env.py:497-501
        if d <= self.r:
            return Gamma / (2 * np.pi * self.r * self.r) * d
        return Gamma / (2 * np.pi * d)

    # ------------------------------------------------------------------ device step
    def _params(self):
        """The launch's AsvParams: the first robot's vehicle / perception values and this env's rewards
        (robots with other values get a per-robot table, set_batch_params). Rebuilt only when those values
        change (params_from evaluates P = inv(A^T A) A^T with numpy: ~75 us, once per env step otherwise)."""
        rob = self.robots[0] if self.robots else None
        key = (rob.physics_signature() if rob is not None else None, self.env_key())
        cached = getattr(self, "_params_cache", None)
        if cached is None or cached[0] != key:
            cached = (key, _abi.params_from(rob, self))
            self._params_cache = cached
        return cached[1]

    def env_key(self):
        """The env-level launch parameters (rewards, episode limit, core radius): envs that share them can
        share one launch, whatever their robots' own parameters."""
        return (self.timestep_penalty, self.COLREGs_penalty, self.collision_penalty, self.goal_reward, self.r)

    def _ensure_batch(self, R, O, Cc):
        shape = (R, O, Cc)
        if self._batch is None or any(a > b for a, b in zip(shape, self._shape)):
            R2, O2, C2 = (max(a, b) for a, b in zip(shape, self._shape))
            self._batch = DeviceEnvBatch(1, max(R2, 1), max(O2, 1), max(C2, 1), device=self._device,
                                         obs64=True)
            self._shape = (self._batch.max_robots, self._batch.max_obs, self._batch.max_cores)
        return self._batch

    def _pack(self, actions, is_continuous_action, R, O, Cm):
        """Host SoA image of this env for one env-step launch, padded to (R robots, O obstacles,
        Cm cores): robot fields, flags, obstacles, cores, actions and the perception noise drawn
        from each active robot's RandomState in the reference's order (wamv.py:465-510): obstacles,
        then the other active robots, five draws per candidate."""
        n = len(self.robots)
        assert len(self.cores) <= Cm, "the batch was sized for fewer cores"
        rs = np.zeros((_abi.NUM_FIELDS, R))
        fl = np.zeros(R, np.uint8)
        for i, rob in enumerate(self.robots):
            rs[_abi.F_X:_abi.F_THETA + 1, i] = (rob.x, rob.y, rob.theta)
            rs[_abi.F_VR0:_abi.F_VR2 + 1, i] = rob.velocity_r
            rs[_abi.F_V0:_abi.F_V2 + 1, i] = rob.velocity
            rs[_abi.F_TL:_abi.F_RP + 1, i] = (rob.left_thrust, rob.right_thrust, rob.left_pos, rob.right_pos)
            rs[_abi.F_GX:_abi.F_GY + 1, i] = rob.goal
            rs[_abi.F_PHI, i] = rob.phi
            fl[i] = ((_abi.FLAG_DEACTIVATED if rob.deactivated else 0) | (_abi.FLAG_COLLISION if rob.collision else 0)
                     | (_abi.FLAG_REACH_GOAL if rob.reach_goal else 0))
        obst = np.zeros((max(O, 1), 3))
        for k, o in enumerate(self.obstacles):
            obst[k] = (o.x, o.y, o.r)
        cores = np.zeros((max(Cm, 1), 4))
        for k, c in enumerate(self.cores):
            cores[k] = (c.x, c.y, float(c.clockwise), c.Gamma)
        acts = np.zeros((R, 2))
        if actions is not None:
            for i, a in enumerate(actions):
                if a is None or self.robots[i].deactivated:
                    continue
                if is_continuous_action:
                    acts[i] = (float(a[0]), float(a[1]))
                else:
                    acts[i, 0] = int(a)
        noise = np.zeros((R, O + R, 5))
        for i, rob in enumerate(self.robots):
            if rob.deactivated:
                continue
            for k in range(len(self.obstacles)):
                noise[i, k] = rob.perception.draw_candidate_noise()
            for j, other in enumerate(self.robots):
                if other is rob or other.deactivated:
                    continue
                noise[i, O + j] = rob.perception.draw_candidate_noise()
        return dict(rs=rs, fl=fl, obst=obst, cores=cores, acts=acts, noise=noise, n=n, n_obs=len(self.obstacles),
                    n_cores=len(self.cores), ep_ts=int(self.episode_timesteps))

    def _apply(self, out, do_dynamics):
        """Write one launch's results (this env's slice) back into the Robot objects."""
        rs, fl = out["rs"], out["fl"]
        for i, rob in enumerate(self.robots):
            if do_dynamics and not rob.deactivated:
                rob.x, rob.y, rob.theta = float(rs[_abi.F_X, i]), float(rs[_abi.F_Y, i]), float(rs[_abi.F_THETA, i])
                rob.velocity_r = rs[_abi.F_VR0:_abi.F_VR2 + 1, i].copy()
                rob.velocity = rs[_abi.F_V0:_abi.F_V2 + 1, i].copy()
                rob.left_thrust, rob.right_thrust = float(rs[_abi.F_TL, i]), float(rs[_abi.F_TR, i])
            rob.collision = bool(fl[i] & _abi.FLAG_COLLISION)
            rob.reach_goal = bool(fl[i] & _abi.FLAG_REACH_GOAL)
            if not rob.deactivated:
                rob.apply_COLREGs = bool(fl[i] & _abi.FLAG_COLREGS)
                rob.phi = float(rs[_abi.F_PHI, i])

    def _device_step(self, actions, is_continuous_action, do_dynamics):
        n = len(self.robots)
        b = self._ensure_batch(n, len(self.obstacles), len(self.cores))
        return run_env_step(b, [self], [actions], is_continuous_action, do_dynamics)[0]

    def _observations(self, out):
        observations, collisions, reach_goals = [], [], []
        for i, rob in enumerate(self.robots):
            c = int(out["cnt"][i])
            if c < 0:
                obs = (None, None)
            else:
                o = out["obs64"][i]
                obs = ([float(v) for v in o[:7]], [[float(v) for v in o[7 + 5 * k:12 + 5 * k]] for k in range(c)])
            if self.is_eval_env:
                rob.observation_history.append([obs[0], obs[1]])
            observations.append(obs)
            collisions.append(rob.collision)
            reach_goals.append(rob.reach_goal)
        return observations, collisions, reach_goals

    def get_observations(self):
        """env.py:341-356 on the device (observation only, no dynamics)."""
        out = self._device_step(None, True, do_dynamics=False)
        return self._observations(out)

    def step(self, actions, is_continuous_action=True):
        assert len(actions) == len(self.robots), "Number of actions not equal number of robots!"
        assert self.check_all_reach_goal() is not True, "All robots reach goals, not actions are available!"
        active = [not rob.deactivated for rob in self.robots]
        out = self._device_step(actions, is_continuous_action, do_dynamics=True)
        return self._finish_step(actions, active, out)

    def _finish_step(self, actions, active, out):
        """env.step's bookkeeping after the launch (env.py:262-333): histories, observations,
        rewards, dones, infos, counters."""
        rewards = [0] * len(self.robots)
        if self.is_eval_env:  # env.py:262-269
            for i, rob in enumerate(self.robots):
                if active[i]:
                    rob.action_history.append(actions[i])
                    rob.trajectory.append(rob.trajectory_row())
        observations, _, _ = self._observations(out)
        dones = [False] * len(self.robots)
        infos = [{"state": "normal"}] * len(self.robots)
        for i, rob in enumerate(self.robots):
            code = int(out["info"][i])
            if code == _abi.INFO_ABSENT:
                raise RuntimeError("Robot being deactived can only be caused by collsion or reaching goal!")
            if active[i]:
                rewards[i] = float(out["reward"][i])
            dones[i] = code != _abi.INFO_NORMAL
            infos[i] = {"state": _abi.INFO_STRINGS[code]}
        self.episode_timesteps += 1
        self.total_timesteps += 1
        return observations, rewards, dones, infos

    # ------------------------------------------------------------------ eval configs (env.py:503-778)
    def reset_with_eval_config(self, eval_config):
        self.episode_timesteps = 0
        env = eval_config["env"]
        self.seed = env["seed"]
        self.rd = np.random.RandomState(self.seed)
        self.is_eval_env = env["is_eval_env"]
        self.width = env["width"]
        self.height = env["height"]
        self.r = env["r"]
        self.v_rel_max = env["v_rel_max"]
        self.p = env["p"]
        self.v_range = copy.deepcopy(env["v_range"])
        self.obs_r_range = copy.deepcopy(env["obs_r_range"])
        self.clear_r = env["clear_r"]
        self.angular_speed_max = env["angular_speed_max"]
        self.angular_speed_penalty = env["angular_speed_penalty"]
        self.timestep_penalty = env["timestep_penalty"]
        self.COLREGs_penalty = env["COLREGs_penalty"]
        self.collision_penalty = env["collision_penalty"]
        self.goal_reward = env["goal_reward"]
        self.cores.clear()
        for i in range(len(env["cores"]["positions"])):
            center = env["cores"]["positions"][i]
            self.cores.append(Core(center[0], center[1], env["cores"]["clockwise"][i], env["cores"]["Gamma"][i]))
        self.obstacles.clear()
        for i in range(len(env["obstacles"]["positions"])):
            center = env["obstacles"]["positions"][i]
            self.obstacles.append(Obstacle(center[0], center[1], env["obstacles"]["r"][i]))
        rb = eval_config["robots"]
        self.robots.clear()
        for i in range(env["num_robots"]):
            rob = robot.Robot(seed=self.rd.randint(0, 5 * self.num_robots))
            for k in ["dt", "N", "length", "width", "detect_r", "r", "goal_dis", "power_coefficient", "min_thrust",
                      "max_thrust"]:
                setattr(rob, k, rb[k][i])
            rob.left_thrust_change = np.array(rb["left_thrust_change"][i])
            rob.right_thrust_change = np.array(rb["right_thrust_change"][i])
            rob.compute_actions()
            for k in ["m", "Izz", "xDotU", "yDotV", "yDotR", "nDotR", "nDotV", "xU", "xUU", "yV", "yVV", "yR", "yRV",
                      "yVR", "yRR", "nR", "nRR", "nV", "nVV", "nRV", "nVR"]:
                setattr(rob, k, rb[k][i])
            rob.compute_constant_matrices()
            rob.start = np.array(rb["start"][i])
            rob.goal = np.array(rb["goal"][i])
            rob.init_theta = rb["init_theta"][i]
            rob.init_velocity_r = np.array(rb["init_velocity_r"][i])
            rob.init_left_pos = rb["init_left_pos"][i]
            rob.init_right_pos = rb["init_right_pos"][i]
            rob.init_left_thrust = rb["init_left_thrust"][i]
            rob.init_right_thrust = rb["init_right_thrust"][i]
            per = rb["perception"]
            for k in ["range", "angle", "max_obj_num", "pos_std", "vel_std", "r_kappa", "r_mean_ratio"]:
                setattr(rob.perception, k, per[k][i])
            current_v = self.get_velocity(rob.start[0], rob.start[1])
            rob.reset_state(current_velocity=current_v)
            self.robots.append(rob)
        return self.get_observations()

    def episode_data(self):
        ep = {"env": {}, "robots": {}}
        e = ep["env"]
        e["seed"] = self.seed
        e["is_eval_env"] = self.is_eval_env
        e["width"] = self.width
        e["height"] = self.height
        e["r"] = self.r
        e["v_rel_max"] = self.v_rel_max
        e["p"] = self.p
        e["v_range"] = copy.deepcopy(self.v_range)
        e["obs_r_range"] = copy.deepcopy(self.obs_r_range)
        e["clear_r"] = self.clear_r
        e["angular_speed_max"] = self.angular_speed_max
        e["angular_speed_penalty"] = self.angular_speed_penalty
        e["timestep_penalty"] = self.timestep_penalty
        e["COLREGs_penalty"] = self.COLREGs_penalty
        e["collision_penalty"] = self.collision_penalty
        e["goal_reward"] = self.goal_reward
        e["num_robots"] = self.num_robots
        e["cores"] = {"positions": [[c.x, c.y] for c in self.cores], "clockwise": [c.clockwise for c in self.cores],
                      "Gamma": [c.Gamma for c in self.cores]}
        e["obstacles"] = {"positions": [[o.x, o.y] for o in self.obstacles], "r": [o.r for o in self.obstacles]}
        r = ep["robots"]
        scalar = ["dt", "N", "length", "width", "detect_r", "r", "goal_dis", "power_coefficient", "min_thrust",
                  "max_thrust"]
        hydro = ["m", "Izz", "xDotU", "yDotV", "yDotR", "nDotR", "nDotV", "xU", "xUU", "yV", "yVV", "yR", "yRV",
                 "yVR", "yRR", "nR", "nRR", "nV", "nVV", "nRV", "nVR"]
        for k in scalar:
            r[k] = [getattr(rob, k) for rob in self.robots]
        r["left_thrust_change"] = [list(rob.left_thrust_change) for rob in self.robots]
        r["right_thrust_change"] = [list(rob.right_thrust_change) for rob in self.robots]
        for k in hydro:
            r[k] = [getattr(rob, k) for rob in self.robots]
        r["start"] = [list(rob.start) for rob in self.robots]
        r["goal"] = [list(rob.goal) for rob in self.robots]
        r["init_theta"] = [rob.init_theta for rob in self.robots]
        r["init_velocity_r"] = [list(rob.init_velocity_r) for rob in self.robots]
        for k in ["init_left_pos", "init_right_pos", "init_left_thrust", "init_right_thrust"]:
            r[k] = [getattr(rob, k) for rob in self.robots]
        r["perception"] = {k: [getattr(rob.perception, k) for rob in self.robots]
                           for k in ["range", "angle", "max_obj_num", "pos_std", "vel_std", "r_kappa", "r_mean_ratio"]}
        r["observation_history"] = [copy.deepcopy(rob.observation_history) for rob in self.robots]
        r["action_history"] = [copy.deepcopy(rob.action_history) for rob in self.robots]
        r["trajectory"] = [copy.deepcopy(rob.trajectory) for rob in self.robots]
        return ep

    def save_episode(self, filename):
        with open(filename, "w") as f:
            json.dump(self.episode_data(), f)


def set_batch_params(batch, envs):
    """The launch parameters of `envs` on `batch` (env e in slots [e*R, (e+1)*R)): one AsvParams when
    every robot shares its vehicle / perception values, else a per-robot table as well
    (reset_with_eval_config gives each robot its own dt, N, m, Izz, hydrodynamic coefficients, thrust
    limits, radius, goal distance and perception sigma / kappa, env.py:553-607). The envs share their
    env-level values (env_key)."""
    assert len({env.env_key() for env in envs}) <= 1, "one launch takes one set of env-level parameters"
    batch.params = envs[0]._params() if envs else _abi.params_from()
    sigs = {rob.physics_signature() for env in envs for rob in env.robots}
    if len(sigs) <= 1:
        batch.set_robot_params(None)
        return
    R = batch.max_robots
    table = [batch.params] * (batch.n_envs * R)
    for e, env in enumerate(envs):
        for i, rob in enumerate(env.robots):
            table[e * R + i] = _abi.params_from(rob, env)
    batch.set_robot_params(table)


class _StepStage:
    """Pinned host images of one DeviceEnvBatch's per-step inputs and outputs (run_env_step): the inputs are
    packed into them and copied up without a host wait, the outputs copied down behind the step launch with one
    synchronisation for all of them (instead of a blocking pageable copy per array)."""

    @classmethod
    def of(cls, batch):
        st = getattr(batch, "_step_stage", None)
        if st is None:
            st = batch._step_stage = cls(batch)
        return st

    def __init__(self, batch):
        dev, E, R, O, Cm = batch.device, batch.n_envs, batch.max_robots, batch.max_obs, batch.max_cores
        NT = E * R

        def pin(shape, dtype):
            return torch.zeros(shape, dtype=dtype, pin_memory=True)
        self.rs = pin((_abi.NUM_FIELDS, NT), torch.float64)
        self.fl = pin((NT,), torch.uint8)
        self.acts = pin((NT, 2), torch.float64)
        self.noise = pin((NT, O + R, 5), torch.float64)
        self.cnt = pin((4, E), torch.int32)
        self.obst = pin((E, max(O, 1), 3), torch.float64)
        self.cores = pin((E, max(Cm, 1), 4), torch.float64)
        self.acts_dev = torch.zeros((NT, 2), dtype=torch.float64, device=dev)
        self.noise_dev = torch.zeros((NT, O + R, 5), dtype=torch.float64, device=dev)
        self.out = {k: torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
                    for k, t in (("rs", batch.rs), ("fl", batch.rflags), ("obs64", batch.obs64), ("cnt", batch.obj_cnt),
                                 ("reward", batch.reward), ("info", batch.info))}

    def fill(self, packs, R):
        rs, fl, acts, noise = self.rs.numpy(), self.fl.numpy(), self.acts.numpy(), self.noise.numpy()
        cnt, obst, cores = self.cnt.numpy(), self.obst.numpy(), self.cores.numpy()
        for a in (rs, fl, acts, noise, cnt, obst, cores):
            a.fill(0)
        for e, pk in enumerate(packs):
            sl = slice(e * R, (e + 1) * R)
            rs[:, sl], fl[sl], acts[sl], noise[sl] = pk["rs"], pk["fl"], pk["acts"], pk["noise"]
            cnt[:, e] = (pk["n"], pk["n_obs"], pk["n_cores"], pk["ep_ts"])
            obst[e], cores[e] = pk["obst"], pk["cores"]

    def upload(self, batch):
        for dst, src in ((batch.rs, self.rs), (batch.rflags, self.fl), (batch.n_robots, self.cnt[0]),
                         (batch.n_obs, self.cnt[1]), (batch.n_cores, self.cnt[2]), (batch.ep_ts, self.cnt[3]),
                         (batch.obstacles, self.obst), (batch.cores, self.cores), (self.acts_dev, self.acts),
                         (self.noise_dev, self.noise)):
            dst.copy_(src, non_blocking=True)

    def download(self, batch):
        src = dict(rs=batch.rs, fl=batch.rflags, obs64=batch.obs64, cnt=batch.obj_cnt, reward=batch.reward,
                   info=batch.info)
        for k, t in src.items():
            self.out[k].copy_(t, non_blocking=True)
        torch.cuda.current_stream(batch.device).synchronize()
        # copies: the pinned images are refilled by the next step
        return {k: v.numpy().copy() for k, v in self.out.items()}


def run_env_step(batch, envs, actions_list, is_continuous_action, do_dynamics):
    """One asvrl_env_step launch over several MarineNavEnv3 instances that share their env-level
    parameters: env e occupies slots [e*R, (e+1)*R) of `batch` (a DeviceEnvBatch with n_envs >= len(envs)
    and room for every env's robots, obstacles and cores); robots with their own vehicle / perception
    parameters go through the per-robot table (set_batch_params). Each env's noise comes from its own
    robots' RandomStates, so the results equal stepping the envs one at a time. Returns the
    per-env output slices (host arrays) after writing them back into the robots."""
    set_batch_params(batch, envs)
    E, R, O, Cm = len(envs), batch.max_robots, batch.max_obs, batch.max_cores
    packs = [env._pack(a, is_continuous_action, R, O, Cm) for env, a in zip(envs, actions_list)]
    st = _StepStage.of(batch)
    st.fill(packs, R)
    st.upload(batch)   # pinned host images -> the batch, no host wait
    batch.step(st.acts_dev, is_continuous=is_continuous_action, noise=st.noise_dev, do_dynamics=do_dynamics)
    full = st.download(batch)   # one wait for every output
    outs = []
    for e, env in enumerate(envs):
        sl = slice(e * R, (e + 1) * R)
        out = dict(rs=full["rs"][:, sl], fl=full["fl"][sl], obs64=full["obs64"][sl], cnt=full["cnt"][sl],
                   reward=full["reward"][sl], info=full["info"][sl])
        env._apply(out, do_dynamics)
        outs.append(out)
    return outs
