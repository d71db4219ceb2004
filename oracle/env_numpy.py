"""Per-robot NumPy restatement of MarineNavEnv3 (TEST / BASELINE INFRASTRUCTURE ONLY).

The reference's CPU path kept in its own shape: one Python object per vessel, np.matrix algebra per
Fossen substep, a Python loop over the candidate objects with per-vessel numpy.random.RandomState
perception noise, heapq top-5 -- i.e. the cost structure SURVEY.md 8(d) asks the CPU baseline to have
("the faithful per-robot NumPy restatement ... P processes, OMP_NUM_THREADS=1"). Written against:

  Vessel.substep            wamv.py:201-231  (update_velocity + update_state, theta wrap, thrust update)
  Vessel._fossen            wamv.py:233-279  (compute_motion: C_RB, C_A, D, D_n, tau, inv(A^T A) A^T b)
  Vessel.sense              wamv.py:436-529  (perception_output, check_detection / collision, nsmallest)
  Vessel._colregs           wamv.py:324-434  (ego->vehicle frame, crossing / head-on zones, turn angle)
  NpMarineEnv.reset         env.py:72-176    (rejection sampling of starts/goals, cores, obstacles)
  NpMarineEnv.step          env.py:240-333   (10 substeps, rewards, observations, dones / infos)
  NpMarineEnv.current       env.py:458-501   (vortex current, cores by distance)

Pinned on CPU by tests/test_env_numpy_cpu.py to the reference's own captures: every F3 trace step
(tests/golden/env_traces.npz, the recorded noise injected) within 1e-12 with masks exact, and every F7
reset (env_reset.npz: layouts, perception seeds, observations and the RandomState position after it)
exactly. bench.py's cpu_baseline times it as the reference-style leg (kind "port"); the product never
imports it.
"""
import heapq

import numpy as np

TWO_PI = 2 * np.pi


class Vessel:
    """One WAM-V (wamv.py:43-145 defaults): state in plain attributes, dynamics on np.matrix."""

    def __init__(self, seed):
        self.dt, self.N = 0.05, 10
        self.perception_seed = seed
        self.rd = np.random.RandomState(seed)
        self.range, self.angle, self.max_obj = 20.0, 2 * np.pi, 5
        self.pos_std = self.vel_std = 0.05
        self.kappa, self.r_mean_ratio = 1.0, 0.8
        self.length, self.width = 5.0, 2.5
        self.r = 0.5 * np.sqrt(self.length ** 2 + self.width ** 2)
        self.goal_dis = 2.0
        self.min_thrust, self.max_thrust = -500.0, 1000.0
        steps = np.array([0.0, -500.0, -1000.0, 500.0, 1000.0])
        self.discrete = [(a, b) for a in steps for b in steps]
        self.m, self.Izz = 400, 450
        self.xDotU, self.yDotV, self.yDotR, self.nDotR, self.nDotV = 20, 0, 0, -980, 0
        self.xU, self.xUU, self.yV, self.yVV, self.yR, self.yRV, self.yVR, self.yRR = -100, -150, -100, -150, 0, 0, 0, 0
        self.nR, self.nRR, self.nV, self.nVV, self.nRV, self.nVR = -980, -950, 0, 0, 0, 0
        self.M_RB = np.matrix([[self.m, 0.0, 0.0], [0.0, self.m, 0.0], [0.0, 0.0, self.Izz]])
        self.M_A = -1.0 * np.matrix([[self.xDotU, 0.0, 0.0], [0.0, self.yDotV, self.yDotR], [0.0, self.nDotV, self.nDotR]])
        self.D = -1.0 * np.matrix([[self.xU, 0.0, 0.0], [0.0, self.yV, self.yR], [0.0, self.nV, self.nR]])
        self.start = self.goal = None
        self.x = self.y = self.theta = None
        self.velocity_r = self.velocity = None
        self.left_pos = self.right_pos = 0.0
        self.left_thrust = self.right_thrust = 0.0
        self.collision = self.reach_goal = self.deactivated = False
        self.apply_COLREGs, self.phi = False, None

    # ---------------------------------------------------------------- frames
    def _rot(self):
        c, s = np.cos(self.theta), np.sin(self.theta)
        return np.matrix([[c, -s], [s, c]])

    def to_body(self, v, is_vector=True):
        """world -> vessel frame of a 2-vector (wamv.py:305-322)."""
        R = self._rot()
        Rt = np.transpose(R)
        col = np.reshape(v, (2, 1))
        out = Rt * col if is_vector else Rt * col + (-Rt * np.matrix([[self.x], [self.y]]))
        out.resize((2,))
        return np.array(out)

    def goal_distance(self):
        return np.linalg.norm(self.goal - np.array([self.x, self.y]))

    # ---------------------------------------------------------------- dynamics
    def place(self, current):
        self.x, self.y = self.start[0], self.start[1]
        self.theta = self.init_theta
        self.velocity_r = np.array([0.0, 0.0, 0.0])
        self.velocity = self.velocity_r + current
        self.left_pos = self.right_pos = 0.0
        self.left_thrust = self.right_thrust = 0.0

    def substep(self, action, current, first, continuous):
        self.velocity = self.velocity_r + current
        step = self.velocity * self.dt
        self.x += step[0]
        self.y += step[1]
        self.theta += step[2]
        while self.theta < 0.0:
            self.theta += TWO_PI
        while self.theta >= TWO_PI:
            self.theta -= TWO_PI
        if first:
            if continuous:
                dl, dr = action[0] * 1000.0, action[1] * 1000.0
            else:
                dl, dr = self.discrete[action]
            self.left_thrust = np.clip(self.left_thrust + dl * self.dt * self.N, self.min_thrust, self.max_thrust)
            self.right_thrust = np.clip(self.right_thrust + dr * self.dt * self.N, self.min_thrust, self.max_thrust)
        self._fossen()

    def _fossen(self):
        vrb = self.to_body(self.velocity_r[:2])
        vb = self.to_body(self.velocity[:2])
        u_r, v_r, u, v, r = vrb[0], vrb[1], vb[0], vb[1], self.velocity[2]
        m = self.m
        C_RB = np.matrix([[0.0, -m * r, 0.0], [m * r, 0.0, 0.0], [0.0, 0.0, 0.0]])
        cross = self.yDotV * v_r + self.yDotR * r
        C_A = np.matrix([[0.0, 0.0, cross], [0.0, 0.0, -self.xDotU * u_r],
                         [-self.yDotV * v_r - self.yDotR * r, self.xDotU * u_r, 0.0]])
        au, av, ar = np.abs(u_r), np.abs(v_r), np.abs(r)
        D_n = -1.0 * np.matrix([[self.xUU * au, 0.0, 0.0],
                                [0.0, self.yVV * av + self.yRV * ar, self.yVR * av + self.yRR * ar],
                                [0.0, self.nVV * av + self.nRV * ar, self.nVR * av + self.nRR * ar]])
        Nmat = C_A + self.D + D_n
        fxl, fyl = self.left_thrust * np.cos(self.left_pos), self.left_thrust * np.sin(self.left_pos)
        fxr, fyr = self.right_thrust * np.cos(self.right_pos), self.right_thrust * np.sin(self.right_pos)
        tau = np.matrix([[fxl + fxr], [fyl + fyr],
                         [fxl * self.width / 2 + -fyl * self.length / 2 + -fxr * self.width / 2 + -fyr * self.length / 2]])
        A = self.M_RB + self.M_A
        V = np.matrix([[u, v, r]]).transpose()
        Vr = np.matrix([[u_r, v_r, r]]).transpose()
        b = -C_RB * V - Nmat * Vr + tau
        acc = np.linalg.inv(A.transpose() * A) * A.transpose() * b
        Vr += acc * self.dt
        Vr[:2, :] = self._rot() * Vr[:2, :]
        self.velocity_r = np.squeeze(np.array(Vr))

    # ---------------------------------------------------------------- perception
    def _draw(self, px, py, vx, vy, r, noise):
        """Noisy position, velocity, radius (wamv.py:27-40): five draws from this vessel's own RandomState in
        the reference's order, or the recorded draws `noise` = (n_px, n_py, n_vx, n_vy, vonmises)."""
        if noise is None:
            npx, npy = self.rd.normal(0, self.pos_std), self.rd.normal(0, self.pos_std)
            nvx, nvy = self.rd.normal(0, self.vel_std), self.rd.normal(0, self.vel_std)
            vm = self.rd.vonmises(0, self.kappa)
        else:
            npx, npy, nvx, nvy, vm = noise
        r_obs = self.r_mean_ratio * r + (1 - self.r_mean_ratio) * vm / np.pi * r
        return px + npx, py + npy, vx + nvx, vy + nvy, r_obs

    def _seen(self, ox, oy, orad):
        p = self.to_body(np.array([ox, oy]), False)
        if np.linalg.norm(p) > self.range + orad:
            return False
        ang = np.arctan2(p[1], p[0])
        return not (ang < -0.5 * self.angle or ang > 0.5 * self.angle)

    def sense(self, obstacles, fleet, noise=None, slot0=None):
        """perception_output (wamv.py:436-529). noise: None (draw from this vessel's RandomState) or the
        recorded draws [candidate][5]: obstacle k at row k, fleet vessel j at row slot0 + j."""
        if self.deactivated:
            return (None, None), self.collision, self.reach_goal
        vb = self.to_body(self.velocity[:2])
        gb = self.to_body(self.goal, False)
        own = list(np.concatenate((gb, vb)))
        own += [self.velocity[2], self.left_thrust, self.right_thrust]
        if self.goal_distance() <= self.goal_dis:
            self.reach_goal = True
        found = []
        cands = [(k, o.x, o.y, 0.0, 0.0, o.r) for k, o in enumerate(obstacles)]
        off = len(obstacles) if slot0 is None else slot0
        cands += [(off + j, v.x, v.y, v.velocity[0], v.velocity[1], v.r) for j, v in enumerate(fleet)
                  if v is not self and not v.deactivated]
        for k, tx, ty, tvx, tvy, tr in cands:
            px, py, vx, vy, ro = self._draw(tx, ty, tvx, tvy, tr, None if noise is None else noise[k])
            if not self._seen(px, py, ro):
                continue
            if not self.collision and np.sqrt((self.x - tx) ** 2 + (self.y - ty) ** 2) - tr - self.r <= 0.0:
                self.collision = True
            pb = self.to_body(np.array([px, py]), False)
            vvb = self.to_body(np.array([vx, vy]))
            found.append([pb[0], pb[1], vvb[0], vvb[1], ro])
        kept = heapq.nsmallest(self.max_obj, found, key=lambda o: np.sqrt(o[0] ** 2 + o[1] ** 2) - o[4] - self.r)
        self.apply_COLREGs = False
        for o in kept:
            if self._colregs(o):
                self.apply_COLREGs = True
                break
        return (own, [list(o) for o in kept]), self.collision, self.reach_goal

    # ---------------------------------------------------------------- COLREGs
    @staticmethod
    def _wrap(a):
        while a < -np.pi:
            a += TWO_PI
        while a >= np.pi:
            a -= TWO_PI
        return a

    def _colregs(self, o):
        if np.linalg.norm(np.array(o[2:4])) < 0.5:
            return False
        ev = self.to_body(self.velocity[:2])
        if np.linalg.norm(ev) < 0.5:
            return False
        va = np.arctan2(o[3], o[2])
        R = np.matrix([[np.cos(va), -np.sin(va)], [np.sin(va), np.cos(va)]])
        pp = -np.transpose(R) * np.matrix([[o[0]], [o[1]]])
        pp.resize((2,))
        vp = np.transpose(R) * np.matrix([[ev[0]], [ev[1]]])
        vp.resize((2,))
        pp, vp = np.array(pp), np.array(vp)
        vang = np.arctan2(vp[1], vp[0])
        # left crossing zone (wamv.py:344-362)
        in_box = (-9.0 <= pp[0] <= 12.0) and (-17.0 <= pp[1] <= 0.0)
        tri = (pp[1] - (-7.0)) > (-7.0 / 12.0) * (pp[0] - 12.0)
        crossing = in_box and not tri and (np.pi / 4 <= vang <= 3 * np.pi / 4)
        # head-on zone (wamv.py:364-377)
        head_on = (0.0 <= pp[0] <= 17.0) and (-4.5 <= pp[1] <= 4.5) and np.abs(vang) > 3 * np.pi / 4
        if not (crossing or head_on):
            return False
        ev_ang = np.arctan2(ev[1], ev[0])
        op_ang = np.arctan2(o[1], o[0])
        base = o[4] + 1.0
        dist = np.linalg.norm(np.array(o[:2]))
        a1 = np.arcsin(base / dist)
        a2 = np.arctan2(self.r, np.sqrt(dist ** 2 - base ** 2))
        self.phi = self._wrap(self._wrap(op_ang + a1 + a2) - ev_ang)
        return bool(self.phi > 0)


class Buoy:
    def __init__(self, x, y, r):
        self.x, self.y, self.r = x, y, r


class Vortex:
    def __init__(self, x, y, clockwise, gamma):
        self.x, self.y, self.clockwise, self.Gamma = x, y, clockwise, gamma


class NpMarineEnv:
    """MarineNavEnv3 (env.py:24-501) over Vessel objects; the trainer's deactivation is the caller's."""

    def __init__(self, seed=0, num_robots=5, num_cores=0, num_obs=4, min_start_goal_dis=40.0, width=55.0):
        self.rd = np.random.RandomState(seed)
        self.width = self.height = width
        self.core_r, self.v_rel_max, self.p, self.v_range = 0.5, 1.0, 0.8, (3, 3)
        self.obs_r_range, self.clear_r = (1, 1), 10.0
        self.timestep_penalty, self.COLREGs_penalty = -0.1, -0.1
        self.collision_penalty, self.goal_reward = -5.0, 10.0
        self.num_robots, self.num_cores, self.num_obs = num_robots, num_cores, num_obs
        self.min_start_goal_dis = min_start_goal_dis
        # env.py:56-58: the constructor's own vessels consume seeds from the env stream (6 by default)
        for _ in range(6):
            self.rd.randint(0, 5 * 6)
        self.robots, self.cores, self.obstacles = [], [], []
        self.episode_timesteps = 0

    # ---------------------------------------------------------------- current (env.py:458-501)
    def current(self, x, y):
        if not self.cores:
            return np.zeros(3)
        q = np.array([x, y])
        d = np.array([np.linalg.norm(np.array([c.x, c.y]) - q) for c in self.cores])
        order = np.argsort(d, kind="stable")
        vel = np.zeros((2, 1))
        for i in order:
            c = self.cores[i]
            radial = np.matrix([[c.x - x], [c.y - y]])
            dis = np.linalg.norm(radial)
            radial /= dis
            rot = np.matrix([[0., -1.], [1., 0]]) if c.clockwise else np.matrix([[0., 1.], [-1., 0]])
            speed = c.Gamma / (2 * np.pi * self.core_r * self.core_r) * dis if dis <= self.core_r \
                else c.Gamma / (2 * np.pi * dis)
            vel += rot * radial * speed
        return np.array([vel[0, 0], vel[1, 0], 0.0])

    # ---------------------------------------------------------------- reset (env.py:72-176, 358-456)
    def _start_goal_ok(self, s, g):
        if np.linalg.norm(g - s) < self.min_start_goal_dis:
            return False
        return all(np.linalg.norm(v.start - s) > self.clear_r and np.linalg.norm(v.goal - g) > self.clear_r
                   for v in self.robots)

    def _core_ok(self, c):
        r = self.core_r
        if c.x - r < 0.0 or c.x + r > self.width or c.y - r < 0.0 or c.y + r > self.width:
            return False
        p = np.array([c.x, c.y])
        for v in self.robots:
            if np.linalg.norm(p - v.start) < r + self.clear_r or np.linalg.norm(p - v.goal) < r + self.clear_r:
                return False
        for o in self.cores:
            dx, dy = o.x - c.x, o.y - c.y
            dis = np.sqrt(dx * dx + dy * dy)
            if o.clockwise == c.clockwise:
                if dis < o.Gamma / (2 * np.pi * self.v_rel_max) + c.Gamma / (2 * np.pi * self.v_rel_max):
                    return False
            else:
                big, small = max(o.Gamma, c.Gamma), min(o.Gamma, c.Gamma)
                if big / (2 * np.pi * (dis - 2 * r)) > self.p * (small / (2 * np.pi * r)):
                    return False
        return True

    def _buoy_ok(self, b):
        if b.x - b.r < 0.0 or b.x + b.r > self.width or b.y - b.r < 0.0 or b.y + b.r > self.height:
            return False
        p = np.array([b.x, b.y])
        for v in self.robots:
            if np.linalg.norm(p - v.start) < b.r + self.clear_r or np.linalg.norm(p - v.goal) < b.r + self.clear_r:
                return False
        for c in self.cores:
            if np.sqrt((c.x - b.x) ** 2 + (c.y - b.y) ** 2) <= self.core_r + b.r:
                return False
        for o in self.obstacles:
            if np.sqrt((o.x - b.x) ** 2 + (o.y - b.y) ** 2) <= o.r + b.r:
                return False
        return True

    def reset(self):
        self.episode_timesteps = 0
        self.robots, self.cores, self.obstacles = [], [], []
        lo, hi = 2.0 * np.ones(2), np.array([self.width - 2.0, self.height - 2.0])
        tries = 500
        while True:
            s, g = self.rd.uniform(low=lo, high=hi), self.rd.uniform(low=lo, high=hi)
            tries -= 1
            if self._start_goal_ok(s, g):
                v = Vessel(self.rd.randint(0, 5 * self.num_robots))
                v.start, v.goal = s, g
                v.init_theta = self.rd.uniform(low=0.0, high=2 * np.pi)
                v.place(self.current(s[0], s[1]))
                self.robots.append(v)
            if tries == 0 or len(self.robots) == self.num_robots:
                break
        left = self.num_cores
        if left > 0:
            tries = 500
            while True:
                ctr = self.rd.uniform(low=np.zeros(2), high=np.array([self.width, self.height]))
                cw = self.rd.binomial(1, 0.5)
                vedge = self.rd.uniform(low=self.v_range[0], high=self.v_range[1])
                c = Vortex(ctr[0], ctr[1], cw, 2 * np.pi * self.core_r * vedge)
                tries -= 1
                if self._core_ok(c):
                    self.cores.append(c)
                    left -= 1
                if tries == 0 or left == 0:
                    break
        left = self.num_obs
        if left > 0:
            tries = 500
            while True:
                ctr = self.rd.uniform(low=5.0 * np.ones(2), high=np.array([self.width - 5.0, self.height - 5.0]))
                b = Buoy(ctr[0], ctr[1], self.rd.uniform(low=self.obs_r_range[0], high=self.obs_r_range[1]))
                tries -= 1
                if self._buoy_ok(b):
                    self.obstacles.append(b)
                    left -= 1
                if tries == 0 or left == 0:
                    break
        return self.observe()

    # ---------------------------------------------------------------- step (env.py:240-356)
    def observe(self, noise=None, slot0=None):
        out = [v.sense(self.obstacles, self.robots, None if noise is None else noise[i], slot0)
               for i, v in enumerate(self.robots)]
        return [o[0] for o in out], [o[1] for o in out], [o[2] for o in out]

    def step(self, actions, continuous=True, noise=None, slot0=None):
        rewards = [0] * len(self.robots)
        for i, a in enumerate(actions):
            v = self.robots[i]
            if v.deactivated:
                continue
            before = v.goal_distance()
            for k in range(v.N):
                v.substep(a, self.current(v.x, v.y), k == 0, continuous)
            rewards[i] += self.timestep_penalty
            rewards[i] += before - v.goal_distance()
        obs, coll, reach = self.observe(noise, slot0)
        dones, infos = [False] * len(self.robots), [None] * len(self.robots)
        for i, v in enumerate(self.robots):
            if v.deactivated:
                dones[i] = True
                if v.collision:
                    infos[i] = "deactivated after collision"
                elif v.reach_goal:
                    infos[i] = "deactivated after reaching goal"
                else:
                    raise RuntimeError("Robot being deactived can only be caused by collsion or reaching goal!")
                continue
            if v.apply_COLREGs:
                rewards[i] += self.COLREGs_penalty * v.phi
            if self.episode_timesteps >= 1000:
                dones[i], infos[i] = True, "too long episode"
            elif coll[i]:
                rewards[i] += self.collision_penalty
                dones[i], infos[i] = True, "collision"
            elif reach[i]:
                rewards[i] += self.goal_reward
                dones[i], infos[i] = True, "reach goal"
            else:
                infos[i] = "normal"
        self.episode_timesteps += 1
        return obs, rewards, dones, infos


def rollout(seconds, seed=0, num_robots=5, num_obs=4, min_start_goal_dis=40.0):
    """The reference's training loop shape on one env for `seconds` of wall time (trainer.py:142-172 without
    the agent): uniform(-1, 1) actions, trainer deactivation on collision / goal, a reset when every vessel is
    off or the episode reaches 1000 steps. Returns (env.step calls, elapsed seconds)."""
    import time
    import warnings
    warnings.simplefilter("ignore", PendingDeprecationWarning)   # the reference runs with -W ignore
    env = NpMarineEnv(seed=seed, num_robots=num_robots, num_obs=num_obs, min_start_goal_dis=min_start_goal_dis)
    env.reset()
    act = np.random.RandomState(seed + 1)
    n, t0 = 0, time.perf_counter()
    while True:
        env.step([act.uniform(-1.0, 1.0, 2) for _ in env.robots], True)
        n += 1
        for v in env.robots:
            if not v.deactivated and (v.collision or v.reach_goal):
                v.deactivated = True
        if all(v.deactivated for v in env.robots) or env.episode_timesteps >= 1000:
            env.reset()
        if n % 16 == 0 and time.perf_counter() - t0 >= seconds:
            return n, time.perf_counter() - t0
