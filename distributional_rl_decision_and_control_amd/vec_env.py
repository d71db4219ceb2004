"""VecMarineNavEnv -- E independent MarineNavEnv3 scenes resident in HBM.

The batched counterpart of rfarl's single MarineNavEnv3 (env.py:24): reset, step and the
Trainer's per-step bookkeeping (trainer.py:157-172: deactivate on collision/goal, episode
end at 1000 steps or all deactivated, discounted return) run on the device with no host
round trip. Noise and resets use counter-based Philox streams keyed by (seed, env, robot,
step), so runs are reproducible and rank-independent streams come from `seed + rank`.
The curriculum schedule (env.py:75-94) is applied per reset from the global step count.
"""
import numpy as np
import torch

from . import _abi
from .device_env import DeviceEnvBatch, reset_cfg


class VecMarineNavEnv:
    def __init__(self, n_envs, num_robots=5, num_obs=4, num_cores=0, min_start_goal_dis=40.0, width=55.0,
                 height=None, schedule=None, seed=0, device="cuda", is_continuous=True, gamma=0.99,
                 max_robots=None, max_obs=None, max_cores=None):
        self.n_envs = int(n_envs)
        self.schedule = schedule
        self.max_groups = 0   # step kernel workgroups per launch (0: one launch; see _launch)
        R = max_robots or (max(schedule["num_robots"]) if schedule else num_robots)
        O = max_obs if max_obs is not None else (max(schedule["num_obstacles"]) if schedule else num_obs)
        Cc = max_cores if max_cores is not None else (max(schedule["num_cores"]) if schedule else num_cores)
        self.batch = DeviceEnvBatch(self.n_envs, R, O, Cc, device=device)
        self.max_robots = R
        self.device = self.batch.device
        self.seed = int(seed)
        self.is_continuous = is_continuous
        self.gamma = gamma
        self.width = float(width)
        self.height = float(height if height is not None else width)
        self.cfg = reset_cfg(num_robots, num_obs, num_cores, min_start_goal_dis, self.width, self.height)
        NT = self.n_envs * R
        self.obs = [torch.zeros((NT, _abi.OBS_DIM), dtype=torch.float32, device=self.device) for _ in range(2)]
        self.cnt = [torch.full((NT,), -1, dtype=torch.int8, device=self.device) for _ in range(2)]
        self.counter = torch.zeros(1, dtype=torch.int64, device=self.device)  # steps taken (device)
        self.total_timesteps = 0

    # obs[p] is the state the agent acts on and obs[1 - p] receives the next state. advance_device()
    # flips the parity p (swap=True: no copy; a captured HIP graph of an EVEN number of iterations then
    # ends on the parity it started from) or copies 1 -> 0 (swap=False: any graph sees the same buffers).
    swap = False
    _p = 0
    # auto_reset in one launch (asvrl_env_reset_observe) instead of the reset sampler + a masked observation
    # pass over every env; False: the two launches (A/B, tests/test_env_kernel_gpu.py)
    fused_reset = True

    @property
    def obs_cur(self):
        return self.obs[self._p]

    @property
    def cnt_cur(self):
        return self.cnt[self._p]

    @property
    def obs_next(self):
        return self.obs[1 - self._p]

    @property
    def cnt_next(self):
        return self.cnt[1 - self._p]

    def apply_schedule(self, total_timesteps):
        """Curriculum stage for the next resets (env.py:75-94)."""
        if self.schedule is None:
            return
        steps = np.array(self.schedule["timesteps"])
        idx = len(steps[steps - total_timesteps <= 0]) - 1
        self.cfg = reset_cfg(self.schedule["num_robots"][idx], self.schedule["num_obstacles"][idx],
                             self.schedule["num_cores"][idx], self.schedule["min_start_goal_dis"][idx], self.width,
                             self.height)

    def reset(self):
        """Reset every env (device rejection sampler) and observe into obs_cur."""
        b = self.batch
        b.reset(self.cfg, None, seed=self.seed, counter=0x40000000, counter_dev=self.counter)
        b.step(None, do_dynamics=False, seed=self.seed, counter=0x80000000, counter_dev=self.counter,
               fast_noise=True, obs=self.obs_cur, obj_cnt=self.cnt_cur)
        return self.obs_cur

    def step(self, actions):
        """One MarineNavEnv3.step on all envs + trainer bookkeeping. actions f64 [E*R, 2].
        Writes obs_next / cnt_next, batch.reward / done / info / env_done."""
        self.batch.step(actions, is_continuous=self.is_continuous, trainer_deactivate=True, seed=self.seed,
                        counter=0, counter_dev=self.counter, gamma=self.gamma, obs=self.obs_next,
                        obj_cnt=self.cnt_next, fast_noise=True,   # f32 Philox draws (noise_mode 2)
                        launch=self._launch())

    def _launch(self):
        """The step kernel's shape: automatic, or launches of at most `max_groups` workgroups one after another
        (the rollout's share of the chip beside a concurrent learner; results do not depend on it)."""
        return (0, 0, 0, self.max_groups) if self.max_groups > 0 else None

    def auto_reset(self, counted=False, events=None):
        """Reset the envs whose episode ended in the last step and observe them into obs_next.
        counted: the step counter was already incremented for this step (by the replay push launch);
        the draws are keyed as if it had not been. events: three HIP events recorded on the current
        stream before the reset, between the reset and the observation pass, and after it (bench.py; with
        fused_reset only the first two)."""
        b = self.batch
        d = 1 if counted else 0
        if events is not None:
            events[0].record()
        # the one-launch form takes no workgroup cap (one wave-per-env workgroup per env): with max_groups set (the
        # --env-groups A/B knob) the reset keeps the capped two-launch form, so the cap applies to every env pass
        if self.fused_reset and b.robot_params is None and self.max_groups <= 0:
            # one launch: reset + the reset observation of the ended envs only (asvrl_env_reset_observe)
            b.reset_observe(self.cfg, b.env_done, seed=self.seed, counter=0x40000000 - d, counter_dev=self.counter,
                            obs_counter=0x80000000 - d, obs=self.obs_next, obj_cnt=self.cnt_next)
            if events is not None:
                events[1].record()   # (events[2] unused: there is no second launch)
            return
        b.reset(self.cfg, b.env_done, seed=self.seed, counter=0x40000000 - d, counter_dev=self.counter)
        if events is not None:
            events[1].record()
        b.step(None, do_dynamics=False, seed=self.seed, counter=0x80000000 - d, counter_dev=self.counter,
               fast_noise=True, env_mask=b.env_done, obs=self.obs_next, obj_cnt=self.cnt_next, launch=self._launch())
        if events is not None:
            events[2].record()

    def advance_device(self, counted=False):
        if self.swap:
            self._p ^= 1
        else:
            self.obs[0].copy_(self.obs[1])
            self.cnt[0].copy_(self.cnt[1])
        if not counted:
            self.counter += 1

    def advance_host(self):
        self.total_timesteps += self.n_envs

    def episode_stats(self):
        """(mean return, success rate, collision rate, timeout rate, finished episodes)."""
        s = self.batch.stats.cpu().numpy()
        n = max(s[1], 1.0)
        return dict(mean_return=s[0] / n, success=s[2] / n, collision=s[3] / n, timeout=s[4] / n,
                    robot_episodes=int(s[1]), env_episodes=int(s[5]))


def split_obs(obs_rows):
    """[M, 40] packed rows -> the (self, objects, mask) triple the networks take."""
    M = obs_rows.shape[0]
    return obs_rows[:, 0:7], obs_rows[:, 7:32].reshape(M, 5, 5), obs_rows[:, 32:37]
