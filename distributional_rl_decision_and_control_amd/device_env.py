"""Device-resident env batch: the HBM layout of E ASV envs and the launches on it.

One DeviceEnvBatch owns the SoA state of `n_envs` MarineNavEnv3 scenes (include/asvrl.h
AsvEnvState) as torch tensors on the GPU and calls the gfx950 kernels through the C ABI.
Both the vectorised training env (vec_env.VecMarineNavEnv) and the drop-in single-env
MarineNavEnv3 (envs/marinenav/env.py) sit on top of it.
"""
import ctypes as C

import torch

from . import _abi
from ._abi import OBS_DIM, NUM_FIELDS


class DeviceEnvBatch:
    def __init__(self, n_envs, max_robots, max_obs, max_cores=0, device="cuda", params=None, obs64=False):
        _abi.lib()  # fail loudly before allocating anything
        if max_robots < 1 or max_robots > 256:
            raise ValueError("max_robots must be in [1, 256]")
        self.n_envs, self.max_robots, self.max_obs, self.max_cores = n_envs, max_robots, max_obs, max_cores
        self.device = torch.device(device)
        self.params = params if params is not None else _abi.params_from()
        E, R, O, Cc = n_envs, max_robots, max(max_obs, 0), max(max_cores, 0)
        NT = E * R
        dev = self.device
        f64 = dict(dtype=torch.float64, device=dev)
        self.rs = torch.zeros((NUM_FIELDS, NT), **f64)
        self.rflags = torch.zeros(NT, dtype=torch.uint8, device=dev)
        self.n_robots = torch.zeros(E, dtype=torch.int32, device=dev)
        self.n_obs = torch.zeros(E, dtype=torch.int32, device=dev)
        self.n_cores = torch.zeros(E, dtype=torch.int32, device=dev)
        self.ep_ts = torch.zeros(E, dtype=torch.int32, device=dev)
        self.obstacles = torch.zeros((E, max(O, 1), 3), **f64)
        self.cores = torch.zeros((E, max(Cc, 1), 4), **f64)
        # outputs
        self.obs = torch.zeros((NT, OBS_DIM), dtype=torch.float32, device=dev)
        self.obs64 = torch.zeros((NT, 32), **f64) if obs64 else None
        self.obj_cnt = torch.zeros(NT, dtype=torch.int8, device=dev)
        self.reward = torch.zeros(NT, **f64)
        self.done = torch.zeros(NT, dtype=torch.uint8, device=dev)
        self.info = torch.zeros(NT, dtype=torch.uint8, device=dev)
        self.env_done = torch.zeros(E, dtype=torch.uint8, device=dev)
        self.stats = torch.zeros(8, **f64)
        # optional per-robot AsvParams table (AsvEnvState.robot_params; set_robot_params)
        self.robot_params = None

    def set_robot_params(self, table):
        """Every robot slot's own vehicle / perception parameters: a sequence of n_envs * max_robots
        AsvParams (reset_with_eval_config, env.py:553-607), or None for `params` everywhere. The
        table's env-level members are ignored (the kernel takes those from `params`)."""
        if table is None:
            self.robot_params = None
            return
        NT = self.n_envs * self.max_robots
        if len(table) != NT:
            raise ValueError(f"robot parameter table: {len(table)} entries for {NT} robot slots")
        arr = (_abi.AsvParams * NT)(*table)
        host = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
        if self.robot_params is None or self.robot_params.numel() != host.numel():
            self.robot_params = torch.empty(host.numel(), dtype=torch.uint8, device=self.device)
        self.robot_params.copy_(host)

    # ------------------------------------------------------------------ ABI structs
    def state_struct(self):
        s = _abi.AsvEnvState()
        s.n_envs, s.max_robots, s.max_obs, s.max_cores = self.n_envs, self.max_robots, self.max_obs, self.max_cores
        s.rs = self.rs.data_ptr()
        s.rflags = self.rflags.data_ptr()
        s.n_robots = self.n_robots.data_ptr()
        s.n_obs = self.n_obs.data_ptr()
        s.n_cores = self.n_cores.data_ptr()
        s.ep_ts = self.ep_ts.data_ptr()
        s.obstacles = self.obstacles.data_ptr()
        s.cores = self.cores.data_ptr()
        s.robot_params = self.robot_params.data_ptr() if self.robot_params is not None else None
        return s

    def out_struct(self, obs=None, obj_cnt=None, with_env_done=True):
        o = _abi.AsvStepOut()
        o.obs = (obs if obs is not None else self.obs).data_ptr()
        o.obs64 = self.obs64.data_ptr() if self.obs64 is not None else None
        o.obj_cnt = (obj_cnt if obj_cnt is not None else self.obj_cnt).data_ptr()
        o.reward = self.reward.data_ptr()
        o.done = self.done.data_ptr()
        o.info = self.info.data_ptr()
        o.env_done = self.env_done.data_ptr() if with_env_done else None
        o.stats = self.stats.data_ptr() if with_env_done else None
        return o

    # ------------------------------------------------------------------ launches
    def step(self, actions, is_continuous=True, noise=None, do_dynamics=True, trainer_deactivate=False,
             seed=0, counter=0, counter_dev=None, gamma=0.0, env_mask=None, obs=None, obj_cnt=None, stream=None,
             fast_noise=False, launch=None):
        """asvrl_env_step. actions: f64 [E*R, 2] device tensor. noise: f64 [E*R, O+R, 5] or None (Philox;
        fast_noise: f32 draws, noise_mode 2). launch: (layout, block, envs_per_block) of the kernel
        (asvrl_env_step_ex; _abi.ENV_LAYOUT_*), None = automatic."""
        ctl = _abi.AsvStepCtl()
        ctl.is_continuous = int(bool(is_continuous))
        ctl.do_dynamics = int(bool(do_dynamics))
        ctl.trainer_deactivate = int(bool(trainer_deactivate))
        ctl.noise_mode = 0 if noise is not None else (2 if fast_noise else 1)
        ctl.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        ctl.counter = int(counter) & 0xFFFFFFFFFFFFFFFF
        ctl.counter_dev = counter_dev.data_ptr() if counter_dev is not None else None
        ctl.gamma = float(gamma)
        ctl.env_mask = env_mask.data_ptr() if env_mask is not None else None
        if actions is not None:
            assert actions.dtype == torch.float64 and actions.is_contiguous()
            assert actions.numel() >= 2 * self.n_envs * self.max_robots
        if noise is not None:
            assert noise.dtype == torch.float64 and noise.is_contiguous()
            assert noise.numel() >= self.n_envs * self.max_robots * (self.max_obs + self.max_robots) * 5
        st = self.state_struct()
        out = self.out_struct(obs, obj_cnt, with_env_done=trainer_deactivate)
        if launch is None:
            rc = _abi.lib().asvrl_env_step(C.byref(self.params), C.byref(st), _abi.ptr(actions), _abi.ptr(noise),
                                           C.byref(ctl), C.byref(out), _abi.stream_ptr(stream))
        else:
            ln = _abi.AsvEnvLaunch(*(int(v) for v in launch))
            rc = _abi.lib().asvrl_env_step_ex(C.byref(self.params), C.byref(st), _abi.ptr(actions), _abi.ptr(noise),
                                              C.byref(ctl), C.byref(out), C.byref(ln), _abi.stream_ptr(stream))
        _abi.check(rc, "asvrl_env_step")

    def reset(self, cfg, env_mask=None, seed=0, counter=0, counter_dev=None, stream=None):
        st = self.state_struct()
        rc = _abi.lib().asvrl_env_reset(C.byref(self.params), C.byref(st), C.byref(cfg), _abi.ptr(env_mask),
                                        int(seed) & 0xFFFFFFFFFFFFFFFF, int(counter) & 0xFFFFFFFFFFFFFFFF,
                                        _abi.ptr(counter_dev), _abi.stream_ptr(stream))
        _abi.check(rc, "asvrl_env_reset")


    def reset_observe(self, cfg, env_mask, seed=0, counter=0, counter_dev=None, obs_counter=0, obs=None,
                      obj_cnt=None, fast_noise=True, stream=None):
        """asvrl_env_reset_observe: reset the envs of env_mask (reset's sampler at (seed, counter)) and write
        their reset observations (the masked do_dynamics = 0 step at (seed, obs_counter)) in one launch --
        the same values as reset(...) followed by step(None, do_dynamics=False, env_mask=...)."""
        ctl = _abi.AsvStepCtl()
        ctl.is_continuous = 1
        ctl.do_dynamics = 0
        ctl.trainer_deactivate = 0
        ctl.noise_mode = 2 if fast_noise else 1
        ctl.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        ctl.counter = int(obs_counter) & 0xFFFFFFFFFFFFFFFF
        ctl.counter_dev = counter_dev.data_ptr() if counter_dev is not None else None
        ctl.gamma = 0.0
        ctl.env_mask = env_mask.data_ptr()
        st = self.state_struct()
        out = self.out_struct(obs, obj_cnt, with_env_done=False)
        rc = _abi.lib().asvrl_env_reset_observe(C.byref(self.params), C.byref(st), C.byref(cfg), _abi.ptr(env_mask),
                                                int(seed) & 0xFFFFFFFFFFFFFFFF, int(counter) & 0xFFFFFFFFFFFFFFFF,
                                                _abi.ptr(counter_dev), C.byref(ctl), C.byref(out),
                                                _abi.stream_ptr(stream))
        _abi.check(rc, "asvrl_env_reset_observe")


def reset_cfg(num_robots=5, num_obs=4, num_cores=0, min_start_goal_dis=40.0, width=55.0, height=55.0,
              clear_r=10.0, obs_r_range=(1.0, 1.0), v_range=(3.0, 3.0), v_rel_max=1.0, p=0.8):
    """AsvResetCfg with the reference's env.py:33-54 defaults (curriculum values override)."""
    c = _abi.AsvResetCfg()
    c.num_robots, c.num_obs, c.num_cores = int(num_robots), int(num_obs), int(num_cores)
    c.min_start_goal_dis, c.width, c.height, c.clear_r = float(min_start_goal_dis), float(width), float(height), float(clear_r)
    c.obs_r_lo, c.obs_r_hi = float(obs_r_range[0]), float(obs_r_range[1])
    c.v_lo, c.v_hi = float(v_range[0]), float(v_range[1])
    c.v_rel_max, c.p_rel = float(v_rel_max), float(p)
    return c


def current_field(cores, core_r, xy, stream=None):
    """Ocean current (env.py:458-501) at points xy [n,2] (device f64) for cores [n_cores,4]."""
    n = xy.shape[0]
    out = torch.empty((n, 3), dtype=torch.float64, device=xy.device)
    nc = 0 if cores is None else int(cores.shape[0])
    rc = _abi.lib().asvrl_current_field(_abi.ptr(cores) if nc else None, nc, float(core_r), _abi.ptr(xy), n,
                                        _abi.ptr(out), _abi.stream_ptr(stream))
    _abi.check(rc, "asvrl_current_field")
    return out
