"""ctypes front-end of the C oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
It wraps oracle/build/libasv_oracle.so (built by `make -C oracle`) -- the per-robot C
restatement of MarineNavEnv3.step (rfarl/rfarl/envs/marinenav/env.py:240-333) -- and the
golden fixtures' trace layout (tools/capture_oracle.py).
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libasv_oracle.so")


class OrParams(C.Structure):
    _fields_ = [
        ("dt", C.c_double), ("N", C.c_int32),
        ("length", C.c_double), ("width", C.c_double), ("r", C.c_double), ("goal_dis", C.c_double),
        ("min_thrust", C.c_double), ("max_thrust", C.c_double), ("m", C.c_double), ("Izz", C.c_double),
    ] + [(n, C.c_double) for n in
         ["xDotU", "yDotV", "yDotR", "nDotR", "nDotV", "xU", "xUU", "yV", "yVV", "yR", "yRV", "yVR",
          "yRR", "nR", "nRR", "nV", "nVV", "nRV", "nVR"]] + [
        ("P", C.c_double * 9), ("thrust_change", C.c_double * 5),
        ("range", C.c_double), ("angle", C.c_double), ("r_mean_ratio", C.c_double),
        ("max_obj_num", C.c_int32),
        ("timestep_penalty", C.c_double), ("COLREGs_penalty", C.c_double),
        ("collision_penalty", C.c_double), ("goal_reward", C.c_double), ("core_r", C.c_double),
        ("episode_limit", C.c_int32),
    ]


class OrRobot(C.Structure):
    _fields_ = [("x", C.c_double), ("y", C.c_double), ("theta", C.c_double),
                ("vr", C.c_double * 3), ("v", C.c_double * 3), ("tl", C.c_double), ("tr", C.c_double),
                ("lp", C.c_double), ("rp", C.c_double), ("goal", C.c_double * 2),
                ("deactivated", C.c_uint8), ("collision", C.c_uint8), ("reach_goal", C.c_uint8),
                ("apply_colregs", C.c_uint8), ("phi", C.c_double)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        dp = C.POINTER(C.c_double)
        L.or_default_params.argtypes = [C.POINTER(OrParams)]
        L.or_current.argtypes = [dp, C.c_int, C.c_double, C.c_double, C.c_double, dp]
        L.or_robot_act.argtypes = [C.POINTER(OrParams), C.POINTER(OrRobot), dp, C.c_int, dp, C.c_int]
        L.or_robot_act.restype = C.c_double
        L.or_env_step.argtypes = [C.POINTER(OrParams), C.POINTER(OrRobot), C.c_int, C.c_int, dp, C.c_int,
                                  C.c_int, dp, C.c_int, dp, C.c_int, dp, C.POINTER(C.c_int32), dp,
                                  C.POINTER(C.c_uint8), C.POINTER(C.c_uint8), dp, dp, C.POINTER(C.c_int32)]
        L.or_env_step.restype = C.c_int
        L.or_batch_rollout.argtypes = [C.POINTER(OrParams), C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64,
                                       C.c_int, dp]
        L.or_batch_rollout.restype = C.c_int64
        fp = C.POINTER(C.c_float)
        L.or_c51_project.argtypes = [fp, fp, fp, fp, C.c_int, C.c_int, C.c_float, C.c_float, C.c_float, fp]
        ip = C.POINTER(C.c_int)
        L.or_device_reset.argtypes = [C.c_void_p, C.c_double, C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_uint64,
                                      C.c_int, dp, ip, dp, ip, dp, ip]
        _lib = L
    return _lib


def device_reset(cfg, core_r, R, O, Cmax, seed, counter, e):
    """The device reset of env e restated one candidate at a time (or_device_reset; cfg: an AsvResetCfg,
    whose layout OrResetCfg mirrors). Returns (robots [n][5] x, y, gx, gy, theta, cores [n][4],
    obstacles [n][3])."""
    rob = np.zeros((max(R, 1), 5))
    cor = np.zeros((max(Cmax, 1), 4))
    obs = np.zeros((max(O, 1), 3))
    nr, nc, no = C.c_int(), C.c_int(), C.c_int()
    lib().or_device_reset(C.addressof(cfg), float(core_r), R, O, Cmax, seed, counter, e, _dp(rob), C.byref(nr),
                          _dp(cor), C.byref(nc), _dp(obs), C.byref(no))
    return rob[:nr.value], cor[:nc.value], obs[:no.value]


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def default_params(P=None):
    p = OrParams()
    lib().or_default_params(C.byref(p))
    if P is not None:
        for k in range(9):
            p.P[k] = float(P.reshape(-1)[k])
    return p


def robots_from_states(states, goals, deact=None, coll=None, reach=None):
    n = states.shape[0]
    arr = (OrRobot * n)()
    for i in range(n):
        s = states[i]
        r = arr[i]
        r.x, r.y, r.theta = s[0], s[1], s[2]
        for k in range(3):
            r.vr[k] = s[3 + k]
            r.v[k] = s[6 + k]
        r.tl, r.tr, r.lp, r.rp = s[9], s[10], s[11], s[12]
        r.goal[0], r.goal[1] = goals[i]
        r.deactivated = int(deact[i]) if deact is not None else 0
        r.collision = int(coll[i]) if coll is not None else 0
        r.reach_goal = int(reach[i]) if reach is not None else 0
        r.phi = np.nan
    return arr


def robot_states(arr, n):
    out = np.zeros((n, 13))
    for i in range(n):
        r = arr[i]
        out[i] = [r.x, r.y, r.theta, r.vr[0], r.vr[1], r.vr[2], r.v[0], r.v[1], r.v[2], r.tl, r.tr, r.lp, r.rp]
    return out


def current(cores, core_r, x, y):
    cores = np.ascontiguousarray(cores, dtype=np.float64)
    out = np.zeros(3)
    lib().or_current(_dp(cores), cores.shape[0], core_r, x, y, _dp(out))
    return out


def robot_act(p, state, goal, action, continuous, cores=None):
    arr = robots_from_states(state[None], goal[None])
    a = np.ascontiguousarray(action, dtype=np.float64)
    if cores is None or len(cores) == 0:
        cp, nc = None, 0
    else:
        cores = np.ascontiguousarray(cores, dtype=np.float64)
        cp, nc = _dp(cores), cores.shape[0]
    rew = lib().or_robot_act(C.byref(p), arr, _dp(a), int(continuous), cp, nc)
    return robot_states(arr, 1)[0], rew


def env_step(p, state_before, goals, deact, coll, reach, obstacles, n_obs, O, cores, n_cores, actions,
             continuous, noise, ep_ts):
    """One MarineNavEnv3.step on the oracle. Returns a dict like the fixture step record."""
    n = state_before.shape[0]
    R = n
    arr = robots_from_states(state_before, goals, deact, coll, reach)
    obstacles = np.ascontiguousarray(obstacles, dtype=np.float64)
    cores = np.ascontiguousarray(cores, dtype=np.float64)
    acts = np.ascontiguousarray(actions, dtype=np.float64)
    noise = np.ascontiguousarray(noise, dtype=np.float64)
    assert noise.shape == (R, O + R, 5)
    ts = C.c_int32(int(ep_ts))
    rew = np.zeros(n)
    dn = np.zeros(n, np.uint8)
    inf = np.zeros(n, np.uint8)
    so = np.zeros((n, 7))
    ob = np.zeros((n, 5, 5))
    cnt = np.zeros(n, np.int32)
    rc = lib().or_env_step(C.byref(p), arr, n, R, _dp(obstacles), int(n_obs), O, _dp(cores), int(n_cores),
                           _dp(acts), int(continuous), _dp(noise), C.byref(ts), _dp(rew),
                           dn.ctypes.data_as(C.POINTER(C.c_uint8)), inf.ctypes.data_as(C.POINTER(C.c_uint8)),
                           _dp(so), _dp(ob), cnt.ctypes.data_as(C.POINTER(C.c_int32)))
    if rc != 0:
        raise RuntimeError("Robot being deactived can only be caused by collsion or reaching goal!")
    return dict(state_after=robot_states(arr, n), reward=rew, done=dn, info=inf, self_obs=so, obj_obs=ob,
                obj_cnt=cnt, collision=np.array([arr[i].collision for i in range(n)], np.uint8),
                reach=np.array([arr[i].reach_goal for i in range(n)], np.uint8),
                apply_colregs=np.array([arr[i].apply_colregs for i in range(n)], np.uint8),
                phi=np.array([arr[i].phi for i in range(n)]), ep_ts=ts.value)


def batch_rollout(E, R, O, steps, seed=0, threads=1):
    p = default_params()
    chk = C.c_double(0)
    n = lib().or_batch_rollout(C.byref(p), E, R, O, steps, seed, threads, C.byref(chk))
    return n, chk.value


def c51_project(pns_a, returns, nonterminal, support, vmin=-1.0, vmax=1.0, gamma_n=0.99 ** 3):
    pns_a = np.ascontiguousarray(pns_a, dtype=np.float32)
    B, atoms = pns_a.shape
    R = np.ascontiguousarray(returns, dtype=np.float32).reshape(B)
    nt = np.ascontiguousarray(nonterminal, dtype=np.float32).reshape(B)
    sup = np.ascontiguousarray(support, dtype=np.float32)
    m = np.zeros((B, atoms), np.float32)
    fp = C.POINTER(C.c_float)
    lib().or_c51_project(pns_a.ctypes.data_as(fp), R.ctypes.data_as(fp), nt.ctypes.data_as(fp),
                         sup.ctypes.data_as(fp), B, atoms, vmin, vmax, float(np.float32(gamma_n)),
                         m.ctypes.data_as(fp))
    return m


# ---------------------------------------------------------------------------- fixtures
GOLDEN = os.path.join(HERE, "..", "tests", "golden")


def load_traces(fname="env_traces.npz"):
    z = np.load(os.path.join(GOLDEN, fname))
    names = list(z["names"])
    out = {}
    for nm in names:
        out[nm] = {k.split("/", 1)[1]: z[k] for k in z.files if k.startswith(nm + "/")}
    return out


def trace_step_inputs(tr, t):
    """Oracle inputs for step t of a fixture trace (teacher-forced state)."""
    n = int(tr["n_robots"])
    R = int(tr["R"])
    O = int(tr["O"])
    sb = tr["state_before"][t][:n]
    deact = tr["deact_before"][t][:n]
    # flags before the step: sticky collision / reach of robots still active are 0 (the
    # trainer deactivates on either flag); deactivated robots carry theirs from the last step
    if t == 0:
        coll = np.zeros(n, np.uint8)
        reach = np.zeros(n, np.uint8)
    else:
        coll = tr["collision"][t - 1][:n]
        reach = tr["reach"][t - 1][:n]
    noise = np.nan_to_num(tr["noise"][t][:n][:, :O + n], nan=0.0)
    noise_full = np.zeros((n, O + n, 5))
    noise_full[:, :O] = noise[:, :O]
    noise_full[:, O:O + n] = noise[:, O:O + n]
    return dict(state_before=sb, goals=tr["goals"][:n], deact=deact, coll=coll, reach=reach,
                obstacles=tr["obstacles"], n_obs=int(tr["n_obs"]), O=O, cores=tr["cores"],
                n_cores=int(tr["n_cores"]), actions=tr["actions"][t][:n], noise=noise_full,
                ep_ts=int(tr["ep_ts"][t]), R=R)


def trainer_bookkeeping(rewards, deact_before, collision, reach, ep_ts, gamma=0.99, episode_limit=1000):
    """Trainer.learn's per-step bookkeeping (rfarl/rfarl/policy/trainer.py:157-172) over a trace:
    ep_rewards[i] += gamma ** ep_length * r_i for every robot not deactivated before the step,
    then deactivation on collision or goal, then end_episode = ep_length >= 1000 or all
    deactivated. rewards [T][n], deact_before [T][n], collision / reach [T][n] (flags after the
    step), ep_ts [T] (the env's episode_timesteps before the step = the trainer's ep_length).
    Returns (ep_return [T][n], deact_after [T][n], end_episode [T])."""
    T, n = np.asarray(rewards).shape
    ret = np.zeros(n)
    rets, deacts, ends = np.zeros((T, n)), np.zeros((T, n), np.uint8), np.zeros(T, np.uint8)
    for t in range(T):
        deact = np.asarray(deact_before[t][:n]).astype(bool).copy()
        ep_length = int(ep_ts[t])
        for i in range(n):
            if deact[i]:
                continue
            ret[i] += gamma ** ep_length * float(rewards[t][i])
            if collision[t][i] or reach[t][i]:
                deact[i] = True
        rets[t], deacts[t] = ret, deact
        ends[t] = (ep_length >= episode_limit) or bool(deact.all())
    return rets, deacts, ends
