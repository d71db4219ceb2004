"""CPU: pin the per-robot NumPy restatement (oracle/env_numpy.py, the reference-style CPU baseline leg of
bench.py) to the reference's own captures before timing it as "the reference's CPU path":

  * every step of every F3 trace (tests/golden/env_traces.npz, MarineNavEnv3.step of env.py:240-333 with every
    perception draw recorded and injected here), teacher-forced: state within 1e-12, rewards and
    observations within 1e-12, collision / reach / done / info / COLREGs masks and object counts exact;
  * every F7 reset (env_reset.npz, env.py:72-176): starts, goals, headings, obstacles, cores, the vessels'
    perception seeds and the env RandomState's position after the reset exact, the first observations
    (each vessel's own RandomState draws) within 1e-12.
"""
import numpy as np
import pytest

from oracle import env_numpy as en
from oracle import env_oracle as eo

pytestmark = pytest.mark.filterwarnings("ignore::PendingDeprecationWarning")

INFO = {"normal": 0, "too long episode": 1, "collision": 2, "reach goal": 3, "deactivated after collision": 4,
        "deactivated after reaching goal": 5}


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b) / np.maximum(1.0, np.abs(b)))) if a.size else 0.0


def _pack(obs, n):
    so, oo, oc = np.zeros((n, 7)), np.zeros((n, 5, 5)), np.full(n, -1, np.int32)
    for i, (own, objs) in enumerate(obs):
        if own is None:
            continue
        so[i] = own
        oc[i] = len(objs)
        for k, o in enumerate(objs):
            oo[i, k] = o
    return so, oo, oc


@pytest.mark.parametrize("name", list(eo.load_traces().keys()))
def test_numpy_env_step_traces(name):
    tr = eo.load_traces()[name]
    n = int(tr["n_robots"])
    for t in range(len(tr["reward"])):
        i = eo.trace_step_inputs(tr, t)
        env = en.NpMarineEnv(seed=0, width=float(tr["width"]))
        env.obstacles = [en.Buoy(*o) for o in i["obstacles"][:i["n_obs"]]]
        env.cores = [en.Vortex(c[0], c[1], bool(c[2]), c[3]) for c in i["cores"][:i["n_cores"]]]
        env.core_r = float(tr["core_r"])
        env.episode_timesteps = i["ep_ts"]
        for k in range(n):
            v = en.Vessel(0)
            s = i["state_before"][k]
            v.x, v.y, v.theta = s[0], s[1], s[2]
            v.velocity_r, v.velocity = s[3:6].copy(), s[6:9].copy()
            v.left_thrust, v.right_thrust, v.left_pos, v.right_pos = s[9], s[10], s[11], s[12]
            v.goal = np.array(i["goals"][k], np.float64)
            v.deactivated, v.collision, v.reach_goal = bool(i["deact"][k]), bool(i["coll"][k]), bool(i["reach"][k])
            env.robots.append(v)
        cont = not name.startswith("disc")
        acts = [None if i["deact"][k] else (i["actions"][k] if cont else int(i["actions"][k][0])) for k in range(n)]
        with np.errstate(invalid="ignore"):
            obs, rew, done, info = env.step(acts, cont, noise=i["noise"], slot0=i["O"])
        sa = np.array([[v.x, v.y, v.theta, *v.velocity_r, *v.velocity, v.left_thrust, v.right_thrust, v.left_pos,
                        v.right_pos] for v in env.robots])
        so, oo, oc = _pack(obs, n)
        assert _rel(sa, tr["state_after"][t][:n]) < 1e-12, (name, t)
        assert _rel(rew, tr["reward"][t][:n]) < 1e-12, (name, t)
        act = i["deact"] == 0
        assert _rel(so[act], tr["self_obs"][t][:n][act]) < 1e-12, (name, t)
        assert _rel(oo[act], tr["obj_obs"][t][:n][act]) < 1e-12, (name, t)
        ref_cnt = np.where(tr["obs_valid"][t][:n] == 1, tr["obj_cnt"][t][:n], -1)
        assert np.array_equal(oc, ref_cnt), (name, t)
        assert np.array_equal(np.array(done, np.uint8), tr["done"][t][:n]), (name, t)
        assert np.array_equal(np.array([INFO[x] for x in info], np.uint8), tr["info"][t][:n]), (name, t)
        assert np.array_equal(np.array([v.collision for v in env.robots], np.uint8), tr["collision"][t][:n])
        assert np.array_equal(np.array([v.reach_goal for v in env.robots], np.uint8), tr["reach"][t][:n])
        app = np.array([v.apply_COLREGs for v in env.robots], np.uint8)
        assert np.array_equal(app[act], tr["apply_colregs"][t][:n][act]), (name, t)


def _reset_cases():
    z = np.load(eo.GOLDEN + "/env_reset.npz")
    return z, int(z["n_cases"])


SCHED = {"timesteps": [0, 1000000, 2000000, 3000000, 4000000, 5000000], "num_robots": [3, 4, 5, 5, 5, 5],
         "num_obstacles": [0, 0, 0, 2, 3, 4], "min_start_goal_dis": [30.0, 35.0, 40.0, 40.0, 40.0, 40.0]}


@pytest.mark.parametrize("c", range(_reset_cases()[1]))
def test_numpy_env_reset_layouts(c):
    z, _ = _reset_cases()
    p = f"c{c}/"
    kind, seed, ts = str(z[p + "kind"]), int(z[p + "seed"]), int(z[p + "total_timesteps"])
    if kind == "sched":   # env.py:75-87: the curriculum stage of total_timesteps
        idx = len([s for s in SCHED["timesteps"] if s - ts <= 0]) - 1
        env = en.NpMarineEnv(seed=seed, num_robots=SCHED["num_robots"][idx], num_obs=SCHED["num_obstacles"][idx],
                             min_start_goal_dis=SCHED["min_start_goal_dis"][idx])
    elif kind == "cores":
        env = en.NpMarineEnv(seed=seed, num_robots=4, num_cores=4, num_obs=3, min_start_goal_dis=30.0)
    else:
        env = en.NpMarineEnv(seed=seed, num_robots=17, num_obs=4, min_start_goal_dis=40.0, width=110.0)
    with np.errstate(invalid="ignore"):
        obs, coll, reach = env.reset()
    n = int(z[p + "n_robots"])
    assert len(env.robots) == n
    np.testing.assert_array_equal(np.array([v.start for v in env.robots]), z[p + "start"])
    np.testing.assert_array_equal(np.array([v.goal for v in env.robots]), z[p + "goal"])
    np.testing.assert_array_equal(np.array([v.init_theta for v in env.robots]), z[p + "init_theta"])
    np.testing.assert_array_equal(np.array([v.perception_seed for v in env.robots]), z[p + "perception_seed"])
    np.testing.assert_array_equal(np.array([[o.x, o.y, o.r] for o in env.obstacles]).reshape(-1, 3), z[p + "obstacles"])
    np.testing.assert_array_equal(np.array([[k.x, k.y, float(k.clockwise), k.Gamma] for k in env.cores]).reshape(-1, 4),
                                  z[p + "cores"])
    st = env.rd.get_state()
    np.testing.assert_array_equal(st[1][:8], z[p + "rng_after"])
    assert st[2] == int(z[p + "rng_pos_after"])
    so, oo, oc = _pack(obs, n)
    assert _rel(so, z[p + "self_obs"]) < 1e-12
    assert _rel(oo, z[p + "obj_obs"]) < 1e-12
    np.testing.assert_array_equal(oc, z[p + "obj_cnt"])


def test_numpy_env_rollout_runs():
    n, el = en.rollout(0.5, seed=3)
    assert n > 10 and el >= 0.5


def test_reference_style_training_loop_runs():
    """oracle/ref_loop.py (bench.py's reference-style CPU leg): act + env.step + replay + train_AC_IQN at B = 64
    every 4 steps on one process, both modes."""
    from oracle import ref_loop
    r = ref_loop.train_loop(1.0, seed=2)
    assert r["steps"] >= 8 and r["learns"] >= 1 and r["seconds"] >= 1.0
    e = ref_loop.train_loop(0.3, seed=2, env_only=True)
    assert e["learns"] == 0 and e["steps"] >= 8
