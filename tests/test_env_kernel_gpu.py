"""GPU parity of the env-step kernel against the reference's own outputs (tests/golden).

Every step of every captured MarineNavEnv3 trace becomes one env of a single batched launch
(teacher-forced: the captured pre-step state, flags, actions and the exact perception noise
the reference drew), so one kernel launch is checked against ~800 reference steps:
  * f64 state, rewards and observations within 1e-12 (abs, scaled by magnitude),
  * collision / reach-goal / done / info / object-count / COLREGs masks bit-exact.
"""
import numpy as np
import pytest
import torch

from oracle import env_oracle as eo

pytestmark = pytest.mark.gpu

TOL = 1e-12


def _close(a, b, tol=TOL):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    scale = np.maximum(1.0, np.abs(b))
    return np.all(np.abs(a - b) <= tol * scale), float(np.max(np.abs(a - b) / scale)) if a.size else 0.0


def _batch_from_traces(traces, continuous):
    """Flatten (trace, step) pairs into env rows of one DeviceEnvBatch."""
    rows = []
    for name, tr in traces.items():
        if name.startswith("disc") == continuous:
            continue
        for t in range(len(tr["reward"])):
            rows.append((name, t, eo.trace_step_inputs(tr, t), tr))
    return rows


def _run_rows(rows, continuous, launch=None):
    from distributional_rl_decision_and_control_amd.device_env import DeviceEnvBatch
    from distributional_rl_decision_and_control_amd import _abi

    E = len(rows)
    R = max(r[2]["state_before"].shape[0] for r in rows)
    O = max(r[2]["O"] for r in rows)
    Cm = 8
    z = np.load(eo.GOLDEN + "/env_dynamics.npz")
    params = _abi.params_from()
    assert np.array_equal(np.array(params.P[:]), z["P"].reshape(-1)), "host P differs from the reference's numpy P"
    b = DeviceEnvBatch(E, R, O, Cm, obs64=True, params=params)
    rs = np.zeros((_abi.NUM_FIELDS, E * R))
    fl = np.zeros(E * R, np.uint8)
    nrob = np.zeros(E, np.int32)
    nobs = np.zeros(E, np.int32)
    ncor = np.zeros(E, np.int32)
    ep = np.zeros(E, np.int32)
    obst = np.zeros((E, O, 3))
    cores = np.zeros((E, Cm, 4))
    acts = np.zeros((E * R, 2))
    noise = np.zeros((E * R, O + R, 5))
    for e, (_, _, inp, tr) in enumerate(rows):
        n = inp["state_before"].shape[0]
        base = e * R
        sb = inp["state_before"]
        rs[:13, base:base + n] = sb.T
        rs[_abi.F_GX, base:base + n] = inp["goals"][:, 0]
        rs[_abi.F_GY, base:base + n] = inp["goals"][:, 1]
        fl[base:base + n] = (inp["deact"] * _abi.FLAG_DEACTIVATED) | (inp["coll"] * _abi.FLAG_COLLISION) | (
            inp["reach"] * _abi.FLAG_REACH_GOAL)
        nrob[e] = n
        nobs[e] = inp["n_obs"]
        ncor[e] = inp["n_cores"]
        ep[e] = inp["ep_ts"]
        Oe = inp["O"]
        obst[e, :Oe] = inp["obstacles"]
        cores[e, :inp["n_cores"]] = inp["cores"][:inp["n_cores"]]
        acts[base:base + n] = inp["actions"]
        nz = inp["noise"]  # [n, Oe + n, 5]
        noise[base:base + n, :Oe] = nz[:, :Oe]
        noise[base:base + n, O:O + n] = nz[:, Oe:Oe + n]
    dev = b.device
    b.rs.copy_(torch.from_numpy(rs))
    b.rflags.copy_(torch.from_numpy(fl))
    b.n_robots.copy_(torch.from_numpy(nrob))
    b.n_obs.copy_(torch.from_numpy(nobs))
    b.n_cores.copy_(torch.from_numpy(ncor))
    b.ep_ts.copy_(torch.from_numpy(ep))
    b.obstacles.copy_(torch.from_numpy(obst))
    b.cores.copy_(torch.from_numpy(cores))
    a_d = torch.from_numpy(acts).to(dev)
    n_d = torch.from_numpy(noise).to(dev)
    b.step(a_d, is_continuous=continuous, noise=n_d, launch=launch)
    torch.cuda.synchronize()
    return b, R


def _check_rows(rows, b, R):
    from distributional_rl_decision_and_control_amd import _abi
    rs = b.rs.cpu().numpy()
    fl = b.rflags.cpu().numpy()
    o64 = b.obs64.cpu().numpy()
    cnt = b.obj_cnt.cpu().numpy()
    rew = b.reward.cpu().numpy()
    done = b.done.cpu().numpy()
    info = b.info.cpu().numpy()
    obs32 = b.obs.cpu().numpy()
    worst = {}
    for e, (name, t, inp, tr) in enumerate(rows):
        n = inp["state_before"].shape[0]
        sl = slice(e * R, e * R + n)
        checks = {
            "state": (rs[:13, sl].T, tr["state_after"][t][:n]),
            "reward": (rew[sl], tr["reward"][t][:n]),
            "self_obs": (o64[sl, :7], tr["self_obs"][t][:n]),
            "obj_obs": (o64[sl, 7:32].reshape(n, 5, 5), tr["obj_obs"][t][:n]),
        }
        for k, (got, ref) in checks.items():
            ok, err = _close(got, ref)
            worst[k] = max(worst.get(k, 0.0), err)
            assert ok, f"{name} step {t}: {k} off by {err}"
        valid = tr["obs_valid"][t][:n]
        ref_cnt = np.where(valid == 1, tr["obj_cnt"][t][:n], -1)
        assert np.array_equal(cnt[sl].astype(int), ref_cnt.astype(int)), f"{name} step {t}: object count"
        assert np.array_equal(done[sl], tr["done"][t][:n]), f"{name} step {t}: done mask"
        assert np.array_equal(info[sl], tr["info"][t][:n]), f"{name} step {t}: info"
        assert np.array_equal((fl[sl] & _abi.FLAG_COLLISION) > 0, tr["collision"][t][:n] > 0), f"{name} {t}: collision"
        assert np.array_equal((fl[sl] & _abi.FLAG_REACH_GOAL) > 0, tr["reach"][t][:n] > 0), f"{name} {t}: reach"
        act = inp["deact"] == 0
        assert np.array_equal(((fl[sl] & _abi.FLAG_COLREGS) > 0)[act], tr["apply_colregs"][t][:n][act] > 0)
        phi_ref = tr["phi"][t][:n]
        m = ~np.isnan(phi_ref)
        if m.any():
            ok, err = _close(rs[_abi.F_PHI, sl][m], phi_ref[m])
            assert ok, f"{name} step {t}: phi off by {err}"
        # packed f32 row == the reference's state_batch(...).float() layout
        so = tr["self_obs"][t][:n].astype(np.float32)
        oo = tr["obj_obs"][t][:n].astype(np.float32).reshape(n, 25)
        mask = (np.arange(5)[None, :] < ref_cnt[:, None]).astype(np.float32)
        for i in range(n):
            if ref_cnt[i] < 0:
                assert not obs32[e * R + i].any()
                continue
            np.testing.assert_array_equal(obs32[e * R + i, :7], so[i])
            np.testing.assert_array_equal(obs32[e * R + i, 7:32], oo[i])
            np.testing.assert_array_equal(obs32[e * R + i, 32:37], mask[i])
    return worst


# every shipped kernel layout (asvrl_env_step_ex): the automatic choice (pair-parallel, 256 lanes at
# these sizes), the per-robot sweep (the automatic fallback when the pair layout's LDS does not fit,
# e.g. R ~ 64), the large-batch shape (one wave of 8 envs, from 16384 envs), the many-robot shape
# (256 lanes, 7 envs) and a non-default pair shape (128 threads, 2 envs per workgroup)
LAYOUTS = {"auto": None, "sweep": (2, 0, 0), "pairs_b64_e8": (1, 64, 8), "pairs_b256_e7": (1, 256, 7),
           "pairs_b128_e2": (1, 128, 2)}


@pytest.mark.parametrize("layout", list(LAYOUTS))
@pytest.mark.parametrize("continuous", [True, False])
def test_env_step_matches_reference_traces(continuous, layout):
    traces = eo.load_traces()
    rows = _batch_from_traces(traces, continuous)
    assert len(rows) > 0
    b, R = _run_rows(rows, continuous, LAYOUTS[layout])
    worst = _check_rows(rows, b, R)
    print("worst relative errors:", worst)


@pytest.mark.parametrize("case", ["cont", "disc", "cont_cores"])
def test_dynamics_matches_reference(case):
    """F1: N Fossen substeps from random states (wamv.py:204-279), incl. theta wrap, thrust
    saturation, discrete action grid and the 4-core current field."""
    from distributional_rl_decision_and_control_amd.device_env import DeviceEnvBatch
    from distributional_rl_decision_and_control_amd import _abi
    z = np.load(eo.GOLDEN + "/env_dynamics.npz")
    sb, sa, acts = z[case + "/state_before"], z[case + "/state_after"], z[case + "/actions"]
    E = sb.shape[0]
    b = DeviceEnvBatch(E, 1, 0, 8)
    rs = np.zeros((_abi.NUM_FIELDS, E))
    rs[:13] = sb.T
    b.rs.copy_(torch.from_numpy(rs))
    b.n_robots.fill_(1)
    if case == "cont_cores":
        b.n_cores.fill_(4)
        c = np.zeros((E, 8, 4))
        c[:, :4] = z["cores"][None]
        b.cores.copy_(torch.from_numpy(c))
    b.step(torch.from_numpy(acts).cuda(), is_continuous=case != "disc",
           noise=torch.zeros((E, 1, 5), dtype=torch.float64, device="cuda"))
    got = b.rs[:13].T.cpu().numpy()
    ok, err = _close(got, sa)
    assert ok, f"dynamics {case}: max rel err {err}"


def test_current_field_matches_reference():
    from distributional_rl_decision_and_control_amd.device_env import current_field
    z = np.load(eo.GOLDEN + "/env_dynamics.npz")
    out = current_field(torch.from_numpy(z["cores"]).cuda(), float(z["core_r"]),
                        torch.from_numpy(z["current_query"]).cuda()).cpu().numpy()
    ok, err = _close(out, z["current_value"])
    assert ok, err


def test_env_step_philox_invariants_full_size():
    """Config-2 size (4096 envs x 5 robots, 4 buoys): device reset + 50 Philox-noise steps.
    Size-independent properties: theta in [0, 2pi), thrust within bounds, masks consistent
    with info codes, deactivated robots frozen, identical results on a replay."""
    from distributional_rl_decision_and_control_amd.device_env import DeviceEnvBatch, reset_cfg
    from distributional_rl_decision_and_control_amd import _abi
    E, R, O = 4096, 5, 4

    def run():
        b = DeviceEnvBatch(E, R, O, 0)
        b.reset(reset_cfg(5, 4, 0, 40.0), seed=7)
        b.step(None, do_dynamics=False, seed=7, counter=0)
        g = torch.Generator(device="cuda").manual_seed(3)
        snaps = []
        for t in range(50):
            a = (torch.rand((E * R, 2), generator=g, device="cuda", dtype=torch.float64) * 2 - 1).contiguous()
            prev_fl = b.rflags.clone()
            prev_rs = b.rs.clone()
            b.step(a, seed=7, counter=t + 1, trainer_deactivate=True, gamma=0.99)
            th = b.rs[_abi.F_THETA]
            assert bool(((th >= 0) & (th < 2 * np.pi)).all())
            for f in (_abi.F_TL, _abi.F_TR):
                assert bool(((b.rs[f] >= -500) & (b.rs[f] <= 1000)).all())
            was_off = (prev_fl & _abi.FLAG_DEACTIVATED) > 0
            assert torch.equal(b.rs[:13][:, was_off], prev_rs[:13][:, was_off])
            info = b.info
            fl = b.rflags
            coll = (fl & _abi.FLAG_COLLISION) > 0
            assert bool((coll[info == _abi.INFO_COLLISION]).all())
            assert bool((b.done[info == _abi.INFO_NORMAL] == 0).all())
            snaps.append(b.reward.clone())
        return torch.stack(snaps), b

    r1, b1 = run()
    r2, _ = run()
    assert torch.equal(r1, r2), "Philox path must be deterministic for a fixed seed"
    n = b1.n_robots.cpu().numpy()
    assert n.min() >= 1 and n.max() <= R
    assert b1.n_obs.cpu().numpy().max() <= O


@pytest.mark.parametrize("R,O,Cn,W", [(5, 4, 0, 55.0), (5, 4, 4, 55.0), (17, 4, 0, 110.0)])
def test_device_reset_invariants(R, O, Cn, W):
    """asvrl_env_reset (wave-per-env rejection sampler) satisfies every acceptance rule of
    MarineNavEnv3.reset (env.py:106-162, check_core :378-418, check_obstacle :420-456) on all
    envs, clears the robot state, deactivates unused slots, and is deterministic in
    (seed, counter). Rules checked: start-goal distance >= min_start_goal_dis; pairwise
    starts and goals > clear_r; starts/goals in [2, W-2]; obstacles in [5, W-5], clear of
    starts/goals by r + clear_r and of each other by r_i + r_j; cores inside the map and
    clear of starts/goals by core_r + clear_r."""
    from distributional_rl_decision_and_control_amd import _abi
    from distributional_rl_decision_and_control_amd.device_env import DeviceEnvBatch, reset_cfg
    E = 2048
    cfg = reset_cfg(R, O, Cn, 40.0, width=W, height=W)

    def make(counter):
        b = DeviceEnvBatch(E, R, O, max(Cn, 1))
        b.rs.fill_(123.0)
        b.reset(cfg, seed=11, counter=counter)
        torch.cuda.synchronize()
        return b

    b = make(0)
    b2 = make(0)
    assert torch.equal(b.rs, b2.rs) and torch.equal(b.obstacles, b2.obstacles) and torch.equal(b.cores, b2.cores)
    b3 = make(1)
    assert not torch.equal(b.rs, b3.rs)
    rs = b.rs.cpu().numpy().reshape(-1, E, R)
    fl = b.rflags.cpu().numpy().reshape(E, R)
    nr = b.n_robots.cpu().numpy()
    no = b.n_obs.cpu().numpy()
    nc = b.n_cores.cpu().numpy()
    assert (b.ep_ts.cpu().numpy() == 0).all()
    assert nr.min() >= 1 and nr.max() <= R and (nr == R).mean() > 0.9
    assert no.max() <= O and (no == O).mean() > 0.9
    assert nc.max() <= Cn and (nc == Cn).mean() > 0.9
    x, y, gx, gy = rs[_abi.F_X], rs[_abi.F_Y], rs[_abi.F_GX], rs[_abi.F_GY]
    core_r = float(b.params.core_r)
    for e in range(0, E, 7):
        n = nr[e]
        assert (fl[e, :n] == 0).all() and (fl[e, n:] == _abi.FLAG_DEACTIVATED).all()
        sx, sy, tx, ty = x[e, :n], y[e, :n], gx[e, :n], gy[e, :n]
        assert (np.hypot(tx - sx, ty - sy) >= 40.0).all()
        for arr in (sx, sy, tx, ty):
            assert ((arr >= 2.0) & (arr <= W - 2.0)).all()
        for vx, vy in ((sx, sy), (tx, ty)):
            d = np.hypot(vx[:, None] - vx[None], vy[:, None] - vy[None])
            assert (d[~np.eye(n, dtype=bool)] > 10.0).all()
        for f in range(_abi.F_VR0, _abi.F_RP + 1):
            assert (rs[f][e, :n] == 0.0).all()
        assert ((rs[_abi.F_THETA][e, :n] >= 0) & (rs[_abi.F_THETA][e, :n] < 2 * np.pi)).all()
        ob = b.obstacles[e, :no[e]].cpu().numpy()
        for (ox, oy, r) in ob:
            assert 5.0 <= ox <= W - 5.0 and 5.0 <= oy <= W - 5.0
            assert (np.hypot(sx - ox, sy - oy) >= r + 10.0).all() and (np.hypot(tx - ox, ty - oy) >= r + 10.0).all()
        if len(ob) > 1:
            d = np.hypot(ob[:, None, 0] - ob[None, :, 0], ob[:, None, 1] - ob[None, :, 1])
            rr = ob[:, None, 2] + ob[None, :, 2]
            assert (d[~np.eye(len(ob), dtype=bool)] > rr[~np.eye(len(ob), dtype=bool)]).all()
        co = b.cores[e, :nc[e]].cpu().numpy()
        for (cx, cy, cw, G) in co:
            assert core_r <= cx <= W - core_r and core_r <= cy <= W - core_r
            assert (np.hypot(sx - cx, sy - cy) >= core_r + 10.0).all()
            assert (np.hypot(tx - cx, ty - cy) >= core_r + 10.0).all()
            assert cw in (0.0, 1.0) and G > 0


@pytest.mark.parametrize("fast", [False, True])
def test_philox_perception_noise_distribution(fast):
    """Philox perception noise (noise_mode 1: f64 draws, 2: f32 draws) follows Perception's
    distributions (wamv.py:27-40): position / velocity noise N(0, 0.05), radius
    0.8 r + 0.2 r vm / pi with vm ~ vonmises(0, kappa=1). 65536 identical one-robot scenes
    with one buoy 5 m ahead, observed once; moments against scipy to a few standard errors."""
    from scipy import stats
    from distributional_rl_decision_and_control_amd import _abi
    from distributional_rl_decision_and_control_amd.device_env import DeviceEnvBatch
    E = 65536
    b = DeviceEnvBatch(E, 1, 1, 0)
    b.rs.zero_()
    b.rs[_abi.F_X].fill_(10.0)
    b.rs[_abi.F_Y].fill_(10.0)
    b.rs[_abi.F_GX].fill_(40.0)
    b.rs[_abi.F_GY].fill_(40.0)
    b.obstacles[:, 0, 0] = 15.0
    b.obstacles[:, 0, 1] = 10.0
    b.obstacles[:, 0, 2] = 1.0
    b.n_robots.fill_(1)
    b.n_obs.fill_(1)
    b.step(None, do_dynamics=False, seed=123, counter=7, fast_noise=fast)
    o = b.obs.double().cpu().numpy()
    assert (b.obj_cnt.cpu().numpy() == 1).all()
    px, py, vx, vy, rr = (o[:, 7 + k] for k in range(5))
    n = len(px)
    for v, mu in ((px, 5.0), (py, 0.0), (vx, 0.0), (vy, 0.0)):
        assert abs(v.mean() - mu) < 4 * 0.05 / np.sqrt(n)
        assert abs(v.std() / 0.05 - 1) < 0.02
    vm_std = stats.vonmises(1.0).std()
    assert abs(rr.mean() - 0.8) < 4 * 0.2 / np.pi * vm_std / np.sqrt(n)
    assert abs(rr.std() / (0.2 / np.pi * vm_std) - 1) < 0.02
    # the full shape of the von Mises draw: KS against scipy
    vm = (rr - 0.8) / 0.2 * np.pi
    assert stats.kstest(vm[:20000], stats.vonmises(1.0).cdf).pvalue > 1e-3
    # f32 draws: the radius comes from the inverse-CDF table at a uniform built from the low bytes of the
    # Gaussians' Philox words -- uncorrelated with each of them (and the KS above over all 65536)
    assert stats.kstest(vm, stats.vonmises(1.0).cdf).pvalue > 1e-3
    for v in (px, py, vx, vy):
        assert abs(np.corrcoef(vm, v)[0, 1]) < 4 / np.sqrt(n)


def test_config5_full_size():
    """BASELINE config 5 at full size: 4096 envs x 17 vehicles (ego + 16), 4 buoys, 110 m map
    (the reference's 55 m map cannot place 17 robots, env.py:33-40,106-120).
    Device reset, 50 Philox (f32 noise, the training path) steps with the trainer bookkeeping, on
    both kernel layouts (pair-parallel and the per-robot sweep must agree bit for bit: same Philox
    substreams, same operation order), then the fused rollout + AC-IQN learn loop (B = 4096,
    N = 32) for a few iterations: every env gets all 17 robots, invariants hold, losses finite."""
    from distributional_rl_decision_and_control_amd import _abi
    from distributional_rl_decision_and_control_amd.device_env import DeviceEnvBatch, reset_cfg
    from distributional_rl_decision_and_control_amd.vec_trainer import VecTrainer
    E, R, O, W = 4096, 17, 4, 110.0

    def run(launch):
        b = DeviceEnvBatch(E, R, O, 0)
        b.reset(reset_cfg(R, O, 0, 40.0, width=W, height=W), seed=5)
        b.step(None, do_dynamics=False, seed=5, counter=0, fast_noise=True, launch=launch)
        g = torch.Generator(device="cuda").manual_seed(4)
        outs = []
        for t in range(50):
            a = (torch.rand((E * R, 2), generator=g, device="cuda", dtype=torch.float64) * 2 - 1).contiguous()
            prev_fl, prev_rs = b.rflags.clone(), b.rs.clone()
            b.step(a, seed=5, counter=t + 1, trainer_deactivate=True, gamma=0.99, fast_noise=True, launch=launch)
            th = b.rs[_abi.F_THETA]
            assert bool(((th >= 0) & (th < 2 * np.pi)).all())
            was_off = (prev_fl & _abi.FLAG_DEACTIVATED) > 0
            assert torch.equal(b.rs[:13][:, was_off], prev_rs[:13][:, was_off])
            cnt = b.obj_cnt.view(E, R)
            assert int(cnt.max().item()) <= 5
            outs.append(torch.cat([b.reward, b.rs[_abi.F_RET], b.obs.reshape(-1).double(),
                                   b.rflags.double(), b.env_done.double()]))
        return b, torch.stack(outs)

    b, o_pairs = run(None)
    assert (b.n_robots.cpu().numpy() == R).all(), "every env must place all 17 robots on the 110 m map"
    assert (b.n_obs.cpu().numpy() == O).all()
    _, o_sweep = run((_abi.ENV_LAYOUT_SWEEP, 0, 0))
    assert torch.equal(o_pairs, o_sweep), "pair-parallel and per-robot-sweep layouts differ"
    # perception keeps up to 5 of the 20 candidates; every count 0..5 occurs at this size
    cnt = b.obj_cnt.cpu().numpy()
    assert all((cnt == k).any() for k in range(6)), np.bincount(cnt[cnt >= 0], minlength=6)

    tr = VecTrainer(n_envs=E, agent_type="AC-IQN", num_robots=R, num_obs=O, width=W, batch_size=4096, num_tau=32,
                    seed=5, buffer_size=E * R * 8)
    while tr.replay_size_host() < tr.learning_starts:
        tr.iteration()
    p0 = torch.cat([p.detach().reshape(-1) for p in tr.local.critic.parameters()]).clone()
    for _ in range(3):
        out = tr.iteration()
    torch.cuda.synchronize()
    losses = [float(x.item()) for x in out[:2]]
    assert np.all(np.isfinite(losses)), losses
    p1 = torch.cat([p.detach().reshape(-1) for p in tr.local.critic.parameters()])
    assert bool(torch.isfinite(p1).all()) and not torch.equal(p0, p1)


CROSS_SHAPES = [(1, 0, 55.0, 0), (1, 3, 55.0, 0), (3, 0, 55.0, 0), (5, 4, 55.0, 2), (12, 8, 110.0, 0),
                (30, 2, 110.0, 0)]


@pytest.mark.parametrize("fast", [True, False])
@pytest.mark.parametrize("R,O,W,C", CROSS_SHAPES)
def test_pair_kernel_matches_sweep(R, O, W, C, fast):
    """The pair kernel (automatic shape, a forced one-wave shape, a 128-lane shape, the step split into launches
    of at most 7 workgroups) against the per-robot sweep, bit
    for bit, over (robots, buoys) shapes the traces do not reach: one robot, no buoys, vortex cores,
    12 and 30 robots (absent robots where the sampler cannot place all). Device reset, Philox noise in
    f32 and f64, 12 steps with the trainer bookkeeping (returns, deactivation, episode end) and one
    masked observation pass over every third env; f32 and f64 observations, state, flags, counts."""
    from distributional_rl_decision_and_control_amd import _abi
    from distributional_rl_decision_and_control_amd.device_env import DeviceEnvBatch, reset_cfg
    E = 300

    def run(launch):
        b = DeviceEnvBatch(E, R, O, C, obs64=True)
        b.reset(reset_cfg(R, O, C, 20.0, width=W, height=W), seed=11)
        b.step(None, do_dynamics=False, seed=11, counter=0, fast_noise=fast, launch=launch)
        g = torch.Generator(device="cuda").manual_seed(3)
        outs = []
        for t in range(12):
            a = (torch.rand((E * R, 2), generator=g, device="cuda", dtype=torch.float64) * 2 - 1).contiguous()
            b.step(a, seed=11, counter=t + 1, trainer_deactivate=True, gamma=0.99, fast_noise=fast, launch=launch)
            outs.append(torch.cat([b.reward, b.rs.reshape(-1), b.obs.reshape(-1).double(), b.obs64.reshape(-1),
                                   b.rflags.double(), b.obj_cnt.double(), b.done.double(), b.info.double(),
                                   b.env_done.double(), b.ep_ts.double()]))
            if t == 5:
                mask = torch.zeros(E, dtype=torch.uint8, device="cuda")
                mask[::3] = 1
                b.step(None, do_dynamics=False, seed=11, counter=100, fast_noise=fast, env_mask=mask, launch=launch)
                outs.append(torch.cat([b.obs.reshape(-1).double(), b.obs64.reshape(-1), b.obj_cnt.double()]))
        return b, outs

    b, ref = run((_abi.ENV_LAYOUT_SWEEP, 0, 0))
    cnt = b.obj_cnt.cpu().numpy()
    assert (cnt >= -1).all() and (cnt <= 5).all()
    # None: automatic; a forced one-wave shape; a 128-lane shape of about 100 robots (which the automatic rule
    # never picks: within 1 % of it at 2^18 envs, profiles/r06af_env_shape_interleaved.txt); the automatic shape as
    # launches of at most 7 workgroups
    for launch in (None, (_abi.ENV_LAYOUT_PAIRS, 64, max(1, 64 // R)), (_abi.ENV_LAYOUT_PAIRS, 128, max(1, 100 // R)),
                   (0, 0, 0, 7)):
        _, got = run(launch)
        for t, (x, y) in enumerate(zip(ref, got)):
            # exact, NaN = NaN: phi is NaN, in both layouts and in the reference, when COLREGs evaluates an
            # object closer than its radius + 1 (asin of a ratio > 1, wamv.py:388); it never enters a reward
            torch.testing.assert_close(x, y, rtol=0, atol=0, equal_nan=True,
                                       msg=f"layout {launch} differs from the sweep at output {t}")


@pytest.mark.parametrize("R,O,Cn,W,obs_r,v", [(5, 4, 0, 55.0, (1.0, 1.0), (3.0, 3.0)),
                                              (5, 4, 3, 55.0, (0.5, 3.0), (2.0, 4.0)),
                                              (17, 4, 0, 110.0, (1.0, 1.0), (3.0, 3.0)),
                                              (8, 12, 4, 80.0, (0.5, 2.5), (1.0, 5.0))])
def test_device_reset_matches_sequential_restatement(R, O, Cn, W, obs_r, v):
    """asvrl_env_reset evaluates a wave of 64 candidates at a time and accepts in candidate order; the
    C oracle (or_device_reset) restates the same sampler one candidate at a time, as MarineNavEnv3.reset
    draws them (env.py:106-162). Bit-identical robots (start, goal, heading), cores and obstacles on
    every env, for a full reset and for a masked reset at a device counter (the training loop's
    auto-reset), where the envs outside the mask must stay untouched."""
    from oracle import env_oracle as eo
    from distributional_rl_decision_and_control_amd import _abi
    from distributional_rl_decision_and_control_amd.device_env import DeviceEnvBatch, reset_cfg
    E = 384
    cfg = reset_cfg(R, O, Cn, 30.0, width=W, height=W, obs_r_range=obs_r, v_range=v)
    b = DeviceEnvBatch(E, R, O, max(Cn, 1))
    core_r = float(b.params.core_r)

    def check(envs, seed, counter):
        rs = b.rs.cpu().numpy().reshape(-1, E, R)
        nr, nc, no = b.n_robots.cpu().numpy(), b.n_cores.cpu().numpy(), b.n_obs.cpu().numpy()
        cores, obst, fl = b.cores.cpu().numpy(), b.obstacles.cpu().numpy(), b.rflags.cpu().numpy().reshape(E, R)
        for e in envs:
            rob, cor, ob = eo.device_reset(cfg, core_r, R, O, max(Cn, 1), seed, counter, int(e))
            n = len(rob)
            assert nr[e] == n and nc[e] == len(cor) and no[e] == len(ob), e
            got = np.stack([rs[_abi.F_X][e, :n], rs[_abi.F_Y][e, :n], rs[_abi.F_GX][e, :n], rs[_abi.F_GY][e, :n],
                            rs[_abi.F_THETA][e, :n]], axis=1)
            np.testing.assert_array_equal(got, rob)
            np.testing.assert_array_equal(cores[e, :len(cor)], cor)
            np.testing.assert_array_equal(obst[e, :len(ob)], ob)
            assert (fl[e, n:] == _abi.FLAG_DEACTIVATED).all() and (fl[e, :n] == 0).all()

    b.reset(cfg, seed=21, counter=5)
    torch.cuda.synchronize()
    check(range(E), 21, 5)
    # masked, counter partly on the device: the key and counter of the envs reset now are (5 + 7 + 2^33)
    mask = (torch.arange(E, device="cuda") % 3 == 1).to(torch.uint8)
    before = b.rs.clone()
    cdev = torch.tensor([7 + (1 << 33)], dtype=torch.int64, device="cuda")
    b.reset(cfg, mask, seed=21, counter=5, counter_dev=cdev)
    torch.cuda.synchronize()
    m = mask.cpu().numpy().astype(bool)
    rs0, rs1 = before.cpu().numpy().reshape(-1, E, R), b.rs.cpu().numpy().reshape(-1, E, R)
    np.testing.assert_array_equal(rs0[:, ~m], rs1[:, ~m])
    check(np.nonzero(m)[0], 21, 5 + 7 + (1 << 33))


@pytest.mark.parametrize("R,O,Cn,W", [(5, 4, 0, 55.0), (5, 4, 2, 55.0), (17, 4, 0, 110.0)])
def test_fused_auto_reset_matches_two_launches(R, O, Cn, W):
    """VecMarineNavEnv.auto_reset in one launch (asvrl_env_reset_observe: per ended env, the reset sampler
    then that env's reset observation) against the two-launch form (asvrl_env_reset + the masked
    do_dynamics = 0 asvrl_env_step over every env): bit-identical env state, observation rows, object counts
    and per-robot outputs, with the counter on the device as in the captured training loop."""
    from distributional_rl_decision_and_control_amd.vec_env import VecMarineNavEnv
    E = 512
    envs = []
    for fused in (True, False):
        v = VecMarineNavEnv(E, num_robots=R, num_obs=O, num_cores=Cn, width=W, seed=9, max_cores=max(Cn, 1))
        v.fused_reset = fused
        v.reset()
        envs.append(v)
    g = torch.Generator(device="cuda").manual_seed(4)
    for t in range(6):
        a = torch.rand((E * R, 2), generator=g, device="cuda", dtype=torch.float64) * 2 - 1
        done = (torch.rand(E, generator=g, device="cuda") < 0.3).to(torch.uint8)
        for v in envs:
            v.step(a)
            v.batch.env_done.copy_(done)   # a third of the envs end their episode
            v.auto_reset(counted=t % 2 == 1)
            v.advance_device(counted=t % 2 == 1)
        torch.cuda.synchronize()
        f, s = envs
        for name in ("rs", "rflags", "n_robots", "n_obs", "n_cores", "ep_ts", "obstacles", "cores", "reward", "done",
                     "info"):
            assert torch.equal(getattr(f.batch, name), getattr(s.batch, name)), (t, name)
        assert torch.equal(f.obs_cur, s.obs_cur) and torch.equal(f.cnt_cur, s.cnt_cur), t
