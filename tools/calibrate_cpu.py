#!/usr/bin/env python3
"""CPU-baseline calibration: the reference's own MarineNavEnv3.step loop vs the
oracle's C port of it, both single-threaded on the same workload, in the build container.

Runs ONLY here, where the read-only reference is mounted at /root/reference (it imports the reference's
Python code). Writes profiles/r04_cpu_calibration.json (--out), which bench.py's cpu_baseline leg reads to
state what its C-port number means in reference-Python terms. Nothing on the GPU box reads the
reference.

Workload (the harness SURVEY.md section 8d describes): MarineNavEnv3(seed=s) with 5 robots, 4 buoys,
no cores, min_start_goal_dis 40 on the 55 m map; uniform(-1, 1) continuous actions; a robot is
deactivated after a collision or reaching its goal (trainer.py:168-170); the env is reset when all are
deactivated or after 1000 steps (trainer.py:172). The C port (oracle/asv_oracle.c or_batch_rollout)
runs the same loop, including its resets.

    PYTHONDONTWRITEBYTECODE=1 python3 -W ignore tools/calibrate_cpu.py [--seconds 10]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/rfarl"


def reference_rate(seconds):
    sys.path.insert(0, REF)
    sys.dont_write_bytecode = True
    from rfarl.envs.marinenav.env import MarineNavEnv3
    steps, resets, seed = 0, 0, 0
    rng = np.random.RandomState(1)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        env = MarineNavEnv3(seed=seed)
        env.num_robots, env.num_cores, env.num_obs, env.min_start_goal_dis = 5, 0, 4, 40.0
        env.reset()
        resets += 1
        seed += 1
        while time.perf_counter() - t0 < seconds:
            acts = [None if r.deactivated else list(rng.uniform(-1, 1, 2)) for r in env.robots]
            env.step(acts, True)
            steps += 1
            for r in env.robots:
                if r.collision or r.reach_goal:
                    r.deactivated = True
            if env.check_all_deactivated() or env.episode_timesteps >= 1000:
                break
    el = time.perf_counter() - t0
    return steps / el, steps, resets, el


def port_rate(seconds):
    sys.path.insert(0, ROOT)
    from oracle import env_oracle as eo
    eo.build()
    E = 16
    t0 = time.perf_counter()
    n, _ = eo.batch_rollout(E, 5, 4, 64, seed=3, threads=1)
    probe = time.perf_counter() - t0
    S = max(64, int(64 * seconds / max(probe, 1e-3)))
    t0 = time.perf_counter()
    n, _ = eo.batch_rollout(E, 5, 4, S, seed=4, threads=1)
    el = time.perf_counter() - t0
    return n / el, n, el


def numpy_rate(seconds):
    """oracle/env_numpy.py (the per-robot NumPy restatement bench.py times on the GPU box), same loop."""
    sys.path.insert(0, ROOT)
    from oracle import env_numpy as en
    n, el = en.rollout(seconds, seed=0)
    return n / el, n, el


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--out", default="r04_cpu_calibration.json")
    a = ap.parse_args()
    ref, ref_n, resets, ref_s = reference_rate(a.seconds)
    port, port_n, port_s = port_rate(a.seconds)
    npr, np_n, np_s = numpy_rate(a.seconds)
    out = {"workload": "MarineNavEnv3.step, 5 robots, 4 buoys, 55 m map, uniform actions, trainer deactivation, "
                       "reset on all-deactivated / 1000 steps",
           "reference_python_env_steps_per_s_1thread": ref, "reference_steps": ref_n, "reference_resets": resets,
           "reference_seconds": ref_s,
           "c_port_env_steps_per_s_1thread": port, "c_port_steps": port_n, "c_port_seconds": port_s,
           "c_port_over_reference": port / ref,
           "numpy_restatement_env_steps_per_s_1thread": npr, "numpy_restatement_steps": np_n,
           "numpy_restatement_seconds": np_s, "numpy_restatement_over_reference": npr / ref,
           "host": f"build container, {os.cpu_count()} CPUs, 1 thread each",
           "python": sys.version.split()[0], "numpy": np.__version__}
    path = os.path.join(ROOT, "profiles", a.out)
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
