"""CPU: the F9b fixture (tests/golden/eval_iqn_ref.npz, tools/capture_oracle.capture_eval_iqn) is self-consistent:
one recorded act_iqn call per active robot and step, in the reference's (config, step, robot) order, whose
actions are the robots' recorded action histories, and whose taus are valid quantile fractions (U[0, 1))."""
import numpy as np

from oracle import env_oracle as eo


def test_iqn_eval_fixture_calls_match_action_histories():
    z = np.load(eo.GOLDEN + "/eval_iqn_ref.npz")
    p = "IQN/"
    keys, acts, taus = z[p + "calls/key"], z[p + "calls/action"], z[p + "calls/taus"]
    assert taus.shape == (len(keys), 32) and taus.dtype == np.float32
    assert (taus >= 0).all() and (taus < 1).all()
    # (config, step, robot) strictly increasing in the sequential evaluation's order
    order = keys[:, 0].astype(np.int64) * 10 ** 8 + keys[:, 1].astype(np.int64) * 100 + keys[:, 2]
    assert (np.diff(order) > 0).all()
    for e in range(int(keys[:, 0].max()) + 1):
        robots = sorted(int(k.split("/")[-1]) for k in z.files if k.startswith(f"{p}act/{e}/"))
        for i in robots:
            sel = (keys[:, 0] == e) & (keys[:, 2] == i)
            np.testing.assert_array_equal(acts[sel].astype(np.float64), z[f"{p}act/{e}/{i}"].reshape(-1))
