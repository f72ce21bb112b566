"""CPU: the rollout oracle (oracle/rollout_oracle.py) against fixtures produced by
the reference's own SB3 (tests/golden/gen_rollout_golden.py)."""
import numpy as np
import pytest

import _fixtures as F
from oracle import rollout_oracle as R

CASES = ["a", "b", "c", "d"]


@pytest.mark.parametrize("case", CASES)
def test_gae_oracle_is_bit_exact_vs_reference(case):
    d = F.load("rollout_gae.npz")
    g = lambda k: d[case + "__" + k]
    # the stored `dones` column is the episode-start flag passed to add()
    assert np.array_equal(g("dones_stored"), g("starts").astype(np.float32))
    adv, ret = R.gae(g("rewards"), g("values"), g("starts"), g("last_values"), g("last_dones"), float(g("gamma")),
                     float(g("lam")))
    assert adv.dtype == np.float32 and ret.dtype == np.float32
    assert np.array_equal(adv, g("advantages"))
    assert np.array_equal(ret, g("returns"))
    assert np.array_equal(R.swap_and_flatten(adv).ravel(), g("flat_advantages"))


def test_vecnormalize_oracle_matches_reference():
    d = F.load("vecnormalize.npz")
    n, dim = d["obs"].shape[1:]
    v = R.VecNormalizeOracle(n, dim, gamma=float(d["gamma"]), clip_obs=float(d["clip_obs"]),
                             clip_reward=float(d["clip_reward"]), epsilon=float(d["epsilon"]))
    o0 = v.reset(d["obs"][0])
    assert np.array_equal(o0, d["norm_obs0"])
    for k in range(len(d["rew"])):
        o, r = v.step(d["obs"][k + 1], d["rew"][k], d["done"][k].astype(bool))
        assert np.array_equal(o, d["norm_obs"][k])
        assert np.array_equal(r, d["norm_rew"][k])
        assert np.array_equal(v.state(), d["rms"][k])


def test_chan_merge_equals_concatenated_batch():
    """The sharded statistic: merging per-shard (n, mean, M2) in rank order == np.mean/np.var of the whole batch."""
    rng = np.random.RandomState(3)
    x = rng.randn(1000, 14) * rng.uniform(0.1, 50, 14) + 7
    shards = np.array_split(x, 4)
    recs = [(len(s), s.mean(0), ((s - s.mean(0)) ** 2).sum(0)) for s in shards]
    n, mean, m2 = R.chan_merge(recs)
    assert n == 1000
    np.testing.assert_allclose(mean, x.mean(0), rtol=1e-13, atol=1e-12)
    np.testing.assert_allclose(m2 / n, x.var(0), rtol=1e-12)
