"""Oracle checks for double DQN + prioritized replay (beyond the reference, so parity with the
reference is not applicable: these pin the oracle's restatement of the published algorithms by their properties).

Proportional prioritized replay (Schaul et al. 2016, stratified sampling, IS weights (N P(i))^-beta / max):
  - the f32 heap total equals a pairwise f32 restatement in numpy, bit for bit;
  - stratified draws are non-decreasing in the sample index and land in the sample's own segment of the
    prefix sums; zero leaves are never drawn; equal leaves give IS weights of exactly 1;
  - IS weights follow (len p_i / T)^-beta normalised by the batch max (rtol 1e-6).
Double DQN (van Hasselt et al. 2016): with identical samples, y_ddqn <= y_dqn for every non-terminal sample
(Q_target(s', argmax Q_online) <= max Q_target) and equal for terminal ones.
"""
import numpy as np

import oracle as O


def heap_total(leaves):
    L = 1
    while L < len(leaves):
        L *= 2
    lvl = np.zeros(L, np.float32)
    lvl[:len(leaves)] = leaves
    while lvl.shape[0] > 1:
        lvl = (lvl[0::2] + lvl[1::2]).astype(np.float32)
    return lvl[0]


def test_sumtree_total_and_uniform_weights():
    for cap in (1, 2, 3, 1000, 4097):
        leaves = np.ones(cap, np.float32)
        slots, w, total = O.per_sample(leaves, 5, 0, 2, 0, cap, 0.4, 16)
        assert total == np.float32(cap)
        assert (slots < cap).all() and (w == 1.0).all()


def test_stratified_draws_follow_prefix_sums():
    rng = np.random.default_rng(1)
    cap, length, B = 3000, 2500, 256
    leaves = np.zeros(cap, np.float32)
    leaves[:length] = rng.gamma(0.5, 1.0, length).astype(np.float32) ** 0.6
    leaves[rng.integers(0, length, 300)] = 0.0
    slots, w, total = O.per_sample(leaves, 11, 40, 3, 1, length, 0.4, B)
    assert total == heap_total(leaves)
    cs = np.cumsum(leaves.astype(np.float64))
    for u in range(3):
        s = slots[u].astype(np.int64)
        assert (np.diff(s) >= 0).all()
        assert (leaves[s] > 0).all() and (s < length).all()
        lo = np.where(s > 0, cs[s - 1], 0.0)
        seg = total / B
        # the segment [b seg, (b+1) seg) overlaps the leaf's prefix interval [lo, lo + leaf) (f32 slack)
        b = np.arange(B)
        assert (lo <= (b + 1) * seg * (1 + 1e-5) + 1e-5).all() and (cs[s] >= b * seg * (1 - 1e-5) - 1e-5).all()
        p = leaves[s].astype(np.float64) / total
        wr = (length * p) ** -0.4
        assert np.allclose(w[u], wr / wr.max(), rtol=1e-5)
        assert w[u].max() == 1.0


def test_det_powf_accuracy():
    """det_powf (the x^y both sides of the prioritized replay evaluate) against the correctly rounded
    float32 of the binary64 power: within one ulp everywhere, equal almost everywhere; the edge values of powf."""
    rng = np.random.default_rng(7)
    n = 400_000
    x = np.concatenate([rng.random(n // 4) * 3 + 1e-6,                       # |td| + eps
                        np.exp(rng.uniform(-20, 20, n // 4)),                # wide magnitudes
                        rng.uniform(1e-3, 4096.0, n // 4),                   # len p of the IS weights
                        rng.integers(1, 1 << 20, n // 4).astype(np.float64)]).astype(np.float32)
    y = np.concatenate([np.full(n // 4, 0.6), rng.uniform(-3, 3, n // 4), np.full(n // 4, -0.4),
                        rng.uniform(-1, 1, n // 4)]).astype(np.float32)
    got = O.det_powf(x, y)
    ref = np.power(x.astype(np.float64), y.astype(np.float64))
    ok = np.isfinite(ref) & (ref < 3e38) & (ref > 1e-37)
    exp32 = ref[ok].astype(np.float32)
    ulps = np.abs(got[ok].view(np.int32).astype(np.int64) - exp32.view(np.int32).astype(np.int64))
    assert ulps.max() <= 1, ulps.max()
    assert (ulps == 0).mean() > 0.999, (ulps == 0).mean()
    e = O.det_powf(np.array([0, 0, 0, 1, 2, np.inf, np.inf, np.nan, -1], np.float32),
                   np.array([0.6, -0.4, 0, 0.6, 0, 1, -1, 1, 0.5], np.float32))
    assert e[0] == 0 and np.isinf(e[1]) and e[2] == 1 and e[3] == 1 and e[4] == 1
    assert np.isinf(e[5]) and e[6] == 0 and np.isnan(e[7]) and np.isnan(e[8])


def test_high_priority_dominates():
    cap, B = 512, 512
    leaves = np.full(cap, 1e-3, np.float32)
    leaves[77] = 100.0
    slots, w, _ = O.per_sample(leaves, 3, 0, 1, 0, cap, 1.0, B)
    frac = (slots[0] == 77).mean()
    assert frac > 0.98, frac
    # the over-sampled transition carries the smallest IS weight
    assert w[0][slots[0] == 77].max() == w[0].min()


def _learner(flags, **kw):
    p = dict(n_envs=8, batch_size=16, history_buffer_len=400, update_after_actions=8, epsilon_pure_random_steps=50_000,
             max_steps_per_episode=60, target_sync_steps=64, flags=flags)
    p.update(kw)
    return O.Learner(O.default_params(**p))


def test_double_dqn_targets_bounded_by_dqn():
    a, b = _learner(0), _learner(O.DOUBLE_DQN)
    n = 0
    for v in range(10):
        a.vector_step()
        b.vector_step()
        ra, rb = a.last(), b.last()
        assert np.array_equal(ra["indices"], rb["indices"])   # sampling is unchanged by double DQN
        if v == 0:
            continue
        if len(ra["losses"]) and v < 8:   # before the first target sync both target nets are the initial weights
            n += len(ra["losses"])
            assert (rb["targets"] <= ra["targets"] + 1e-6).all()
    assert n > 0


def test_prioritized_replay_learner_bookkeeping():
    L = _learner(O.PER, per_alpha=0.6, per_beta=0.4, per_eps=1e-6)
    seen_first = False
    for v in range(12):
        L.vector_step()
        r = L.last()
        w, leaves, pmax = L.priorities()
        c = L.counters()
        if not len(r["losses"]):
            continue
        if not seen_first:   # every stored transition entered at priority 1: uniform draws, unit weights
            assert (w == 1.0).all()
            seen_first = True
        assert ((w > 0) & (w <= 1)).all() and (w.max(axis=1) == 1.0).all()
        assert (r["indices"] < c["replay_len"]).all()
        # every drawn slot holds (|td| + eps)^alpha - or max priority if a later push overwrote it
        assert (leaves[:c["replay_len"]] > 0).all() and (leaves[c["replay_len"]:] == 0).all()
        assert pmax >= leaves.max() - 1e-7
    assert seen_first
