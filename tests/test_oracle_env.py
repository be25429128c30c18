"""Pins the CPU oracle (the parity checker) against the reference's own known-answer tests.

Reference KATs restated here:
  mechanics.rs:659-675  ball_collision_test_left_wall   (3 rstest cases, exact assert_eq)
  mechanics.rs:677-693  ball_collision_test_right_wall  (3 cases, exact)
  mechanics.rs:708-752  ball_collision_test_rectangle   (7 cases; tol 0.01 normals, 0.1 way, approx in [0, 0.8))
  self_driving_tf_q_learner.rs:345-361 generate_distinct_random_ids (distinct, in range, 100 repeats)
plus Random123's published Philox4x32-10 known-answer vectors for the build's bit source.
"""
import math

import numpy as np
import pytest

import oracle as O

GRID = 600.0


@pytest.mark.parametrize("center,radius,mv,expected", [
    ((10.0, 10.0), 5.0, (-2.0, 2.0), None),
    ((5.0, 10.0), 5.0, (-5.0, 0.0), (0.0, 0.0, 1.0, 0.0)),
    ((7.0, 7.0), 5.0, (-5.0, 0.0), (2.0, 0.0, 1.0, 0.0)),
])
def test_kat_left_wall(center, radius, mv, expected):
    assert O.wall_left(center, radius, mv) == expected


@pytest.mark.parametrize("center,radius,mv,expected", [
    ((GRID - 10.0, 10.0), 5.0, (2.0, 2.0), None),
    ((GRID - 5.0, 10.0), 5.0, (5.0, 0.0), (0.0, 0.0, -1.0, 0.0)),
    ((GRID - 7.0, 7.0), 5.0, (5.0, 0.0), (2.0, 0.0, -1.0, 0.0)),
])
def test_kat_right_wall(center, radius, mv, expected):
    assert O.wall_right(center, radius, mv) == expected


S2 = 1.0 / math.sqrt(2.0)


@pytest.mark.parametrize("center,radius,mv,lo,hi,expected", [
    ((100.0, 100.0), 5.0, (10.0, 0.0), (150.0, 90.0), (170.0, 110.0), None),
    ((100.0, 100.0), 5.0, (5.0, 0.0), (110.0, 90.0), (130.0, 110.0), (5.0, -1.0, 0.0)),
    ((100.0, 100.0), 5.0, (3.0, -3.0), (100.0, 70.0), (120.0, 93.0), (2.83, 0.0, 1.0)),
    ((100.0, 100.0), 5.0, (-8.0, -8.0), (70.0, 80.0), (90.0, 100.0), (7.07, 1.0, 0.0)),
    ((100.0, 100.0), 5.0, (-1.46, -1.46), (80.0, 80.0), (95.0, 95.0), (2.07, S2, S2)),
    ((100.0, 100.0), 5.0, (-5.0, -5.0), (80.0, 80.0), (95.0, 95.0), (2.07, S2, S2)),
    ((100.0, 100.0), 5.0, (-4.2, -4.2), (80.0, 80.0), (90.0, 90.0), None),
])
def test_kat_rectangle(center, radius, mv, lo, hi, expected):
    got = O.rect_check(center, radius, mv, lo, hi)
    assert (got is None) == (expected is None)
    if got is not None:
        way, approx, nx, ny = got
        assert abs(nx - expected[1]) <= 0.01
        assert abs(ny - expected[2]) <= 0.01
        assert abs(way - expected[0]) <= 0.1
        assert 0.0 <= approx < 0.8


def test_philox_known_answers():
    # Random123 kat_vectors: philox4x32 10 <ctr x4> <key x2> <expected x4>
    kats = [
        ([0, 0, 0, 0], [0, 0], [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]),
        ([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2, [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]),
        ([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0],
         [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]),
    ]
    for ctr, key, exp in kats:
        assert list(O.philox(ctr, key)) == exp


def test_distinct_random_ids_property_100x():
    # self_driving_tf_q_learner.rs:345-361: 50 of 0..100, distinct and in range, repeated 100 times
    for rep in range(100):
        r = O.sample_distinct(seed=7, update_idx=rep, rank=0, length=100, B=50)
        assert len(set(r.tolist())) == 50
        assert all(0 <= v < 100 for v in r.tolist())


def test_rand_derivations_ranges():
    L = O.lib()
    vals = [L.orc_gen_range_f32(3, i, 0, 1, -0.35, -0.15) for i in range(2000)]
    assert all(-0.35 <= np.float32(v) < np.float32(-0.15) for v in vals)
    assert abs(np.mean(vals) + 0.25) < 0.01
    f = [L.orc_gen_f64_01(3, i, 0, 2) for i in range(2000)]
    assert all(0.0 <= v < 1.0 for v in f)
    a = [L.orc_gen_u8(3, i, 0, 2, 2, 3) for i in range(3000)]
    counts = np.bincount(a, minlength=3)
    assert counts.sum() == 3000 and counts.min() > 900


def test_env_initial_state_matches_constants():
    env = O.Env(seed=5)
    s = env.state()
    assert (s["ball_x"], s["ball_y"]) == (300.0, 300.0)
    assert -0.35 <= s["dir_x"] < -0.15 and s["dir_y"] == -1.0
    assert (s["panel_min_x"], s["panel_min_y"], s["panel_max_x"], s["panel_max_y"]) == (270.0, 565.0, 330.0, 575.0)
    assert s["bricks"] == (1 << 60) - 1 and s["score"] == 0 and s["finished"] == 0
    assert not env.tensor().any()   # FrameRingBuffer::new is all zeros


def test_env_episode_runs_and_frame_ring():
    env = O.Env(seed=11)
    total, steps, done = 0.0, 0, False
    slots = []
    while not done and steps < 5000:
        slots.append(int(env.state()["next_slot"]))
        r, done = env.step(steps % 3)
        total += r
        steps += 1
        assert r in (0.0, 1.0, 2.0, 3.0)
    assert done, "ball must eventually leave past the panel"
    assert slots[:8] == [0, 1, 2, 3, 0, 1, 2, 3]
    s = env.state()
    assert s["fault"] == 0
    assert total == s["score"] == 60 - bin(int(s["bricks"])).count("1")
    vals = set(np.unique(env.tensor()).tolist())
    assert vals <= {0, 96, 236, 255}
    env.reset()
    assert int(env.state()["reset_count"]) == 1 and not env.tensor().any()


def test_panel_dynamics_quirks():
    env = O.Env(seed=1)
    env.step(2)                      # accelerate right -> speed 20
    assert env.state()["panel_speed"] == 20.0
    for _ in range(10):
        env.step(2)
    assert env.state()["panel_speed"] == 160.0    # PANEL_MAX_SPEED clamp
    env.step(0)
    assert env.state()["panel_speed"] == 153.0    # slow down by 7
    for _ in range(12):
        env.step(1)
    assert env.state()["panel_speed"] < 0
    env.step(0)
    # decrease_speed clamps negative speeds to 0 via .max(0.0) (mechanics.rs:624) — reference quirk kept
    assert env.state()["panel_speed"] == 0.0


def test_acos_threshold_is_tiny_negative():
    t = O.lib().orc_acos_threshold()
    assert -1e-6 < t < 0.0
    assert math.acos(np.float32(t)) <= np.float32(math.pi / 2) + 1e-7
