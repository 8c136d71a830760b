"""Controller-tick oracle (oracle/controller_ref.py) pinned by analytic identities.

The reference has no tests for controller.cpp and Eigen/ROS are absent here, so
the restatement is checked against independent float64 math (rotation
matrices) and the observation layout SURVEY.md §8a derives from
controller.cpp:200-212 / controller.hpp:45-68.
"""
import numpy as np
import pytest

from oracle import controller_ref as cr


def rotmat(q):
    """float64 body->world rotation matrix of unit quaternions (w,x,y,z)."""
    w, x, y, z = (q[:, i].astype(np.float64) for i in range(4))
    return np.stack([
        np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)], -1),
        np.stack([2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)], -1),
        np.stack([2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], -1),
    ], 1)


def test_gravity_identity_and_zero_quaternion():
    q = np.array([[1, 0, 0, 0], [0, 0, 0, 0]], np.float32)
    g = cr.gravity_b(q)
    assert np.array_equal(g[0], np.array([0, 0, -1], np.float32))
    # Eigen's inverse() of a zero quaternion is the zero quaternion: q * v = v
    assert np.array_equal(g[1], np.array([0, 0, -1], np.float32))


def test_gravity_axis_rotations():
    s = np.sqrt(0.5)
    q = np.array([[s, s, 0, 0], [s, 0, s, 0], [s, 0, 0, s], [0, 1, 0, 0]], np.float32)
    g = cr.gravity_b(q)
    # R^T (0,0,-1): roll +90 -> (0,-1,0); pitch +90 -> (1,0,0); yaw keeps it; roll 180 -> (0,0,1)
    want = np.array([[0, -1, 0], [1, 0, 0], [0, 0, -1], [0, 0, 1]], np.float64)
    np.testing.assert_allclose(g, want, atol=2e-7)


def test_gravity_random_unit_quaternions_vs_rotation_matrix():
    rng = np.random.default_rng(7)
    q = rng.normal(size=(2000, 4))
    q = (q / np.linalg.norm(q, axis=1, keepdims=True)).astype(np.float32)
    g = cr.gravity_b(q)
    ref = np.einsum("bji,j->bi", rotmat(q), np.array([0, 0, -1.0]))  # R^T g_w
    np.testing.assert_allclose(g, ref, atol=2e-6)


def test_history_layout_matches_survey():
    """Two ticks with known signals land where SURVEY §8a says: each block [t-1, t]."""
    B, H = 2, 2
    rng = np.random.default_rng(1)
    obs = np.zeros((B, 98), np.float32)
    act = np.zeros((B, 12), np.float32)
    st1, st2 = cr.synthetic_states(rng, B), cr.synthetic_states(rng, B)
    a_prev = rng.normal(size=(B, 12)).astype(np.float32)
    o1, _ = cr.assemble_obs(obs, act, st1, None, H)
    o2, _ = cr.assemble_obs(o1, a_prev, st2, None, H)
    g1, g2 = cr.gravity_b(st1[:, :4]), cr.gravity_b(st2[:, :4])
    assert np.array_equal(o2[:, 0:3], g1) and np.array_equal(o2[:, 3:6], g2)
    assert np.array_equal(o2[:, 6:9], st1[:, 4:7]) and np.array_equal(o2[:, 9:12], st2[:, 4:7])
    assert np.array_equal(o2[:, 12:18], np.zeros((B, 6), np.float32))  # no joystick yet: cmd stays 0
    q2 = (st2[:, 7:19].astype(np.float64) - cr.Q0).astype(np.float32)
    assert np.array_equal(o2[:, 30:42], q2)
    assert np.array_equal(o2[:, 42:54], st1[:, 19:31]) and np.array_equal(o2[:, 54:66], st2[:, 19:31])
    assert np.array_equal(o2[:, 66:78], act) and np.array_equal(o2[:, 78:90], a_prev)
    c2 = (st2[:, 31:35][:, [1, 0, 3, 2]] >= 22).astype(np.float32)
    assert np.array_equal(o2[:, 94:98], c2)


@pytest.mark.parametrize("H", [1, 3])
def test_history_generalises(H):
    B = 3
    rng = np.random.default_rng(H)
    obs = rng.normal(size=(B, 49 * H)).astype(np.float32)
    act = rng.normal(size=(B, 12)).astype(np.float32)
    st = cr.synthetic_states(rng, B)
    new, _ = cr.assemble_obs(obs, act, st, None, H)
    cum = 0
    for (_, d) in cr.BLOCKS:
        s = H * cum
        assert np.array_equal(new[:, s:s + (H - 1) * d], obs[:, s + d:s + H * d])
        cum += d
    s_act = H * 33 + (H - 1) * 12
    assert np.array_equal(new[:, s_act:s_act + 12], act)


def test_vel_cmd_sticky_and_formula():
    prev = np.array([[0.1, 0.2, 0.3], [0.4, 0.5, 0.6]], np.float32)
    joy = np.array([[1, -0.5, 0.7, 0.25, 0], [0, 0.9, 0.9, 0.9, 0]], np.float32)
    c = cr.vel_cmd(joy, prev)
    assert c[0, 0] == np.float32(0.7)
    assert c[0, 1] == np.float32(0.25 * 0.8 * -1)  # pow(-0.5, 2) * -1 * 0.8 in double
    assert c[0, 2] == np.float32(0.25) * np.float32(0.7)
    assert np.array_equal(c[1], prev[1])  # no axes: previous command kept
    assert np.array_equal(cr.vel_cmd(None, prev), prev)


def test_post_process_clamp_stop_and_gains():
    y = np.array([[2000.0, -5000.0] + [0.5] * 10, [1.0] * 12], np.float32)
    joy = np.array([[1, 0, 0, 0, 0], [1, 0, 0, 0, 1]], np.float32)
    a, q_des, kp, kd = cr.post_process(y, joy)
    assert a[0, 0] == 1000 and a[0, 1] == -1000 and a[0, 2] == np.float32(0.5)
    assert np.all(a[1] == 0)
    np.testing.assert_array_equal(q_des[1], cr.Q0)
    assert q_des[0, 2] == cr.Q0[2] + 0.5 * 0.25
    assert np.all(kp[0] == 28.0) and np.all(kp[1] == 5.0) and np.all(kd == 0.5)
    nan = np.full((1, 12), np.nan, np.float32)
    assert np.all(np.isnan(cr.post_process(nan, None)[0]))  # std::clamp passes NaN through


def test_nan_status_only_for_checked_blocks():
    rng = np.random.default_rng(3)
    B = 4
    st = cr.synthetic_states(rng, B)
    obs = np.zeros((B, 98), np.float32)
    act = np.zeros((B, 12), np.float32)
    st[1, 5] = np.nan     # gyro
    act[2, 3] = np.nan    # previous action
    st[3, 33] = np.nan    # foot force: compared, never NaN in the observation
    _, status = cr.assemble_obs(obs, act, st, None, 2)
    assert status.tolist() == [0, 1, 1, 0]


def test_tick_composes():
    rng = np.random.default_rng(5)
    B = 5
    st, joy = cr.synthetic_states(rng, B), cr.synthetic_joy(rng, B)
    obs = np.zeros((B, 98), np.float32)
    act = np.zeros((B, 12), np.float32)
    W = rng.normal(size=(98, 12)).astype(np.float32)
    o, a, q_des, kp, kd, status = cr.tick(lambda x: x @ W, st, joy, obs, act, 2)
    a2, *_ = cr.post_process(o @ W, joy)
    assert np.array_equal(a, a2) and not status.any()
