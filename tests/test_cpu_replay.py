"""ObservationAction log format + replay harness, host side.

The fixture tests/golden/replay_bag is a rosbag2 sqlite3 bag of
/observation_action written by tests/golden/make_replay_log.py (a synthetic
closed-loop run of the oracle controller tick: the reference ships no recorded
data). The message layout is pinned by the .msg definition
(onnx_interfaces/msg/ObservationAction.msg:1-2) and CDR's fixed-array rules.
"""
import os
import struct

import numpy as np
import pytest

from conftest import GOLDEN

BAG = os.path.join(GOLDEN, "replay_bag")


def test_cdr_layout_matches_hand_packed_message():
    from go2_onnx_controller_amd import replay
    rng = np.random.default_rng(0)
    o = rng.normal(size=98).astype(np.float32)
    a = rng.normal(size=12).astype(np.float32)
    raw = b"\x00\x01\x00\x00" + struct.pack("<98f", *o) + struct.pack("<12f", *a)
    assert replay.encode_cdr(o, a) == raw
    o2, a2 = replay.decode_cdr(raw)
    assert np.array_equal(o2, o) and np.array_equal(a2, a)
    be = b"\x00\x00\x00\x00" + struct.pack(">98f", *o) + struct.pack(">12f", *a)
    o3, a3 = replay.decode_cdr(be)
    assert np.array_equal(o3, o) and np.array_equal(a3, a)
    with pytest.raises(ValueError):
        replay.decode_cdr(raw[:100])
    with pytest.raises(ValueError):
        replay.decode_cdr(b"\x01\x07" + raw[2:])


def test_fixture_bag_reads_and_is_consistent():
    from go2_onnx_controller_amd import replay
    log = replay.read_log(BAG)
    assert log.observation.shape == (80, 98) and log.action.shape == (80, 12)
    assert np.all(np.diff(log.t_ns) > 0)
    assert replay.history_breaks(log).size == 0
    assert np.all(log.action[40:46] == 0) and np.all(np.any(log.action[:40] != 0, axis=1))
    assert np.all(log.observation[:5, 12:18] == 0)  # no joystick axes yet: vel_cmd stays 0


def test_fixture_matches_the_oracle_policy():
    """Pins the fixture: the fp64 oracle policy + clamp reproduces every logged
    action that the stop button did not zero, bit for bit."""
    from go2_onnx_controller_amd import replay
    from oracle import mlp_ref
    log = replay.read_log(BAG)
    y = mlp_ref.MlpRef.from_onnx(os.path.join(GOLDEN, "model.onnx")).f64(log.observation)
    a = replay.post_process(y.astype(np.float32))
    live = np.ones(80, bool)
    live[40:46] = False
    assert np.array_equal(a[live], log.action[live])


def test_history_breaks_detect_drops_and_corruption():
    from go2_onnx_controller_amd import replay
    log = replay.read_log(BAG)
    keep = np.ones(80, bool)
    keep[30] = False  # a dropped message
    dropped = replay.ObservationActionLog(log.t_ns[keep], log.observation[keep], log.action[keep])
    assert replay.history_breaks(dropped).tolist() == [30]
    bad = replay.ObservationActionLog(log.t_ns, log.observation.copy(), log.action.copy())
    bad.action[50, 3] += 1e-3  # logged action disagrees with the next tick's history
    assert replay.history_breaks(bad).tolist() == [51]


def test_bag_and_npz_round_trip(tmp_path):
    from go2_onnx_controller_amd import replay
    log = replay.read_log(BAG)
    out = replay.write_bag(str(tmp_path / "copy"), log)
    back = replay.read_log(out)
    assert np.array_equal(back.t_ns, log.t_ns)
    assert np.array_equal(back.observation, log.observation) and np.array_equal(back.action, log.action)
    db = [f for f in os.listdir(out) if f.endswith(".db3")][0]
    assert np.array_equal(replay.read_log(os.path.join(out, db)).action, log.action)
    npz = str(tmp_path / "log.npz")
    np.savez(npz, observation=log.observation, action=log.action)
    z = replay.read_log(npz)
    assert np.array_equal(z.observation, log.observation) and z.t_ns.tolist() == list(range(80))
