#!/usr/bin/env python3
"""Writes tests/golden/replay_bag/ — a rosbag2 (sqlite3) recording of
/observation_action for a synthetic 80-tick closed-loop run of the reference
controller's tick (oracle/controller_ref.py: observation assembly, shipped
policy in fp64, clamp / stop-button post-processing), one robot at 50 Hz.

The reference ships no recorded robot data; this log has
the exact message layout `ros2 bag record /observation_action` produces, so the
replay harness (go2_onnx_controller_amd/replay.py) is exercised on the format
real logs come in. Regenerate: python tests/golden/make_replay_log.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from go2_onnx_controller_amd import replay  # noqa: E402
from oracle import controller_ref as cr, mlp_ref  # noqa: E402


def main():
    rng = np.random.default_rng(50)
    ref = mlp_ref.MlpRef.from_onnx(os.path.join(HERE, "model.onnx"))
    T = 80
    obs = np.zeros((1, 98), np.float32)
    act = np.zeros((1, 12), np.float32)
    log_o, log_a, log_t = [], [], []
    t0 = 1_700_000_000_000_000_000
    for t in range(T):
        ph = 2 * np.pi * t / 25
        st = np.zeros((1, 36), np.float32)
        q = np.array([1.0, 0.03 * np.sin(ph), 0.02 * np.cos(ph), 0.01 * t / T])
        st[0, 0:4] = q / np.linalg.norm(q)
        st[0, 4:7] = rng.normal(0, 0.3, 3)
        st[0, 7:19] = cr.Q0 + 0.15 * np.sin(ph + np.arange(12))
        st[0, 19:31] = 0.15 * 2 * np.pi / 25 * 50 * np.cos(ph + np.arange(12))
        st[0, 31:35] = [25 + 20 * np.sin(ph + k * np.pi / 2) for k in range(4)]
        joy = np.array([[1.0, 0.4 * np.sin(ph / 3), 0.6, 0.2, 1.0 if 40 <= t < 46 else 0.0]], np.float32)
        if t < 5:
            joy[0, 0] = 0.0  # no joystick axes yet: the command stays at zero
        obs, act, *_ = cr.tick(lambda x: ref.f64(x), st, joy, obs, act, 2)
        log_o.append(obs[0].copy())
        log_a.append(act[0].copy())
        log_t.append(t0 + t * 20_000_000 + int(rng.integers(0, 200_000)))
    log = replay.ObservationActionLog(np.array(log_t, np.int64), np.array(log_o), np.array(log_a))
    replay.write_bag(os.path.join(HERE, "replay_bag"), log)
    print("wrote", os.path.join(HERE, "replay_bag"), len(log_t), "ticks")


if __name__ == "__main__":
    main()
